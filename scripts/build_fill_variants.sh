#!/bin/bash
# Variant libraries differing only in fill.hip's compile flags (diagnostics):
# allpathslg_amd/libapg_<name>.so for each NAME=FLAGS argument.
set -e
cd "$(dirname "$0")/../allpathslg_amd/csrc"
make -s -j8
for spec in "$@"; do
  name="${spec%%=*}"; flags="${spec#*=}"
  d=../../build/var_$name
  mkdir -p $d
  cp ../../build/obj/*.o $d/
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -Wall -Wno-unused-result -munsafe-fp-atomics \
    -I../../include $flags -c fill.hip -o $d/fill.hip.o
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o ../libapg_$name.so $d/*.o -lpthread -ldl
  echo "built libapg_$name.so ($flags)"
done
