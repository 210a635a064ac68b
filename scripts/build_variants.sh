#!/bin/bash
# Variant libraries differing only in one source file's compile flags (A/B):
#   scripts/build_variants.sh <file.hip> NAME=FLAGS ...
# -> allpathslg_amd/libapg_<NAME>.so (load with APG_LIB_VARIANT=<NAME>).
set -e
src="$1"; shift
cd "$(dirname "$0")/../allpathslg_amd/csrc"
make -s -j8
for spec in "$@"; do
  name="${spec%%=*}"; flags="${spec#*=}"
  d=../../build/var_$name
  rm -rf $d && mkdir -p $d
  cp ../../build/obj/*.o $d/
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -Wall -Wno-unused-result -munsafe-fp-atomics \
    -I../../include $flags -c "$src" -o $d/"$src".o
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o ../libapg_$name.so $d/*.o -lpthread -ldl
  echo "built libapg_$name.so ($flags)"
done
