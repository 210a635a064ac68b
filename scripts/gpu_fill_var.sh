#!/bin/bash
# FillFragments compile-time variants (scripts/build_fill_variants.sh) on the
# repeat-rich and iid genomes: fill ms per variant.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5fv
mkdir -p $O
for g in rep iid; do
  for v in "" ${VARS:-p50 p90 x2 r24 r44} ""; do
    if [ $g = iid ]; then export FILL_GENOME=iid; else unset FILL_GENOME; fi
    APG_LIB_VARIANT=$v FILL_CASES=base timeout -k 10 300 python -u scripts/diag/fill_rep.py > $O/${g}_$v.txt 2>&1 || { tail -5 $O/${g}_$v.txt; exit 1; }
    echo "$g variant '${v}': $(grep '^base' $O/${g}_$v.txt)"
  done
done
