#!/bin/bash
# FillFragments determinism: repeated one-pass calls (tree library, and the
# SGPR-spills-to-memory build) against the oracle at max_steps 300 and 1024.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5split
mkdir -p $O
for v in "" mem; do
  for st in 300 1024; do
    echo "== lib '$v' max_steps $st"
    APG_LIB_VARIANT=$v DET_STEPS=$st timeout -k 10 200 python -u scripts/diag/fill_det.py > $O/det_${v}_$st.txt 2>&1 || { tail -5 $O/det_${v}_$st.txt; exit 1; }
    cat $O/det_${v}_$st.txt
  done
done
