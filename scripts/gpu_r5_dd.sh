#!/bin/bash
# k_sk_bucket_dd variants (APG_DD_VAR), one process each, same box.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5dd
mkdir -p $O
for v in ${VARS:-0 1 2 4 8 6 14 15 0}; do
  APG_DD_VAR=$v timeout -k 10 200 python3 scripts/diag/dd_ab.py 5 >> $O/ab.log 2>&1 || { echo "variant $v failed"; tail -5 $O/ab.log; exit 1; }
done
grep DDVAR $O/ab.log | cut -c1-60
