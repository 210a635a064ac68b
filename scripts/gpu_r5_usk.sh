#!/bin/bash
# K=96 node bucket size A/B (APG_USK_BUCKET_KMERS), unipath parity at the
# larger sizes first.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5usk
mkdir -p $O
for n in 4096 8192; do
  APG_USK_BUCKET_KMERS=$n timeout -k 10 300 python -u -m pytest tests/test_gpu_unipath.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/unipath_$n.log 2>&1 || { tail -30 $O/unipath_$n.log; exit 1; }
  echo "unipath tests at $n: $(tail -n 1 $O/unipath_$n.log)"
done
A="APG_USK_BUCKET_KMERS=2048" B="APG_USK_BUCKET_KMERS=4096" C="APG_USK_BUCKET_KMERS=8192" VARIANTS="A B C A B C" bash scripts/gpu_ab.sh > $O/ab.txt 2>&1 || { tail -20 $O/ab.txt; exit 1; }
grep "^==\|^value\|usk_\|u_" $O/ab.txt
