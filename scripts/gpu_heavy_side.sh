#!/bin/bash
# Heavy buckets' overflow path beside the bucket pass: parity tests, then
# the repeats line A/B (APG_SK_HEAVY_SIDE=0 / default).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5heavy
mkdir -p $O
timeout -k 10 700 python -u -m pytest tests/test_gpu_repeats.py tests/test_gpu_kmer.py tests/test_gpu_precorrect.py tests/test_gpu_fused.py tests/test_gpu_palindromes.py tests/test_distributed.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -n 1 $O/tests.log
BA_OVERRIDE="--steps 2 --warmup 1 --no-cpu-baseline --c3-jump-pairs 0 --no-file-to-graph --align-pairs 0 --jump-pairs 0 --no-placement --repeat-steps 2" A="APG_SK_HEAVY_SIDE=0" B="APG_SK_HEAVY_SIDE=1" VARIANTS="A B A B" bash scripts/gpu_ab.sh > $O/ab.txt 2>&1 || { tail -20 $O/ab.txt; exit 1; }
grep "^==\|^value\|^repeats\|rep sk_bucket\|rep fill\|  sk_bucket_solid" $O/ab.txt
