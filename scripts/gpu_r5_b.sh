#!/bin/bash
# Background-qualities loader: its tests, then the bench (compact line +
# detail) and the per-phase clocks of the solid-set dedup count.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5b
mkdir -p $O
PT="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
echo "== tests" && timeout -k 10 600 $PT tests/test_gpu_load.py tests/test_gpu_precorrect.py tests/test_gpu_fused.py tests/test_gpu_readset.py > $O/tests.log 2>&1 && tail -2 $O/tests.log \
 && echo "== bench" && timeout -k 10 600 python3 bench.py --steps 10 --warmup 3 --detail-json $O/bench_detail.json > $O/bench.json 2> $O/bench.err && cat $O/bench.json \
 && echo "== sk_prof" && APG_SK_PROF=1 timeout -k 10 300 python3 scripts/diag/sk_prof.py > $O/sk_prof.log 2>&1; grep "sk_prof\]" $O/sk_prof.log | tail -4
