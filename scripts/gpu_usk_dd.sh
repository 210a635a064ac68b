#!/bin/bash
# Bucket-wide K=96 record dedup: unipath parity tests, then the bench step
# (with the dedup counters) for usk_bucket's time.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5uskdd
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_unipath.py tests/test_gpu_repeats.py tests/test_gpu_readset.py tests/test_gpu_locs.py tests/test_gpu_ucov.py "tests/test_gpu_configs.py::test_c1_ecoli_whole_chain_matches_oracle" -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -n 1 $O/tests.log
A="" B="APG_USK_DEDUP_STATS=1" VARIANTS="A B A" bash scripts/gpu_ab.sh > $O/ab.txt 2>&1 || { tail -20 $O/ab.txt; exit 1; }
grep "^==\|^value\|usk_\|u_walk" $O/ab.txt
grep usk_dedup gpurun_out/ab_B.err | tail -2
