#!/bin/bash
# Round-5 GPU call: new parity tests first (fail fast), the whole -m gpu suite,
# smoke, then the driver's own bench command (compact line + detail file).
# Each GPU step has its own limit; && ends the call at the first failure.
set -o pipefail
R="$GRAFT_REPO_ROOT"
cd "$R"
O=gpurun_out/r5
mkdir -p $O
PT="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
echo "== new tests" && timeout -k 10 400 $PT tests/test_gpu_partition.py tests/test_gpu_palindromes.py \
   "tests/test_gpu_repeats.py::test_overflow_table_retry_unbounded" > $O/new_tests.log 2>&1 \
 && tail -2 $O/new_tests.log \
 && { [ "${FULL:-1}" = 0 ] || { echo "== pytest -m gpu" && timeout -k 10 900 $PT tests -m gpu > $O/pytest_gpu.log 2>&1 && tail -2 $O/pytest_gpu.log; }; } \
 && echo "== smoke" && timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 \
 && echo "== bench" && timeout -k 10 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 --detail-json $O/bench_detail.json > $O/bench.json 2> $O/bench.err \
 && cat $O/bench.json && wc -c $O/bench.json && echo "== done"
