#!/bin/bash
# Round-5 checkpoint, part 1: the whole -m gpu suite, smoke, the driver's
# bench command.  Each GPU step has its own limit; && ends at the first failure.
set -o pipefail
R="$GRAFT_REPO_ROOT"
cd "$R"
O=gpurun_out/r5final
mkdir -p $O
PT="python -u -m pytest -x -q --timeout 600 --timeout-method thread"
echo "== pytest -m gpu" && timeout -k 10 900 $PT tests -m gpu > $O/pytest_gpu.log 2>&1 && tail -n 2 $O/pytest_gpu.log \
 && echo "== smoke" && timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 \
 && echo "== bench" && timeout -k 10 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 --detail-json $O/bench_detail.json > $O/bench.json 2> $O/bench.err \
 && cat $O/bench.json && wc -c $O/bench.json && echo "== done"
