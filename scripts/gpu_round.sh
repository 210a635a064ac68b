#!/bin/bash
# One GPU session: parity tests -> smoke -> bench -> rocprofv3 kernel stats.
# Every GPU step has its own time limit; steps are chained with && so the
# first failure (fault, abort, timeout) ends the call.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
OUT=gpurun_out
echo "== pytest -m gpu" && timeout -k 10 ${T_TEST:-900} python -m pytest tests -m gpu -x -q ${PYTEST_ARGS:-} > $OUT/pytest_gpu.log 2>&1 \
 && tail -3 $OUT/pytest_gpu.log \
 && echo "== smoke" && timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 \
 && tail -2 $OUT/smoke.log \
 && echo "== bench" && timeout -k 10 600 python bench.py --steps ${STEPS:-5} --warmup 2 > $OUT/bench.json 2> $OUT/bench.err \
 && cat $OUT/bench.json \
 && echo "== rocprof" && cd /tmp && export TMPDIR=/tmp \
 && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/$OUT/prof" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 3 --warmup 1 --no-cpu-baseline > "$GRAFT_REPO_ROOT/$OUT/bench_prof.json" 2> "$GRAFT_REPO_ROOT/$OUT/bench_prof.err" \
 && echo "== done"
