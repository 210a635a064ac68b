#!/bin/bash
# Kernel + copy timeline of the bench step (warm): idle gaps on the GPU between
# consecutive operations, largest first (scripts/timeline_gaps.py).
set -o pipefail
R="$GRAFT_REPO_ROOT"
cd /tmp && export TMPDIR=/tmp
mkdir -p "$R/gpurun_out"
BA="--steps 1 --warmup 1 --no-cpu-baseline --c3-jump-pairs 0 --no-file-to-graph --align-pairs 0 --jump-pairs 0 --no-placement --repeat-steps 0 ${BENCH_ARGS}"
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d "$R/gpurun_out/tl" -o t -- python3 "$R/bench.py" $BA \
    > "$R/gpurun_out/tl.out" 2> "$R/gpurun_out/tl.err" \
 && python3 "$R/scripts/timeline_gaps.py" "$R/gpurun_out/tl"
