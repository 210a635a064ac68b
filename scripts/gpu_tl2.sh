#!/bin/bash
# Steady-state kernel + copy timeline of the bench step (2 warmup steps: the
# grow-only workspaces have their final sizes), per stream and idle gaps.
set -o pipefail
R="$GRAFT_REPO_ROOT"
O=${OUT:-tl2}
cd /tmp && export TMPDIR=/tmp
mkdir -p "$R/gpurun_out"
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d "$R/gpurun_out/$O" -o t -- python3 "$R/bench.py" \
    --steps 1 --warmup 2 --no-cpu-baseline --c3-jump-pairs 0 --no-file-to-graph --align-pairs 0 --jump-pairs 0 --no-placement --repeat-steps 0 ${BENCH_ARGS:-} \
    > "$R/gpurun_out/$O.out" 2> "$R/gpurun_out/$O.err" \
 && python3 "$R/scripts/timeline_gaps.py" "$R/gpurun_out/$O" > "$R/gpurun_out/$O.gaps.txt" \
 && python3 "$R/scripts/timeline_streams.py" "$R/gpurun_out/$O" > "$R/gpurun_out/$O.streams.txt" \
 && head -n 60 "$R/gpurun_out/$O.streams.txt"
