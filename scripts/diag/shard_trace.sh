#!/bin/bash
# Kernel trace of the sharded bench path at world size 1 (no launcher: the
# rendezvous env is set by hand) -> idle gaps of one step.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
export RANK=0 WORLD_SIZE=1 LOCAL_RANK=0 MASTER_ADDR=127.0.0.1 MASTER_PORT=29671
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/shtrace" -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --sharded ${EXTRA:-} --steps 3 --warmup 1 --no-cpu-baseline --c3-jump-pairs 0 --no-file-to-graph --align-pairs 0 --jump-pairs 0 --no-placement --repeat-steps 0 > "$GRAFT_REPO_ROOT/gpurun_out/shtrace.json" 2> "$GRAFT_REPO_ROOT/gpurun_out/shtrace.err" \
 && python3 "$GRAFT_REPO_ROOT/scripts/trace_gaps.py" "$GRAFT_REPO_ROOT/gpurun_out/shtrace/run_kernel_trace.csv"
