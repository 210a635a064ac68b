#!/bin/bash
# SQ issue counters per kernel over a 1-step bench (fill-oriented set).
set -o pipefail
R="$GRAFT_REPO_ROOT"
cd /tmp && export TMPDIR=/tmp
mkdir -p "$R/gpurun_out"
A="--steps 1 --warmup 0 --no-cpu-baseline --c3-jump-pairs 0 --no-file-to-graph --align-pairs 0 --jump-pairs 0 --no-placement --repeat-steps 0"
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD \
    --output-format csv -d "$R/gpurun_out/pmc_fill" -o p -- python3 "$R/bench.py" $A \
    > "$R/gpurun_out/pmc_fill.out" 2> "$R/gpurun_out/pmc_fill.err" \
 && python3 "$R/scripts/pmc_sq_summary.py" "$R/gpurun_out/pmc_fill"
