#!/bin/bash
# VALU issue vs LDS wait per kernel over a 1-step bench (two --pmc passes:
# SQ counters, then GRBM_GUI_ACTIVE for the kernel's busy cycles).
#   BENCH_ARGS="..." bash scripts/gpu_pmc_valu.sh
set -o pipefail
R="$GRAFT_REPO_ROOT"
cd /tmp && export TMPDIR=/tmp
mkdir -p "$R/gpurun_out"
BA="--steps 1 --warmup 0 --no-cpu-baseline --c3-jump-pairs 0 --no-file-to-graph --align-pairs 0 --jump-pairs 0 --no-placement --repeat-steps 0 ${BENCH_ARGS}"
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_WAIT_ANY \
    --output-format csv -d "$R/gpurun_out/pmc_valu" -o p -- python3 "$R/bench.py" $BA \
    > "$R/gpurun_out/pmc_valu.out" 2> "$R/gpurun_out/pmc_valu.err" \
 && timeout -k 10 300 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVES \
    --output-format csv -d "$R/gpurun_out/pmc_gui" -o p -- python3 "$R/bench.py" $BA \
    > "$R/gpurun_out/pmc_gui.out" 2> "$R/gpurun_out/pmc_gui.err" \
 && python3 "$R/scripts/pmc_valu.py" "$R/gpurun_out/pmc_valu" "$R/gpurun_out/pmc_gui"
