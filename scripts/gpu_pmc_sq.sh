#!/bin/bash
# SQ counters (issue / wait / LDS) per kernel over a 1-step bench.
#   BENCH_ARGS="--spectrum-only" bash scripts/gpu_pmc_sq.sh
set -o pipefail
R="$GRAFT_REPO_ROOT"
cd /tmp && export TMPDIR=/tmp
mkdir -p "$R/gpurun_out"
timeout -k 10 500 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE \
    --output-format csv -d "$R/gpurun_out/pmc_sq" -o p -- python3 "$R/bench.py" --steps 1 --warmup 0 --no-cpu-baseline ${BENCH_ARGS} \
    > "$R/gpurun_out/pmc_sq.out" 2> "$R/gpurun_out/pmc_sq.err" \
 && python3 "$R/scripts/pmc_sq_summary.py" "$R/gpurun_out/pmc_sq"
