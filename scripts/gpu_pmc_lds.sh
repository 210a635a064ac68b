#!/bin/bash
# LDS roofline counters per kernel over a 1-step bench:
#   pass 1  SQ_LDS_IDX_ACTIVE (LDS-array busy cycles, per SE) SQ_LDS_BANK_CONFLICT
#           SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY
#           SQ_INSTS_VALU + GRBM_GUI_ACTIVE (kernel busy cycles)
# LDS utilisation = SQ_LDS_IDX_ACTIVE / (GRBM_GUI_ACTIVE x 256 CUs) — rocprofiler's own
# LdsUtil definition for gfx950 (counter_defs.yaml).  scripts/pmc_lds.py reduces it.
#   OUT=pmc_lds BENCH_ARGS="..." bash scripts/gpu_pmc_lds.sh
set -o pipefail
R="$GRAFT_REPO_ROOT"
O=${OUT:-pmc_lds}
cd /tmp && export TMPDIR=/tmp
mkdir -p "$R/gpurun_out"
timeout -k 10 ${T_PMC:-300} rocprofv3 --pmc SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU GRBM_GUI_ACTIVE \
    --output-format csv -d "$R/gpurun_out/$O" -o p -- python3 "$R/bench.py" --steps 1 --warmup 0 --no-cpu-baseline \
    --c3-jump-pairs 0 --no-file-to-graph --align-pairs 0 --jump-pairs 0 --no-placement --repeat-steps 0 ${BENCH_ARGS} \
    > "$R/gpurun_out/$O.out" 2> "$R/gpurun_out/$O.err" \
 && python3 "$R/scripts/pmc_lds.py" "$R/gpurun_out/$O" > "$R/gpurun_out/$O.txt" && cat "$R/gpurun_out/$O.txt"
