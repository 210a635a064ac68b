#!/bin/bash
# SQ issue / wait counters per kernel over a 1-step bench (two passes, each
# within the per-block counter limits), summarised per kernel.
set -o pipefail
R="$GRAFT_REPO_ROOT"
O="$R/gpurun_out/${TAG:-r4pmc}"
cd /tmp && export TMPDIR=/tmp
mkdir -p "$O"
A="--steps 1 --warmup 1 --no-cpu-baseline --c3-jump-pairs 0 --no-file-to-graph --align-pairs 0 --jump-pairs 0 --no-placement --repeat-steps ${REP:-0}"
pass() {
  local name=$1; shift
  timeout -k 10 ${T_PMC:-240} rocprofv3 --pmc "$@" --output-format csv -d "$O/$name" -o p -- python3 "$R/bench.py" $A \
    > "$O/$name.out" 2> "$O/$name.err" \
   && python3 "$R/scripts/pmc_sq_summary.py" "$O/$name" > "$O/$name.txt" && echo "== $name" && cat "$O/$name.txt"
}
pass sqa SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE \
 && pass sqb SQ_WAVES SQ_INSTS_LDS SQ_WAIT_ANY SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_SCA SQ_WAIT_INST_LDS
