#!/bin/bash
# SQ issue / wait counters of k_fill on the repeat-rich genome
# (scripts/diag/fill_rep.py), one rocprofv3 pass per case.
set -o pipefail
R="$GRAFT_REPO_ROOT"
O="$R/gpurun_out/${TAG:-fillpmc}"
cd /tmp && export TMPDIR=/tmp
mkdir -p "$O"
for c in ${CASES:-x0 pass1}; do
  FILL_CASES=$c timeout -k 10 ${T_PMC:-300} rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
      SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE \
      --output-format csv -d "$O/$c" -o p -- python3 "$R/scripts/diag/fill_rep.py" > "$O/$c.out" 2> "$O/$c.err" \
   && python3 "$R/scripts/pmc_sq_summary.py" "$O/$c" > "$O/$c.txt" && echo "== $c" && cat "$O/$c.out" "$O/$c.txt" || exit $?
done
