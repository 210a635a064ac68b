#!/bin/bash
# SQ instruction counters of the bucket kernels (dedup and per-instance) on
# the C2 reads (scripts/diag/sk_prof.py), one rocprofv3 --pmc pass each.
set -o pipefail
R="$GRAFT_REPO_ROOT"
mkdir -p "$R/gpurun_out"
cd /tmp && export TMPDIR=/tmp
C="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_WAVES"
timeout -k 10 200 rocprofv3 --pmc $C --output-format csv -d "$R/gpurun_out/pmc_sk_dd" -o p -- python3 "$R/scripts/diag/sk_prof.py" > "$R/gpurun_out/pmc_sk_dd.out" 2>&1 \
 && APG_SK_DEDUP=none timeout -k 10 200 rocprofv3 --pmc $C --output-format csv -d "$R/gpurun_out/pmc_sk_old" -o p -- python3 "$R/scripts/diag/sk_prof.py" > "$R/gpurun_out/pmc_sk_old.out" 2>&1 \
 && python3 "$R/scripts/pmc_sq_summary.py" "$R/gpurun_out/pmc_sk_dd" && python3 "$R/scripts/pmc_sq_summary.py" "$R/gpurun_out/pmc_sk_old"
