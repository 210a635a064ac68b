#!/bin/bash
# SQ instruction / wait counters of the K = 96 walk kernels (k_usk_count,
# k_usk_scatter) and their bucket kernel over the bench main step: is the
# walk issue-bound (ACTIVE_INST_VALU close to WAVE_CYCLES / waves per SIMD) or
# latency-bound (WAIT_ANY dominant)?  One rocprofv3 --pmc pass per group.
set -o pipefail
R="$GRAFT_REPO_ROOT"
mkdir -p "$R/gpurun_out"
cd /tmp && export TMPDIR=/tmp
ARGS="--steps 1 --warmup 0 --no-cpu-baseline --c3-jump-pairs 0 --no-file-to-graph --align-pairs 0 --jump-pairs 0 --no-placement --repeat-steps 0"
C1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVES"
C2="SQ_INSTS_SALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_SCA"
timeout -k 10 300 rocprofv3 --pmc $C1 --kernel-include-regex "${KRE:-usk}" --output-format csv -d "$R/gpurun_out/pmc_usk1" -o p -- python3 "$R/bench.py" $ARGS > "$R/gpurun_out/pmc_usk1.out" 2>&1 \
 && timeout -k 10 300 rocprofv3 --pmc $C2 --kernel-include-regex "${KRE:-usk}" --output-format csv -d "$R/gpurun_out/pmc_usk2" -o p -- python3 "$R/bench.py" $ARGS > "$R/gpurun_out/pmc_usk2.out" 2>&1 \
 && python3 "$R/scripts/pmc_sq_summary.py" "$R/gpurun_out/pmc_usk1" && python3 "$R/scripts/pmc_sq_summary.py" "$R/gpurun_out/pmc_usk2"
