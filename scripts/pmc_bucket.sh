#!/bin/bash
# SQ counter passes over the spectrum-only bench (k_sk_bucket<false,SK16>
# dominates it), plus the list of gfx950 counters.
set -o pipefail
R="$GRAFT_REPO_ROOT"
mkdir -p "$R/gpurun_out"
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 -L > "$R/gpurun_out/counters.txt" 2>&1
ARGS="--steps 1 --warmup 0 --no-cpu-baseline ${BENCH_ARGS:---spectrum-only}"
pass() {
  local tag=$1; shift
  timeout -k 10 300 rocprofv3 --pmc "$@" --output-format csv -d "$R/gpurun_out/pmc_$tag" -o p -- python3 "$R/bench.py" $ARGS \
    > "$R/gpurun_out/pmc_$tag.out" 2> "$R/gpurun_out/pmc_$tag.err"
}
pass a SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA \
 && pass b SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_BUSY_CYCLES SQ_WAVES \
 && python3 "$R/scripts/pmc_dump.py" "$R/gpurun_out/pmc_a" "$R/gpurun_out/pmc_b"
