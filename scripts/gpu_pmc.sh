#!/bin/bash
# PMC passes (one counter group per rocprofv3 run, --kernel-trace-free) over a
# short bench run.  Output CSVs land in gpurun_out/pmc_<group>/.
set -o pipefail
R="$GRAFT_REPO_ROOT"
cd /tmp && export TMPDIR=/tmp
# main step only: every timed kernel launches once per run, so a per-launch mean is one size
ARGS="--steps 1 --warmup 0 --no-cpu-baseline --c3-jump-pairs 0 --no-file-to-graph --align-pairs 0 --jump-pairs 0 --no-placement --repeat-steps 0 ${BENCH_ARGS:-}"
run() {
  local tag="$1"; shift
  echo "== pmc $tag: $*"
  timeout -k 10 300 rocprofv3 --pmc "$@" --output-format csv -d "$R/gpurun_out/pmc_$tag" -o p -- python3 "$R/bench.py" $ARGS \
    > "$R/gpurun_out/pmc_$tag.out" 2> "$R/gpurun_out/pmc_$tag.err"
}
run fetch FETCH_SIZE \
 && run write WRITE_SIZE \
 && run tcc TCC_HIT_sum TCC_MISS_sum \
 && run sqwait SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
 && run lds SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAIT_INST_LDS \
 && echo "== pmc done"
