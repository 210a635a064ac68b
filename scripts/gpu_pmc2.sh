#!/bin/bash
# HBM-traffic PMC passes for the roofline "traffic" field: calibrate
# FETCH_SIZE on a known random 64-byte-line pattern (randread), then one
# FETCH_SIZE and one WRITE_SIZE pass over a 1-step bench (separate runs,
# no trace domains besides kernel dispatch).
set -o pipefail
R="$GRAFT_REPO_ROOT"
cd /tmp && export TMPDIR=/tmp
mkdir -p "$R/gpurun_out"
echo "== calibrate" \
 && timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$R/gpurun_out/pmc_cal" -o p -- "$R/tools/microbench/randread" \
      > "$R/gpurun_out/pmc_cal.out" 2> "$R/gpurun_out/pmc_cal.err" \
 && echo "== fetch" \
 && timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$R/gpurun_out/pmc_fetch" -o p -- python3 "$R/bench.py" --steps 1 --warmup 0 --no-cpu-baseline \
      > "$R/gpurun_out/pmc_fetch.out" 2> "$R/gpurun_out/pmc_fetch.err" \
 && echo "== write" \
 && timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$R/gpurun_out/pmc_write" -o p -- python3 "$R/bench.py" --steps 1 --warmup 0 --no-cpu-baseline \
      > "$R/gpurun_out/pmc_write.out" 2> "$R/gpurun_out/pmc_write.err" \
 && echo "== pmc done"
