#!/bin/bash
# Round-6 checkpoint on one GPU box (outputs under gpurun_out/r6final/; copy
# what is judged into profiles/r06/perf_final and profiles/current/pmc).
#   PHASE=tests  the -m gpu suite (IGNORE_BIG=1: without the full-size C2/C3
#                and C4 files, run in their own call) + smoke
#   PHASE=perf   PMC traffic (FETCH_SIZE, WRITE_SIZE) and LDS passes of the
#                main step -> profiles/current/pmc on the box, so the bench's
#                traffic_source / lds_source name the tracked files; the
#                driver's default bench command; rocprofv3 kernel-trace stats
#                of the main step; a kernel + copy timeline of one step
# Every GPU step has its own limit and the steps are chained with &&: the
# first failure ends the call.
set -o pipefail
R="$GRAFT_REPO_ROOT"
cd "$R"
O=gpurun_out/r6final
mkdir -p $O/pmc
A="--steps 1 --warmup 0 --no-cpu-baseline --c3-jump-pairs 0 --no-file-to-graph --align-pairs 0 --jump-pairs 0 --no-placement --repeat-steps 0"
tests() {
  IG=""
  [ "${IGNORE_BIG:-0}" = 1 ] && IG="--ignore=tests/test_gpu_configs.py --ignore=tests/test_gpu_c4.py"
  echo "== pytest -m gpu $IG" \
   && timeout -k 10 ${T_TEST:-1000} python -u -m pytest tests -m gpu $IG -x -q --timeout 600 --timeout-method thread \
        > $O/pytest_gpu.log 2>&1 \
   && tail -n 2 $O/pytest_gpu.log \
   && echo "== smoke" && timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 \
   && echo "== tests done"
}
perf() {
  echo "== pmc" && (cd /tmp && export TMPDIR=/tmp \
     && timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$R/$O/pmc_fetch" -o p -- python3 "$R/bench.py" $A > "$R/$O/pmc_fetch.out" 2>&1 \
     && timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$R/$O/pmc_write" -o p -- python3 "$R/bench.py" $A > "$R/$O/pmc_write.out" 2>&1 \
     && timeout -k 10 300 rocprofv3 --pmc SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU GRBM_GUI_ACTIVE \
          --output-format csv -d "$R/$O/pmc_lds" -o p -- python3 "$R/bench.py" $A > "$R/$O/pmc_lds.out" 2>&1) \
   && cp $(find $O/pmc_fetch -name "*counter_collection.csv" | head -n 1) $O/pmc/fetch.csv \
   && cp $(find $O/pmc_write -name "*counter_collection.csv" | head -n 1) $O/pmc/write.csv \
   && python3 scripts/pmc_traffic.py $O/pmc > $O/pmc/traffic.txt \
   && python3 scripts/pmc_lds.py $O/pmc_lds > $O/pmc/lds.txt \
   && cp $O/pmc_lds/lds.json $O/pmc/lds.json \
   && cp $O/pmc/traffic.json $O/pmc/traffic.txt $O/pmc/lds.json profiles/current/pmc/ \
   && echo "== bench (driver command)" && timeout -k 10 900 python bench.py --detail-json $O/bench_detail.json > $O/bench.json 2> $O/bench.err \
   && cat $O/bench.json \
   && echo "== rocprof" && (cd /tmp && export TMPDIR=/tmp \
     && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$R/$O/prof" -o run --output-format csv -- python3 "$R/bench.py" --steps 3 --warmup 1 --no-cpu-baseline --c3-jump-pairs 0 --no-file-to-graph --align-pairs 0 --jump-pairs 0 --no-placement --repeat-steps 0 > "$R/$O/bench_prof.json" 2> "$R/$O/bench_prof.err" \
     && timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d "$R/$O/tl" -o t -- python3 "$R/bench.py" --steps 1 --warmup 1 --no-cpu-baseline --c3-jump-pairs 0 --no-file-to-graph --align-pairs 0 --jump-pairs 0 --no-placement --repeat-steps 0 > "$R/$O/tl.out" 2> "$R/$O/tl.err") \
   && python3 scripts/timeline_gaps.py $O/tl > $O/timeline_gaps.txt \
   && python3 scripts/timeline_streams.py $O/tl > $O/timeline_streams.txt \
   && echo "== perf done"
}
case "${PHASE:-all}" in
  tests) tests ;;
  perf) perf ;;
  *) tests && perf ;;
esac
