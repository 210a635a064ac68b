#!/bin/bash
# Round checkpoint on one GPU box: parity tests -> smoke -> PMC traffic passes
# (FETCH_SIZE, WRITE_SIZE; scripts/pmc_traffic.py) -> bench with that traffic
# -> rocprofv3 kernel-trace stats of the bench's main step alone (per-kernel
# averages comparable with the bench's HIP-event times).  Each GPU step has
# its own time limit; steps are chained with && so the first failure ends the
# call.  Outputs under gpurun_out/ck/ (copy what is judged into profiles/).
set -o pipefail
R="$GRAFT_REPO_ROOT"
cd "$R"
O=gpurun_out/ck
mkdir -p $O/pmc
A="--steps 1 --warmup 0 --no-cpu-baseline --c3-jump-pairs 0 --no-file-to-graph --align-pairs 0 --jump-pairs 0 --no-placement --repeat-steps 0"
# PHASE=tests: parity tests + smoke only; PHASE=perf: PMC + bench + rocprof only
# (one gpurun call each when the whole does not fit one call's limit)
T_ON=1; P_ON=1
[ "${PHASE:-all}" = tests ] && P_ON=0
[ "${PHASE:-all}" = perf ] && T_ON=0
tests() {
echo "== pytest -m gpu" && timeout -k 10 ${T_TEST:-900} python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 \
 && tail -2 $O/pytest_gpu.log \
 && echo "== smoke" && timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 \

}
perf() {
echo "== pmc" && (cd /tmp && export TMPDIR=/tmp \
   && timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$R/$O/pmc_fetch" -o p -- python3 "$R/bench.py" $A > "$R/$O/pmc_fetch.out" 2>&1 \
   && timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$R/$O/pmc_write" -o p -- python3 "$R/bench.py" $A > "$R/$O/pmc_write.out" 2>&1) \
 && cp $(find $O/pmc_fetch -name "*counter_collection.csv" | head -1) $O/pmc/fetch.csv \
 && cp $(find $O/pmc_write -name "*counter_collection.csv" | head -1) $O/pmc/write.csv \
 && python3 scripts/pmc_traffic.py $O/pmc > $O/pmc/traffic.txt \
 && echo "== bench" && timeout -k 10 600 python bench.py --steps ${STEPS:-5} --warmup 2 --traffic-json $O/pmc/traffic.json > $O/bench.json 2> $O/bench.err \
 && cat $O/bench.json \
 && echo "== rocprof" && (cd /tmp && export TMPDIR=/tmp \
   && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$R/$O/prof" -o run --output-format csv -- python3 "$R/bench.py" --steps 3 --warmup 1 --no-cpu-baseline --c3-jump-pairs 0 --no-file-to-graph --align-pairs 0 --jump-pairs 0 --no-placement --repeat-steps 0 --traffic-json "$R/$O/pmc/traffic.json" > "$R/$O/bench_prof.json" 2> "$R/$O/bench_prof.err") \
 && echo "== done"
}
{ [ $T_ON = 0 ] || tests; } && { [ $P_ON = 0 ] || perf; }
