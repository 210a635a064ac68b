#!/bin/bash
# Round 6: selected GPU tests (TESTS), then bench-step variants on the same
# box.  Each variant V names a variable holding "ENV...|EXTRA_BENCH_ARGS";
# kernel table of each in the log (scripts/ab_summary.py).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
if [ -n "${TESTS:-}" ]; then
  timeout -k 10 ${T_TEST:-700} python -u -m pytest ${TESTS} -m gpu ${XFLAG--x} -v -s --timeout ${T_CASE:-400} \
    --timeout-method thread > gpurun_out/${LOG:-r6_ab}_pytest.log 2>&1
  rc=$?
  tail -4 gpurun_out/${LOG:-r6_ab}_pytest.log
  # ordinary test failures (rc 1) go on to the bench; a timeout, fault or
  # abort ends the call here
  if [ $rc -ne 0 ]; then
    # a timeout, a GPU fault or an abort: nothing more on the GPU in this call
    if [ $rc -ne 1 ] || grep -q -E "Timeout|illegal memory access|Memory access fault|hipErrorLaunchFailure" gpurun_out/${LOG:-r6_ab}_pytest.log; then exit $rc; fi
    FAILED=1
  fi
fi
BA="--steps ${STEPS:-3} --warmup 1 --no-cpu-baseline --c3-jump-pairs 0 --no-file-to-graph --align-pairs 0 --jump-pairs 0 --no-placement --repeat-steps ${REPS:-0}"
for V in ${VARIANTS:-}; do
  SPEC="${!V}"
  ENVV="${SPEC%%|*}"
  ARGS=""
  [[ "$SPEC" == *"|"* ]] && ARGS="${SPEC#*|}"
  env $ENVV timeout -k 10 ${T_BENCH:-300} python bench.py $BA $ARGS --detail-json gpurun_out/${LOG:-r6_ab}_$V.detail.json \
    > gpurun_out/${LOG:-r6_ab}_$V.json 2> gpurun_out/${LOG:-r6_ab}_$V.err || { tail -5 gpurun_out/${LOG:-r6_ab}_$V.err; exit 1; }
  echo "== $V ($SPEC)"
  python scripts/ab_summary.py gpurun_out/${LOG:-r6_ab}_$V.detail.json
done
exit ${FAILED:-0}
