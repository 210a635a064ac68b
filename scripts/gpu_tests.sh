#!/bin/bash
# GPU tests on the box: TESTS (default: every -m gpu test) under one time
# limit, output under gpurun_out/ (pytest -v -s: each test and each rank's
# stage lines appear as they happen).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 ${T_TEST:-1100} python -u -m pytest ${TESTS:-tests} -m gpu -x -v -s --timeout ${T_CASE:-300} \
  --timeout-method thread ${PYTEST_ARGS:-} > gpurun_out/${LOG:-pytest_gpu}.log 2>&1
rc=$?
tail -5 gpurun_out/${LOG:-pytest_gpu}.log
exit $rc
