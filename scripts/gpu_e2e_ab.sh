#!/bin/bash
# End-to-end (file -> graph) A/B: bench's file_to_graph line with env A / B.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5e2e
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_load.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/load_tests.log 2>&1 || { tail -20 $O/load_tests.log; exit 1; }
tail -n 1 $O/load_tests.log
env APG_LOAD_EARLY=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_load.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/load_tests_early.log 2>&1 || { tail -20 $O/load_tests_early.log; exit 1; }
tail -n 1 $O/load_tests_early.log
for V in ${VARIANTS:-A B A B}; do
  ENVV="${!V}"
  env $ENVV timeout -k 10 400 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --c3-jump-pairs 0 --align-pairs 0 --jump-pairs 0 --no-placement --repeat-steps 0 --detail-json $O/$V.detail.json > $O/$V.json 2> $O/$V.err || { tail -5 $O/$V.err; exit 1; }
  python3 - $O/$V.detail.json "$V ($ENVV)" <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))["file_to_graph"]
print(sys.argv[2], {k: round(v, 1) for k, v in d.items() if isinstance(v, float)})
PY
done
