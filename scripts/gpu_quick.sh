#!/bin/bash
# Quick GPU iteration: selected parity tests, then one bench run.
#   PYTEST_SEL="tests/test_gpu_unipath.py" BENCH_ARGS="--steps 3 --warmup 1" bash scripts/gpu_quick.sh
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 ${T_TEST:-600} python -m pytest ${PYTEST_SEL:-tests} -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1
rc=$?
tail -25 gpurun_out/pytest_gpu.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 ${T_BENCH:-600} python bench.py ${BENCH_ARGS:---steps 3 --warmup 1} > gpurun_out/bench.json 2> gpurun_out/bench.err
rc=$?
tail -3 gpurun_out/bench.err
[ $rc -ne 0 ] && exit $rc
python - <<'PY'
import json
b = json.load(open("gpurun_out/bench.json"))
print("value", round(b["value"] / 1e6, 2), "M reads/s  ms/step", round(b["ms_per_step"], 1), "hbm_gb", b["config"].get("hbm_used_gb"))
print("roofline", b["roofline"]["kernel"], round(b["roofline"]["frac"], 3), "checks", all(b["checks"].values()))
ks = sorted(b["kernels"].items(), key=lambda kv: -kv[1]["ms_per_launch"] * kv[1]["launches"])
for k, v in ks[:18]:
    print(f"  {k:24s} {v['ms_per_launch'] * v['launches'] / b['steps']:9.2f} ms/step  {v['GBps']:8.1f} GB/s")
PY
