#!/bin/bash
# A/B on one box: selected parity tests, then the bench step with env A and
# env B (e.g. A="APG_FILL_MEMO=0" B=""; more variants: VARIANTS="A B C D").
# Kernel table of each in the log.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
BA="${BA_OVERRIDE:---steps ${STEPS:-3} --warmup 1 --no-cpu-baseline --c3-jump-pairs 0 --no-file-to-graph --align-pairs 0 --jump-pairs 0 --no-placement --repeat-steps 0}"
if [ -n "${PYTEST_SEL:-}" ]; then
  env ${PYTEST_ENV:-} timeout -k 10 ${T_TEST:-400} python -u -m pytest ${PYTEST_SEL} -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/ab_pytest.log 2>&1 || { tail -30 gpurun_out/ab_pytest.log; exit 1; }
  tail -2 gpurun_out/ab_pytest.log
fi
for V in ${VARIANTS:-A B}; do
  ENVV="${!V}"
  env $ENVV timeout -k 10 ${T_BENCH:-400} python bench.py $BA --detail-json gpurun_out/ab_$V.detail.json > gpurun_out/ab_$V.json 2> gpurun_out/ab_$V.err || { tail -5 gpurun_out/ab_$V.err; exit 1; }
  echo "== $V ($ENVV)"
  python - gpurun_out/ab_$V.detail.json <<'PY'
import json, sys
b = json.load(open(sys.argv[1]))
print("value", round(b["value"] / 1e6, 2), "M reads/s  ms/step", round(b["ms_per_step"], 1), "checks", all(b["checks"].values()))
print("roofline", b["roofline"]["kernel"], round(b["roofline"]["frac"], 3))
ks = sorted(b["kernels"].items(), key=lambda kv: -kv[1]["ms_per_launch"] * kv[1]["launches"])
for k, v in ks[:12]:
    print(f"  {k:24s} {v['ms_per_launch'] * v['launches'] / b['steps']:9.2f} ms/step  {v['GBps']:8.1f} GB/s")
r = b.get("repeats")
if r:
    print("repeats ms/step", round(r["ms_per_step"], 1), "x main", round(r["ms_per_step"] / b["ms_per_step"], 3),
          "checks", all(r["checks"].values()))
    for k, v in list(r["kernels_ms"].items())[:10]:
        print(f"  rep {k:20s} {v:9.2f} ms/step")
PY
done
