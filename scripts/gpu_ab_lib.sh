#!/bin/bash
# A/B of two builds on one box: A = allpathslg_amd/libapg_var.so, B = the
# tree's libapg.so; the bench step with each (kernel table in the log).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
BA="${BA_OVERRIDE:---steps ${STEPS:-3} --warmup 1 --no-cpu-baseline --c3-jump-pairs 0 --no-file-to-graph --align-pairs 0 --jump-pairs 0 --no-placement --repeat-steps 0}"
cp allpathslg_amd/libapg.so /tmp/libapg_B.so
for V in B A; do
  if [ $V = A ]; then cp allpathslg_amd/libapg_var.so allpathslg_amd/libapg.so; fi
  timeout -k 10 ${T_BENCH:-400} python bench.py $BA > gpurun_out/ab_$V.json 2> gpurun_out/ab_$V.err || { tail -5 gpurun_out/ab_$V.err; exit 1; }
  echo "== $V"
  python - gpurun_out/ab_$V.json <<'PY'
import json, sys
b = json.load(open(sys.argv[1]))
print("value", round(b["value"] / 1e6, 2), "M reads/s  ms/step", round(b["ms_per_step"], 1), "checks", all(b["checks"].values()))
ks = sorted(b["kernels"].items(), key=lambda kv: -kv[1]["ms_per_launch"] * kv[1]["launches"])
for k, v in ks[:6]:
    print(f"  {k:24s} {v['ms_per_launch'] * v['launches'] / b['steps']:9.2f} ms/step  {v['GBps']:8.1f} GB/s")
PY
done
cp /tmp/libapg_B.so allpathslg_amd/libapg.so
