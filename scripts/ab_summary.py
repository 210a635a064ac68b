"""One bench detail file -> step time, checks and the largest kernels
(scripts/gpu_r6_ab.sh)."""
import json
import sys

b = json.load(open(sys.argv[1]))
print("value", round(b["value"] / 1e6, 2), "M reads/s  ms/step", round(b["ms_per_step"], 2), "checks",
      all(b["checks"].values()))
ks = sorted(b["kernels"].items(), key=lambda kv: -kv[1]["ms_per_launch"] * kv[1]["launches"])
for k, v in ks[:14]:
    print(f"  {k:24s} {v['ms_per_launch'] * v['launches'] / b['steps']:9.2f} ms/step  {v['GBps']:8.1f} GB/s"
          f"  ovl {v.get('overlapped_launches', 0)}")
r = b.get("repeats")
if r:
    print("repeats ms/step", round(r["ms_per_step"], 2), "x main", round(r["ms_per_step"] / b["ms_per_step"], 3),
          "checks", all(r["checks"].values()))
