"""One bench JSON line -> step time, rate and the per-kernel ms/step table."""
import json
import sys

b = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print("value", round(b["value"] / 1e6, 2), "M reads/s  ms/step", round(b["ms_per_step"], 2), "checks",
      all(b.get("checks", {}).values()))
r = b.get("roofline") or {}
print("roofline", r.get("kernel"), round(r.get("frac") or 0, 4), r.get("ms_per_launch"))
ks = sorted(b.get("kernels", {}).items(), key=lambda kv: -kv[1]["ms_per_launch"] * kv[1]["launches"])
tot = 0.0
for k, v in ks:
    ms = v["ms_per_launch"] * v["launches"] / b["steps"]
    tot += ms
    if ms >= 0.3:
        print(f"  {k:24s} {ms:8.2f} ms/step  {v.get('GBps', 0):8.1f} GB/s")
print("  kernel sum", round(tot, 1))
