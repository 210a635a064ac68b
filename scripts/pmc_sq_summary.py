"""Sum SQ counters per kernel from a rocprofv3 --pmc csv directory."""
import csv
import glob
import sys
from collections import defaultdict

rows = []
for f in glob.glob(sys.argv[1] + "/**/*counter_collection*.csv", recursive=True):
    rows += list(csv.DictReader(open(f)))
agg = defaultdict(lambda: defaultdict(float))
for r in rows:
    k = r.get("Kernel_Name", "?").split("(")[0][-40:]
    agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
names = sorted({c for v in agg.values() for c in v})  # the counters this pass collected
top = sorted(agg.items(), key=lambda kv: -max(kv[1].values()))[:14]
print(f"{'kernel':40s} " + " ".join(f"{n[3:15]:>12s}" for n in names))
for k, v in top:
    print(f"{k:40s} " + " ".join(f"{v[n]:12.3e}" for n in names))
