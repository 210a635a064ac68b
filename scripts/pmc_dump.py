"""Per-kernel sums of every counter in one or more rocprofv3 --pmc csv
directories (top kernels by the first counter seen)."""
import csv
import glob
import sys
from collections import defaultdict

agg = defaultdict(lambda: defaultdict(float))
for d in sys.argv[1:]:
    for f in glob.glob(d + "/**/*counter_collection*.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            k = r.get("Kernel_Name", "?").split("(")[0][-44:]
            agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
names = sorted({n for v in agg.values() for n in v})
top = sorted(agg.items(), key=lambda kv: -kv[1].get("SQ_WAVE_CYCLES", 0))[:8]
for k, v in top:
    print(k)
    for n in names:
        print(f"   {n:24s} {v.get(n, 0):.4e}")
