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
names = ["SQ_WAVE_CYCLES", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS", "SQ_WAVES",
         "SQ_LDS_BANK_CONFLICT", "SQ_LDS_IDX_ACTIVE"]
top = sorted(agg.items(), key=lambda kv: -kv[1]["SQ_WAVE_CYCLES"])[:14]
print(f"{'kernel':40s} " + " ".join(f"{n[3:15]:>12s}" for n in names))
for k, v in top:
    print(f"{k:40s} " + " ".join(f"{v[n]:12.3e}" for n in names))
