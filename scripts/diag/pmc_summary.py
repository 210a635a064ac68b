"""Per-dispatch sums of a rocprofv3 --pmc counter_collection.csv for the
kernels whose name contains argv[2], with derived SQ figures (waves per SIMD,
cycles per VALU instruction per SIMD; GRBM_GUI_ACTIVE summed over 8 XCDs)."""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
agg = collections.defaultdict(lambda: collections.defaultdict(float))
for r in rows:
    if sys.argv[2] in r["Kernel_Name"]:
        agg[r["Dispatch_Id"]][r["Counter_Name"]] += float(r["Counter_Value"])
for d, v in agg.items():
    print(d, {k: f"{x:.4g}" for k, x in v.items()})
    g = v.get("GRBM_GUI_ACTIVE", 0) / 8
    if g and "SQ_WAVE_CYCLES" in v and "SQ_INSTS_VALU" in v:
        print("  waves/SIMD %.2f  cycles/VALU-instr/SIMD %.2f  VALU instr %.4g" %
              (v["SQ_WAVE_CYCLES"] * 4 / 1024 / g, g / (v["SQ_INSTS_VALU"] / 1024), v["SQ_INSTS_VALU"]))
