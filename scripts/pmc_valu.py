"""VALU issue share per kernel from two rocprofv3 --pmc csv directories
(scripts/gpu_pmc_valu.sh).  SQ_ACTIVE_INST_* and SQ_WAIT_* and SQ_WAVE_CYCLES
count quad-cycles (MI355X_MICROARCH.md); GRBM_GUI_ACTIVE is summed over the 8
XCDs.  valu_busy = SQ_ACTIVE_INST_VALU x 4 / (kernel cycles x 256 CUs x 4
SIMDs): the share of SIMD cycles the VALU issued; valu_issue_bound =
SQ_INSTS_VALU x 2 cycles / (the same): what the VALU instructions alone need
at one wave instruction per 2 cycles per SIMD."""
import csv
import glob
import sys
from collections import defaultdict


def load(d):
    per = defaultdict(lambda: defaultdict(float))
    for f in glob.glob(d + "/**/*counter_collection*.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            k = r.get("Kernel_Name", "?").split("(")[0].strip()
            per[k][r["Counter_Name"]] += float(r["Counter_Value"])
            per[k]["_rows"] += 1
    return per


sq, gui = load(sys.argv[1]), load(sys.argv[2])
SIMDS = 256 * 4
rows = []
for k, v in sq.items():
    g = gui.get(k, {}).get("GRBM_GUI_ACTIVE", 0.0) / 8
    if g <= 0:
        continue
    wc = v.get("SQ_WAVE_CYCLES", 0.0)
    rows.append((g, k, v.get("SQ_ACTIVE_INST_VALU", 0.0) * 4 / (g * SIMDS), v.get("SQ_INSTS_VALU", 0.0) * 2 / (g * SIMDS),
                 v.get("SQ_WAIT_INST_LDS", 0.0) / wc if wc else 0.0, v.get("SQ_WAIT_ANY", 0.0) / wc if wc else 0.0,
                 wc * 4 / (g * SIMDS), v.get("SQ_INSTS_LDS", 0.0) / max(v.get("SQ_INSTS_VALU", 1.0), 1.0)))
rows.sort(reverse=True)
print(f"{'kernel':56s} {'Mcyc':>7s} {'valu_busy':>9s} {'valu_iss':>8s} {'wLDS':>6s} {'wAny':>6s} {'waves/SIMD':>10s} {'lds/valu':>8s}")
for g, k, vb, vi, wl, wa, occ, lv in rows[:25]:
    print(f"{k[-56:]:56s} {g / 1e6:7.2f} {vb:9.3f} {vi:8.3f} {wl:6.3f} {wa:6.3f} {occ:10.2f} {lv:8.3f}")
