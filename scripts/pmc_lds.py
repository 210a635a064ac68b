"""LDS roofline per kernel from a rocprofv3 --pmc csv directory
(scripts/gpu_pmc_lds.sh): LDS-array utilisation = SQ_LDS_IDX_ACTIVE /
(GRBM_GUI_ACTIVE x CUs) (rocprofiler's LdsUtil for gfx950), bank-conflict
share of those cycles, LDS instructions per wave cycle, and the share of wave
cycles spent waiting (SQ_WAIT_ANY) and issuing (SQ_ACTIVE_INST_ANY).  Counter
values are summed over every dispatch of a kernel; GRBM_GUI_ACTIVE is the
dispatch's busy cycles; rocprofv3 reports it summed over the 8 XCDs
(MI355X_MICROARCH.md, DVFS note), so one kernel-wall cycle count is the sum
divided by 8.  SQ_LDS_IDX_ACTIVE is summed over every CU's LDS."""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

CUS = 256
XCDS = 8  # GRBM_GUI_ACTIVE instances summed by rocprofv3
rows = []
for f in glob.glob(sys.argv[1] + "/**/*counter_collection*.csv", recursive=True):
    rows += list(csv.DictReader(open(f)))
per = defaultdict(lambda: defaultdict(float))  # (kernel, dispatch) -> counter -> value
for r in rows:
    k = r.get("Kernel_Name", "?").split("(")[0].strip()
    d = r.get("Dispatch_Id", "0")
    per[(k, d)][r["Counter_Name"]] += float(r["Counter_Value"])
agg = defaultdict(lambda: defaultdict(float))
for (k, _), v in per.items():
    for c, x in v.items():
        agg[k][c] += x
    agg[k]["dispatches"] += 1
out = {}
for k, v in agg.items():
    gui = v.get("GRBM_GUI_ACTIVE", 0.0) / XCDS
    idx = v.get("SQ_LDS_IDX_ACTIVE", 0.0)
    wc = v.get("SQ_WAVE_CYCLES", 0.0)
    out[k] = {
        "dispatches": int(v["dispatches"]),
        "lds_util": idx / (gui * CUS) if gui else None,
        "bank_conflict_share": v.get("SQ_LDS_BANK_CONFLICT", 0.0) / idx if idx else None,
        "lds_insts": v.get("SQ_INSTS_LDS", 0.0),
        "valu_insts": v.get("SQ_INSTS_VALU", 0.0),
        "wait_any_share": v.get("SQ_WAIT_ANY", 0.0) / wc if wc else None,
        "active_inst_share": v.get("SQ_ACTIVE_INST_ANY", 0.0) / wc if wc else None,
        "wait_inst_lds_share": v.get("SQ_WAIT_INST_LDS", 0.0) / wc if wc else None,
        "gui_cycles": gui,
        "raw": dict(v),
    }
json.dump(out, open(sys.argv[1].rstrip("/") + ".json", "w"), indent=1)
# by bench timing label (scripts/pmc_traffic.py's symbol map; a timed region of
# two kernels — sk_bucket_solid — sums both): <dir>/lds.json, read by bench.py
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_traffic import KERNELS, matches  # noqa: E402

lab = defaultdict(lambda: defaultdict(float))
for k, v in agg.items():
    for sym, label, _ in KERNELS:
        if matches(k + "(", sym):
            for c in ("GRBM_GUI_ACTIVE", "SQ_LDS_IDX_ACTIVE", "SQ_LDS_BANK_CONFLICT", "SQ_INSTS_LDS", "dispatches"):
                lab[label][c] += v.get(c, 0.0)
            break
by_label = {}
for label, v in lab.items():
    gui = v["GRBM_GUI_ACTIVE"] / XCDS
    idx = v["SQ_LDS_IDX_ACTIVE"]
    by_label[label] = {"lds_util": idx / (gui * CUS) if gui else None,
                       "bank_conflict_share": v["SQ_LDS_BANK_CONFLICT"] / idx if idx else None,
                       "lds_insts_per_dispatch": v["SQ_INSTS_LDS"] / max(v["dispatches"], 1),
                       "definition": "SQ_LDS_IDX_ACTIVE / (GRBM_GUI_ACTIVE / 8 x 256 CUs); peak 1.0 = every CU's "
                                     "LDS array busy every cycle (128 B/clk/CU)"}
json.dump(by_label, open(os.path.join(sys.argv[1], "lds.json"), "w"), indent=1)
top = sorted(out.items(), key=lambda kv: -kv[1]["gui_cycles"])[:20]
print(f"{'kernel':58s} {'disp':>4s} {'gui_Mcyc':>9s} {'lds_util':>8s} {'confl':>6s} {'wait':>6s} {'issue':>6s} {'wLDS':>6s}")
f = lambda x: f"{x:6.3f}" if x is not None else "   n/a"
for k, v in top:
    print(f"{k[-58:]:58s} {v['dispatches']:4d} {v['gui_cycles'] / 1e6:9.2f} {f(v['lds_util']):>8s} "
          f"{f(v['bank_conflict_share'])} {f(v['wait_any_share'])} {f(v['active_inst_share'])} {f(v['wait_inst_lds_share'])}")
