"""Per-stream kernel timeline of the last bench step in a rocprofv3
--kernel-trace csv directory (scripts/gpu_timeline.sh): start / end / ms /
queue of every dispatch longer than 0.15 ms, relative to the step's first
k_sk_count — which stream waits on which."""
import csv
import glob
import sys

rows = []
for f in glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True):
    rows += list(csv.DictReader(open(f)))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
starts = [i for i, r in enumerate(rows) if r["Kernel_Name"].startswith("apg::k_sk_count")]
i0 = starts[-1]
t0 = int(rows[i0]["Start_Timestamp"])
for r in rows[max(0, i0 - 4):]:
    s = (int(r["Start_Timestamp"]) - t0) / 1e6
    e = (int(r["End_Timestamp"]) - t0) / 1e6
    if e - s > 0.15:
        print(f"{s:8.2f} {e:8.2f} {e - s:7.2f} q{r['Queue_Id']} {r['Kernel_Name'].split('(')[0][:64]}")
