"""GPU idle gaps in the last bench step of a rocprofv3 --kernel-trace
--memory-copy-trace csv directory (scripts/gpu_timeline.sh).  The step is
taken as the span of the last k_sk_count dispatch through the last dispatch
before the end; a gap is time with no kernel or copy running on any queue."""
import csv
import glob
import sys

ops = []
for f in glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        ops.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].split("(")[0][-48:]))
for f in glob.glob(sys.argv[1] + "/**/*memory_copy_trace.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        ops.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "copy " + r.get("Direction", "?")))
ops.sort()
starts = [i for i, o in enumerate(ops) if o[2].endswith("k_sk_count")]
i0 = starts[-1]
step = ops[i0:]
t_end = max(o[1] for o in step)
busy, gaps, cur = 0, [], step[0][0]
prev = step[0][2]
for s, e, n in step:
    if s > cur:
        gaps.append((s - cur, prev, n))
    if e > cur:
        busy += e - max(s, cur)
        cur = e
        prev = n
span = t_end - step[0][0]
print(f"step span {span / 1e6:.2f} ms, busy {busy / 1e6:.2f} ms, idle {(span - busy) / 1e6:.2f} ms in {len(gaps)} gaps")
gaps.sort(reverse=True)
for g, a, b in gaps[:40]:
    print(f"{g / 1e3:9.1f} us  after {a:48s} before {b}")
