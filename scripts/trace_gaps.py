#!/usr/bin/env python3
"""Idle time between kernels of one bench step, from a rocprofv3
--kernel-trace CSV: the step's span, busy time, and the largest gaps with the
kernels on either side (host round trips show up as gaps).

  python scripts/trace_gaps.py gpurun_out/prof/run_kernel_trace.csv
"""
import csv
import sys


def main(path, top=25):
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    names = [r["Kernel_Name"].split("(")[0][:44] for r in rows]
    st = [int(r["Start_Timestamp"]) for r in rows]
    en = [int(r["End_Timestamp"]) for r in rows]
    # a step starts with the spectrum's sk_count (the solid pass launches a second one)
    first = [i for i, n in enumerate(names) if n.startswith("apg::k_sk_count")][::2]
    for a, b in zip(first, first[1:]):
        print(f"step span {(st[b] - st[a]) / 1e6:8.2f} ms")
    a, b = first[-2], first[-1]
    busy = sum(en[i] - st[i] for i in range(a, b))
    gaps = sorted(((st[i + 1] - en[i], names[i], names[i + 1]) for i in range(a, b)), reverse=True)
    idle = sum(g for g, _, _ in gaps if g > 0)
    print(f"last full step: span {(st[b] - st[a]) / 1e6:.2f} ms, busy {busy / 1e6:.2f} ms, "
          f"idle {idle / 1e6:.2f} ms over {len(gaps)} gaps")
    for g, x, y in gaps[:top]:
        print(f"{g / 1e3:9.1f} us  {x:46s} -> {y}")
    # kernels around the largest gap
    w = max(range(a, b), key=lambda i: st[i + 1] - en[i])
    print("around the largest gap:")
    for i in range(max(a, w - 6), min(len(rows), w + 8)):
        print(f"  {(st[i] - st[a]) / 1e6:9.3f} ms  dur {(en[i] - st[i]) / 1e3:9.1f} us  {names[i]}")


if __name__ == "__main__":
    main(sys.argv[1])
