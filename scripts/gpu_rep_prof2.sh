#!/bin/bash
# Repeats parity tests, then the counting stage's kernel statistics.
set -o pipefail
R="$GRAFT_REPO_ROOT"
O="$R/gpurun_out/r5rp2"
mkdir -p "$O"
cd "$R" && timeout -k 10 400 python -u -m pytest tests/test_gpu_repeats.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/rep_tests.log 2>&1 || { tail -30 $O/rep_tests.log; exit 1; }
tail -n 1 $O/rep_tests.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/sub" -o p -- python3 "$R/scripts/diag/rep_fused.py" 2 > "$O/sub.log" 2>&1 || { tail -5 "$O/sub.log"; exit 1; }
python3 - "$O/sub/p_kernel_stats.csv" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:24]:
    print(f"{r['Name'].split('(')[0][-50:]:50s} {int(r['Calls']):4d} {float(r['AverageNs'])/1e6:8.3f} ms")
PY
