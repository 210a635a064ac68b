#!/bin/bash
# Kernel statistics of the repeats line's counting stage (rep_fused.py) with
# the overflowed buckets by sub-bucket (default) and through the global table.
set -o pipefail
R="$GRAFT_REPO_ROOT"
O="$R/gpurun_out/r5rp"
cd /tmp && export TMPDIR=/tmp
mkdir -p "$O"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/sub" -o p -- python3 "$R/scripts/diag/rep_fused.py" 2 > "$O/sub.log" 2>&1 \
 && APG_SK_OVF=global timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/glob" -o p -- python3 "$R/scripts/diag/rep_fused.py" 2 > "$O/glob.log" 2>&1 \
 && for v in sub glob; do echo "== $v"; f=$(find "$O/$v" -name "*kernel_stats.csv" | head -1); python3 - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:22]:
    print(f"{r['Name'].split('(')[0][-50:]:50s} {int(r['Calls']):4d} {float(r['AverageNs'])/1e6:8.3f} ms")
PY
grep "sk count\|{" "$O/$v.log" | tail -4; done
