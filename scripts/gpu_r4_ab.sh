#!/bin/bash
# A/B on one GPU box: the bench step (and the repeats / C3 lines) under each
# variant's environment, one process per variant, kernel tables summarised.
#   VARIANTS="base:;sort:APG_SK_UP_SORT=1;nocache:APG_FILL_BRANCH_CACHE=0" bash scripts/gpu_r4_ab.sh
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${TAG:-ab}
mkdir -p $O
A="--steps ${STEPS:-4} --warmup 2 --no-cpu-baseline --no-file-to-graph --align-pairs 0 --jump-pairs 0 --no-placement ${EXTRA:-}"
IFS=';' read -ra VS <<< "${VARIANTS:-base:}"
for v in "${VS[@]}"; do
  name=${v%%:*}; envs=${v#*:}
  echo "== $name ($envs)"
  env $envs timeout -k 10 ${T_BENCH:-300} python bench.py $A > $O/$name.json 2> $O/$name.err || exit $?
  python scripts/bench_summary.py $O/$name.json || exit $?
  python - "$O/$name.json" <<'PY' || exit $?
import json, sys
b = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
for k in ("repeats", "c3"):
    x = b.get(k) or {}
    if x:
        print(f"  {k}: {x.get('ms_per_step', 0):.1f} ms/step", {kk: round(vv, 2) for kk, vv in (x.get("kernels_ms") or {}).items()
                                                            if vv > 2} if isinstance(x.get("kernels_ms"), dict) else "")
PY
done
echo "== done"
