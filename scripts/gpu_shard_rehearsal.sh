#!/bin/bash
# Sharded bench paths on the one-GPU box: world 1 over RCCL (sharded and
# replicated unipath compaction), then world 2 over TCP with both ranks on
# GPU 0 (a functional rehearsal of the driver's N > 1 runs at reduced size).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
L="--steps 3 --warmup 1 --no-cpu-baseline --c3-jump-pairs 0 --no-file-to-graph --align-pairs 0 --jump-pairs 0 --no-placement --repeat-steps 0"
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29611 bench.py --sharded $L > gpurun_out/bench_w1_sharded.json 2> gpurun_out/bench_w1_sharded.err \
 && timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29621 bench.py --sharded --gather-nodes $L > gpurun_out/bench_w1_gather.json 2> gpurun_out/bench_w1_gather.err \
 && timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29631 bench.py --gpus 2 --comm tcp --reads-per-gpu ${RPG:-20000000} $L > gpurun_out/bench_w2_tcp.json 2> gpurun_out/bench_w2_tcp.err
rc=$?
[ $rc -eq 0 ] && timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29641 bench.py --sharded --verbose --steps 1 --warmup 1 --no-cpu-baseline --c3-jump-pairs 0 --no-file-to-graph --align-pairs 0 --jump-pairs 0 --no-placement --repeat-steps 0 > gpurun_out/bench_w1_verbose.json 2> gpurun_out/bench_w1_verbose.err
grep "phase" gpurun_out/bench_w1_verbose.err | tail -9
for f in bench_w1_sharded bench_w1_gather bench_w2_tcp; do
  python - "$f" <<'PY'
import json, sys
f = sys.argv[1]
try:
    b = json.load(open(f"gpurun_out/{f}.json"))
except Exception as e:
    print(f, "no result", e); sys.exit(0)
k = b.get("kernels", {})
top = sorted(k.items(), key=lambda kv: -kv[1]["ms_per_launch"] * kv[1]["launches"])[:12]
print(f, round(b["value"] / 1e6, 2), "M reads/s", round(b["ms_per_step"], 1), "ms/step", "checks", {c: v for c, v in b.get("checks", {}).items() if not v} or "all ok")
print("   ", ", ".join(f"{n} {v['ms_per_launch'] * v['launches'] / b['steps']:.1f}" for n, v in top))
PY
done
exit $rc
