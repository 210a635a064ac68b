#!/bin/bash
# Sharded PreCorrect at P > 1: the distributed parity tests, then the world-2
# TCP rehearsal (both ranks on GPU 0, 20 M reads each) with the self-owned
# records' weak bits written straight into the bitmap (default) and with every
# mask returned (APG_SHARD_SELF=0).  Outputs under gpurun_out/r5s/.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5s
mkdir -p $O
L="--steps 3 --warmup 1 --no-cpu-baseline --c3-jump-pairs 0 --no-file-to-graph --align-pairs 0 --jump-pairs 0 --no-placement --repeat-steps 0"
PT="python -u -m pytest -x -q --timeout 400 --timeout-method thread"
echo "== dist tests" && timeout -k 10 800 $PT tests/test_distributed.py tests/test_distributed_scale.py tests/test_sharded_graph.py > $O/dist_tests.log 2>&1 && tail -2 $O/dist_tests.log \
 && echo "== w2 self" && timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29631 bench.py --gpus 2 --comm tcp --reads-per-gpu 20000000 $L --detail-json $O/w2_self_detail.json > $O/w2_self.json 2> $O/w2_self.err \
 && echo "== w2 all masks" && APG_SHARD_SELF=0 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29641 bench.py --gpus 2 --comm tcp --reads-per-gpu 20000000 $L --detail-json $O/w2_all_detail.json > $O/w2_all.json 2> $O/w2_all.err \
 && for f in w2_self w2_all; do python3 - $O/${f}_detail.json <<'PY'
import json, sys
b = json.load(open(sys.argv[1]))
k = b["kernels"]
w = k.get("weak_apply", {})
print(sys.argv[1], round(b["ms_per_step"], 1), "ms/step", "weak_apply", round(w.get("ms_per_launch", 0) * w.get("launches", 0) / b["steps"], 2), "ms/step",
      "bytes/launch", round(w.get("GBps", 0) * w.get("ms_per_launch", 0) * 1e-3 * 1e9 / 1e6, 1), "MB", "checks", all(b["checks"].values()))
PY
done
