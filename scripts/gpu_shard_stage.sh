#!/bin/bash
# The sharded bench path with staged per-step inputs: world 1 over RCCL at
# the C2 size, then world 2 over TCP with both ranks on GPU 0 (small size).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29533 \
  bench.py --sharded --steps 3 --warmup 1 --no-cpu-baseline --c3-jump-pairs 0 --no-file-to-graph --align-pairs 0 --no-placement --repeat-steps 0 \
  > gpurun_out/bench_shard1.json 2> gpurun_out/bench_shard1.err \
 && cat gpurun_out/bench_shard1.json \
 && timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29534 \
  bench.py --gpus 2 --comm tcp --steps 3 --warmup 1 --reads-per-gpu 10000000 --genome-len 20000000 --no-cpu-baseline \
  --c3-jump-pairs 0 --no-file-to-graph --align-pairs 0 --no-placement --repeat-steps 0 \
  > gpurun_out/bench_shard2.json 2> gpurun_out/bench_shard2.err \
 && cat gpurun_out/bench_shard2.json
