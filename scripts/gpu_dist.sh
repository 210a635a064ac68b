#!/bin/bash
# Sharded path on the GPU box: the C-ABI multi-process tests (TCP comm, ranks
# sharing GPU 0; RCCL world 1 with self P2P), then the sharded bench at
# world size 1 over RCCL.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 400 --timeout-method thread tests/test_distributed.py > gpurun_out/pytest_dist.log 2>&1
rc=$?; tail -15 gpurun_out/pytest_dist.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29533 \
  bench.py --sharded --steps 3 --warmup 1 --no-cpu-baseline --align-pairs 0 --no-placement > gpurun_out/bench_sharded.json 2> gpurun_out/bench_sharded.err
rc=$?; tail -3 gpurun_out/bench_sharded.err; exit $rc
