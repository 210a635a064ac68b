#!/bin/bash
# Round-4 iteration on one GPU box: the changed paths' parity tests, then the
# single-GPU bench step and the sharded step at world size 1 (RCCL), with the
# per-kernel times.  Each GPU step has its own time limit; && chains them so
# the first failure ends the call.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${TAG:-r4}
mkdir -p $O
A="--no-cpu-baseline --c3-jump-pairs 0 --no-file-to-graph --align-pairs 0 --jump-pairs 0 --no-placement --repeat-steps 0"
echo "== tests" && timeout -k 10 ${T_TEST:-900} python -u -m pytest ${TESTS:-tests/test_gpu_fused.py tests/test_distributed.py} \
   -m gpu -x -v --timeout 600 --timeout-method thread > $O/pytest.log 2>&1 \
 && tail -3 $O/pytest.log \
 && echo "== bench" && timeout -k 10 300 python bench.py --steps ${STEPS:-5} --warmup 2 $A > $O/bench.json 2> $O/bench.err \
 && python scripts/bench_summary.py $O/bench.json \
 && echo "== sharded w1" && timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 \
   --master-addr 127.0.0.1 --master-port 29533 bench.py --sharded --steps ${STEPS:-5} --warmup 2 $A \
   > $O/bench_sharded.json 2> $O/bench_sharded.err \
 && python scripts/bench_summary.py $O/bench_sharded.json \
 && echo "== done"
