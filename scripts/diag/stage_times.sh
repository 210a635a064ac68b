cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
L="--steps 2 --warmup 1 --no-cpu-baseline --c3-jump-pairs 0 --no-file-to-graph --align-pairs 0 --jump-pairs 0 --no-placement --repeat-steps 0 --stage-times"
timeout -k 10 300 python bench.py $L > /dev/null 2> gpurun_out/st_single.err && \
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29651 bench.py --sharded $L > /dev/null 2> gpurun_out/st_sharded.err && \
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29661 bench.py --sharded --gather-nodes $L > /dev/null 2> gpurun_out/st_gather.err
for f in single sharded gather; do echo "== $f"; grep "stage" gpurun_out/st_$f.err | tail -5; done
