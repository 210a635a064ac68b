# The fused counting pass's bucket routes (redo / overflow / distinct records)
# with and without the dedup-fed K+1 pass: bench step with --verbose.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
BA="--steps 1 --warmup 0 --verbose --no-cpu-baseline --c3-jump-pairs 0 --no-file-to-graph --align-pairs 0 --jump-pairs 0 --no-placement --repeat-steps 0"
for V in 1 0; do
  APG_SK_UP_DD=$V APG_SK_PROF=1 timeout -k 10 300 python bench.py $BA > gpurun_out/skv_$V.json 2> gpurun_out/skv_$V.err || { tail -5 gpurun_out/skv_$V.err; exit 1; }
  echo "== APG_SK_UP_DD=$V"; grep -E "sk count|sk_prof|K\+1" gpurun_out/skv_$V.err | head -12
done
