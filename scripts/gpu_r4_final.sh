#!/bin/bash
# Round-4 closing runs on one GPU box.  PART=a: the full GPU suite + smoke,
# then the fill knob A/B on both genomes; PART=b: the perf checkpoint (PMC
# traffic passes, bench, rocprof kernel trace) and the LDS and SQ counter
# passes.  Each GPU step has its own time limit; && chains them so the first
# failure ends the call.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
if [ "${PART:-a}" = a ]; then
  PHASE=tests T_TEST=${T_TEST:-900} bash scripts/gpu_checkpoint.sh \
   && echo "== fill knobs" \
   && FILL_CASES=${FILL_CASES:-base,x0,p25,p90,refill8,refill48} timeout -k 10 400 python -u scripts/diag/fill_rep.py > gpurun_out/fill_rep6.log 2>&1 \
   && FILL_GENOME=iid FILL_CASES=${FILL_CASES:-base,x0,p25,p90,refill8,refill48} timeout -k 10 400 python -u scripts/diag/fill_rep.py > gpurun_out/fill_iid6.log 2>&1 \
   && echo "== done"
else
  PHASE=perf bash scripts/gpu_checkpoint.sh \
   && OUT=pmc_lds bash scripts/gpu_pmc_lds.sh > /dev/null \
   && TAG=r4pmc bash scripts/gpu_r4_pmc.sh > /dev/null \
   && echo "== done"
fi
