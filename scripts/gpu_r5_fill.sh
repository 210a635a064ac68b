#!/bin/bash
# Round 5: K=96 walk column A/B (APG_USK_FLAT), FillFragments lean/general
# A/B on the repeat-rich and iid genomes, then a PC-sampling profile of fill.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5f
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_repeats.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/rep_tests.log 2>&1 || { tail -30 $O/rep_tests.log; exit 1; }
tail -2 $O/rep_tests.log
timeout -k 10 300 python -u -m pytest tests/test_gpu_fill.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/fill_tests.log 2>&1 || { tail -30 $O/fill_tests.log; exit 1; }
tail -2 $O/fill_tests.log
env APG_USK_FLAT=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_unipath.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/unipath_flat.log 2>&1 || { tail -30 $O/unipath_flat.log; exit 1; }
tail -2 $O/unipath_flat.log
A="APG_USK_FLAT=0" B="APG_USK_FLAT=1" VARIANTS="A B A B" bash scripts/gpu_ab.sh > $O/ab_flat.txt 2>&1 || { tail -20 $O/ab_flat.txt; exit 1; }
cat $O/ab_flat.txt
FILL_CASES=base,nolean,nofuse,base2 timeout -k 10 300 python -u scripts/diag/fill_rep.py > $O/fill_rep.txt 2>&1 || { tail -20 $O/fill_rep.txt; exit 1; }
cat $O/fill_rep.txt
FILL_GENOME=iid FILL_CASES=base,nolean,nofuse,base2 timeout -k 10 300 python -u scripts/diag/fill_rep.py > $O/fill_iid.txt 2>&1 || { tail -20 $O/fill_iid.txt; exit 1; }
cat $O/fill_iid.txt
BA_OVERRIDE="--steps 2 --warmup 1 --no-cpu-baseline --c3-jump-pairs 0 --no-file-to-graph --align-pairs 0 --jump-pairs 0 --no-placement --repeat-steps 2" A="APG_SK_OVF=global" B="APG_SK_OVF=" C="APG_SK_OVF= APG_EXT_HASH=1" VARIANTS="A B C" bash scripts/gpu_ab.sh > $O/ab_rep.txt 2>&1 || { tail -20 $O/ab_rep.txt; exit 1; }
cat $O/ab_rep.txt
