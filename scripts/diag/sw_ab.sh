set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_align.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/sw_pytest.log 2>&1 || { tail -30 gpurun_out/sw_pytest.log; exit 1; }
tail -2 gpurun_out/sw_pytest.log
timeout -k 10 200 python scripts/diag/sw_only.py 4000000 8 5 && cp allpathslg_amd/libapg.so /tmp/B.so && cp allpathslg_amd/libapg_var.so allpathslg_amd/libapg.so && echo "== old" && timeout -k 10 200 python scripts/diag/sw_only.py 4000000 8 5; rc=$?; cp /tmp/B.so allpathslg_amd/libapg.so; exit $rc
