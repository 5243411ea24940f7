# FP6 per_token path: f6 + f8 GPU tests, then config-2 GEMM timings
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r2i; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_f6.py tests/test_gpu_f8.py -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 || { echo "pytest failed"; grep -E "FAILED|Error|assert" $O/pytest.log | head -20; tail -5 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 60 python tools/gemm_time.py f6 300 || exit 1
timeout -k 10 60 python tools/gemm_time.py f8 300 || exit 1
