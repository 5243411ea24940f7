# f8v2 LDS-staged epilogue: f8 GPU tests, then config-2 timings
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r2h; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_f8.py tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 || { echo "pytest failed"; grep -E "FAILED|Error" $O/pytest.log | head -20; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 60 python tools/gemm_time.py f8 300 || exit 1
timeout -k 10 60 python tools/gemm_time.py f8 300 || exit 1
