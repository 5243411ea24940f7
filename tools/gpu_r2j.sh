# Re-entry check: full GPU suite, then the f6/f8/fq config-2 GEMM timings.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r2j; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 || { echo "pytest failed"; grep -E "FAILED|Error|assert" $O/pytest.log | head -20; tail -5 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 60 python tools/gemm_time.py f6 300 || exit 1
timeout -k 10 60 python tools/gemm_time.py f8 300 || exit 1
timeout -k 10 60 python tools/gemm_time.py fq 300 || exit 1
