# checkpoint-bias fix: full GPU suite, then the config-2 GEMM timings (fq, f8)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r2g; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 || { echo "pytest failed"; grep -E "FAILED|Error" $O/pytest.log | head -20; tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 60 python tools/gemm_time.py f8 300 || exit 1
timeout -k 10 60 python tools/gemm_time.py fq 300 || exit 1
