# fq7 register-operand GEMM: parity tests, then config-2 timings fq7 vs fq.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/fq7; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_fq7.py -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 || { echo "pytest failed"; grep -E "FAILED|Error|assert" $O/pytest.log | head -20; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 60 python tools/gemm_time.py fq7 300 || exit 1
timeout -k 10 60 python tools/gemm_time.py fq 300 || exit 1
for g in 4 16; do SQMP_FQ7_GROUP_M=$g timeout -k 10 60 python tools/gemm_time.py fq7 300 || exit 1; done
