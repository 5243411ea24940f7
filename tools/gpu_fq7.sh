# fq7 register-operand GEMM: parity tests for both tile shapes, then config-2 timings
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/fq7; mkdir -p $O
for j in 2 4; do
SQMP_FQ7_J=$j timeout -k 10 300 python -u -m pytest tests/test_gpu_fq7.py -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest_j$j.log 2>&1 || { echo "pytest J=$j failed"; grep -E "FAILED|Error|assert" $O/pytest_j$j.log | head -20; tail -30 $O/pytest_j$j.log; exit 1; }
tail -1 $O/pytest_j$j.log
done
for j in 2 4; do echo -n "J=$j "; SQMP_FQ7_J=$j timeout -k 10 60 python tools/gemm_time.py fq7 300 || exit 1; done
timeout -k 10 60 python tools/gemm_time.py fq 300 || exit 1
for d in 1 2 3; do echo -n "J=2 diag=$d "; SQMP_FQ7_J=2 SQMP_FQ7_DIAG=$d timeout -k 10 60 python tools/gemm_time.py fq7 300 || exit 1; done
