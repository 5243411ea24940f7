# GEMM change check: GPU parity tests of the GEMM paths, the GEMM timing matrix, quick bench.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
TESTS="${TESTS:-tests/test_gpu_parity.py tests/test_gpu_models.py tests/test_gpu_sweep.py}" bash tools/gpu_tests.sh || exit 1
timeout -k 10 300 python tools/gemm_matrix.py || exit 1
bash tools/gpu_bench_quick.sh
