# GPU parity tests, then the quick bench (both act modes).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -q --maxfail=10 -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?
tail -15 gpurun_out/pytest_gpu.log
[ $rc -ne 0 ] && { echo "gpu tests failed rc=$rc"; exit $rc; }
bash tools/gpu_bench_quick.sh
