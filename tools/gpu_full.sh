# Round check on the GPU box: smoke, GPU tests, config-2 bench, config-4 Llama bench.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo "smoke failed"; tail -30 gpurun_out/smoke.log; exit 1; }
tail -2 gpurun_out/smoke.log
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -60 gpurun_out/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/pytest_gpu.log
timeout -k 10 400 python bench.py > gpurun_out/bench_pg.json 2> gpurun_out/bench_pg.err || { echo "bench failed"; tail -20 gpurun_out/bench_pg.err; exit 1; }
cat gpurun_out/bench_pg.json
if [ -z "$NO_LLAMA" ]; then
timeout -k 10 600 python bench_llama.py ${LLAMA_ARGS} > gpurun_out/bench_llama.json 2> gpurun_out/bench_llama.err || { echo "llama failed"; tail -20 gpurun_out/bench_llama.err; exit 1; }
cat gpurun_out/bench_llama.json
fi
