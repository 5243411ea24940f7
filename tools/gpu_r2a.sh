# Round-2 check: full GPU test suite, then the default bench line and the per_token line.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r2a
O=gpurun_out/r2a
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 180 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1 || { echo "pytest failed"; grep -E "FAILED|Error|error|assert" $O/pytest_gpu.log | head -40; tail -40 $O/pytest_gpu.log; exit 1; }
tail -3 $O/pytest_gpu.log
grep -E "^opt|^llama" $O/pytest_gpu.log || true
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench_driver.json 2> $O/bench_driver.err || { echo "bench failed"; tail -20 $O/bench_driver.err; exit 1; }
cat $O/bench_driver.json
timeout -k 10 300 python bench.py --act per_token --no-cpu > $O/bench_pt.json 2> $O/bench_pt.err || { echo "bench pt failed"; tail -20 $O/bench_pt.err; exit 1; }
cat $O/bench_pt.json
