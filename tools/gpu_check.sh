# GPU tests, then a driver-shaped bench line (20 steps / 5 warmup) of both act modes.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/check
O=gpurun_out/check
timeout -k 10 600 python -u -m pytest ${TESTS:-tests} -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1 || { echo "pytest failed"; grep -E "FAILED|Error|assert" $O/pytest_gpu.log | head -40; tail -30 $O/pytest_gpu.log; exit 1; }
tail -3 $O/pytest_gpu.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench_pg.json 2> $O/bench_pg.err || { echo "bench failed"; tail -20 $O/bench_pg.err; exit 1; }
cat $O/bench_pg.json
