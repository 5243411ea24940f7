# Round evidence, part A: GPU tests, bench lines (headline default, driver-shaped 20/5,
# per_token, fp32), rocprofv3 kernel stats of the default bench.  Results -> gpurun_out/round.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out/round
O=$R/gpurun_out/round
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1 || { echo "pytest failed"; grep -E "FAILED|Error|assert" $O/pytest_gpu.log | head -20; tail -20 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 400 python bench.py > $O/bench_pg.json 2> $O/bench_pg.err || { echo "bench pg failed"; tail -20 $O/bench_pg.err; exit 1; }
cat $O/bench_pg.json
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu > $O/bench_pg_d20.json 2> $O/bench_pg_d20.err || { echo "bench d20 failed"; tail -20 $O/bench_pg_d20.err; exit 1; }
cat $O/bench_pg_d20.json
timeout -k 10 300 python bench.py --act per_token --no-cpu > $O/bench_pt.json 2> $O/bench_pt.err || { echo "bench pt failed"; tail -20 $O/bench_pt.err; exit 1; }
cat $O/bench_pt.json
timeout -k 10 300 python bench.py --dtype fp32 --no-cpu --steps 100 --warmup 100 > $O/bench_fp32.json 2> $O/bench_fp32.err || { echo "bench fp32 failed"; tail -20 $O/bench_fp32.err; exit 1; }
cat $O/bench_fp32.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python $R/bench.py --no-cpu > $O/prof.log 2>&1 || { echo "rocprof failed"; tail -30 $O/prof.log; exit 1; }
echo prof ok
