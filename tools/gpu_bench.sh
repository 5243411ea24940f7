# Bench + rocprofv3 kernel-trace summary on the GPU box (results -> gpurun_out/).
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
timeout -k 10 400 python bench.py > gpurun_out/bench_pg.json 2> gpurun_out/bench_pg.err || { echo "bench pg failed"; tail -20 gpurun_out/bench_pg.err; exit 1; }
cat gpurun_out/bench_pg.json
timeout -k 10 300 python bench.py --act per_token --no-cpu > gpurun_out/bench_pt.json 2> gpurun_out/bench_pt.err || { echo "bench pt failed"; tail -20 gpurun_out/bench_pt.err; exit 1; }
cat gpurun_out/bench_pt.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_pg -o run -- python $R/bench.py --no-cpu --steps 20 > $R/gpurun_out/prof_pg.log 2>&1 || { echo "rocprof failed"; tail -30 $R/gpurun_out/prof_pg.log; exit 1; }
find $R/gpurun_out/prof_pg -name "*stats*" | head
for f in $(find $R/gpurun_out/prof_pg -name "*kernel_stats.csv"); do head -20 $f; done
