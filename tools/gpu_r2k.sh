# Round-2 evidence for the activation-order path: bench (per_group, default = fqt), rocprof
# kernel stats of the bench, PMC passes of the fqt GEMM.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=$R/gpurun_out/r2k; mkdir -p $O
timeout -k 10 400 python bench.py > $O/bench_pg.json 2> $O/bench_pg.err || { echo "bench failed"; tail -20 $O/bench_pg.err; exit 1; }
cat $O/bench_pg.json
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu > $O/bench_pg_d20.json 2> $O/bench_pg_d20.err || { echo "bench d20 failed"; tail -20 $O/bench_pg_d20.err; exit 1; }
cat $O/bench_pg_d20.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python $R/bench.py --no-cpu > $O/prof.log 2>&1 || { echo "rocprof failed"; tail -30 $O/prof.log; exit 1; }
cd $R
PASSES="fqt_a fqt_b fqt_c fqt_d" bash tools/gpu_pmc.sh > $O/pmc.txt 2>&1 || { echo "pmc failed"; tail -20 $O/pmc.txt; exit 1; }
tail -40 $O/pmc.txt
