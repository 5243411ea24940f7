# Round evidence: bench lines (both act modes), rocprofv3 kernel stats of the bench, the
# end-to-end benches (configs 3 and 4) and the config-5 sweep.  Results -> gpurun_out/.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out/round
O=$R/gpurun_out/round
timeout -k 10 400 python bench.py > $O/bench_pg.json 2> $O/bench_pg.err || { echo "bench pg failed"; tail -20 $O/bench_pg.err; exit 1; }
cat $O/bench_pg.json
timeout -k 10 300 python bench.py --act per_token --no-cpu > $O/bench_pt.json 2> $O/bench_pt.err || { echo "bench pt failed"; tail -20 $O/bench_pt.err; exit 1; }
cat $O/bench_pt.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python $R/bench.py --no-cpu > $O/prof.log 2>&1 || { echo "rocprof failed"; tail -30 $O/prof.log; exit 1; }
cd $R
timeout -k 10 400 python bench_e2e.py --model llama2-7b > $O/e2e_llama.json 2> $O/e2e_llama.err || { echo "llama failed"; tail -20 $O/e2e_llama.err; exit 1; }
cat $O/e2e_llama.json
timeout -k 10 400 python bench_e2e.py --model opt-1.3b > $O/e2e_opt.json 2> $O/e2e_opt.err || { echo "opt failed"; tail -20 $O/e2e_opt.err; exit 1; }
cat $O/e2e_opt.json
if [ -n "$SWEEP" ]; then
timeout -k 10 900 python bench_sweep.py $SWEEP_ARGS > $O/sweep.jsonl 2> $O/sweep.err || { echo "sweep failed"; tail -20 $O/sweep.err; exit 1; }
tail -3 $O/sweep.jsonl
fi
