# bench per_token (f8 v2) + a kernel trace of a short Llama e2e run (host gaps vs GPU busy)
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=$R/gpurun_out/r2c; mkdir -p $O
timeout -k 10 300 python bench.py --act per_token --no-cpu > $O/bench_pt.json 2> $O/bench_pt.err || { echo "bench pt failed"; tail -20 $O/bench_pt.err; exit 1; }
cat $O/bench_pt.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/prof_llama -o run -- python $R/bench_e2e.py --model llama2-7b --layers 4 --windows 2 --no-ref --no-cpu > $O/prof_llama.log 2>&1 || { echo "rocprof failed"; tail -30 $O/prof_llama.log; exit 1; }
tail -2 $O/prof_llama.log
