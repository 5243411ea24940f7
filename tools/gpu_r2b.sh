# Round-2 evidence: e2e configs 3 (OPT-1.3B fp32) and 4 (Llama-2-7B fp16) with CPU
# baselines; rocprofv3 kernel trace of the driver-shaped bench; PMC passes for fq and f8.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=$R/gpurun_out/r2b
mkdir -p $O
timeout -k 10 400 python bench_e2e.py --model opt-1.3b --windows 4 > $O/e2e_opt.json 2> $O/e2e_opt.err || { echo "opt failed"; tail -20 $O/e2e_opt.err; exit 1; }
cat $O/e2e_opt.json
timeout -k 10 400 python bench_e2e.py --model llama2-7b --windows 4 > $O/e2e_llama.json 2> $O/e2e_llama.err || { echo "llama failed"; tail -20 $O/e2e_llama.err; exit 1; }
cat $O/e2e_llama.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_driver -o run -- python $R/bench.py --steps 20 --warmup 5 --no-cpu > $O/prof_driver.log 2>&1 || { echo "rocprof failed"; tail -30 $O/prof_driver.log; exit 1; }
cd $R
PASSES="fq_a fq_b fq_c fq_d f8_a f8_b f8_c f8_d" bash tools/gpu_pmc.sh > $O/pmc.txt 2>&1 || { echo "pmc failed"; tail -30 $O/pmc.txt; exit 1; }
cp -r gpurun_out/pmc $O/ 2>/dev/null
tail -60 $O/pmc.txt
