# End-to-end benches: config 4 (Llama-2-7B), config 3 (OPT-1.3B), config 5 sweep.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python bench_e2e.py --model llama2-7b > gpurun_out/e2e_llama.json 2> gpurun_out/e2e_llama.err || { echo "llama failed"; tail -20 gpurun_out/e2e_llama.err; exit 1; }
cat gpurun_out/e2e_llama.json
timeout -k 10 400 python bench_e2e.py --model opt-1.3b > gpurun_out/e2e_opt.json 2> gpurun_out/e2e_opt.err || { echo "opt failed"; tail -20 gpurun_out/e2e_opt.err; exit 1; }
cat gpurun_out/e2e_opt.json
if [ -n "$SWEEP" ]; then
timeout -k 10 900 python bench_sweep.py $SWEEP_ARGS > gpurun_out/sweep.jsonl 2> gpurun_out/sweep.err || { echo "sweep failed"; tail -20 gpurun_out/sweep.err; exit 1; }
cat gpurun_out/sweep.jsonl
fi
