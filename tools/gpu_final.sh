# Final-tree evidence refresh for the fq7 default: smoke, Llama e2e (8 and 40 windows),
# config-5 sweep.  Results -> gpurun_out/{round,e2e,final}.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out/final
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/final/smoke.log 2>&1 || { echo "smoke failed"; tail -20 gpurun_out/final/smoke.log; exit 1; }
tail -1 gpurun_out/final/smoke.log
timeout -k 10 500 python bench_e2e.py --model llama2-7b --windows 40 > gpurun_out/final/e2e40_llama.json 2> gpurun_out/final/e2e40_llama.err || { echo "llama40 failed"; tail -20 gpurun_out/final/e2e40_llama.err; exit 1; }
cut -c1-300 gpurun_out/final/e2e40_llama.json
timeout -k 10 900 python bench_sweep.py > gpurun_out/final/sweep.jsonl 2> gpurun_out/final/sweep.err || { echo "sweep failed"; tail -20 gpurun_out/final/sweep.err; exit 1; }
tail -1 gpurun_out/final/sweep.jsonl
