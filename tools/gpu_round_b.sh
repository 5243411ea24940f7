# Round evidence, part B: smoke(), end-to-end benches (configs 3 and 4), the config-5 sweep,
# PMC passes of the fp32 GEMM (sqmp_gemm_h2).  Results -> gpurun_out/{e2e,pmc,round}.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out/round
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/round/smoke.log 2>&1 || { echo "smoke failed"; tail -20 gpurun_out/round/smoke.log; exit 1; }
tail -1 gpurun_out/round/smoke.log
bash tools/gpu_e2e.sh || exit 1
timeout -k 10 900 python bench_sweep.py > gpurun_out/round/sweep.jsonl 2> gpurun_out/round/sweep.err || { echo "sweep failed"; tail -20 gpurun_out/round/sweep.err; exit 1; }
tail -2 gpurun_out/round/sweep.jsonl
if [ -n "$PMC" ]; then
PASSES="h2_a h2_b h2_c h2_d" bash tools/gpu_pmc.sh > gpurun_out/pmc_h2.txt 2>&1 || { echo "pmc failed"; tail -20 gpurun_out/pmc_h2.txt; exit 1; }
fi
