# Round evidence, part B: end-to-end benches (configs 3 and 4) and PMC passes of the fp32
# GEMM (sqmp_gemm_h2).  Results -> gpurun_out/e2e, gpurun_out/pmc.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
bash tools/gpu_e2e.sh || exit 1
PASSES="h2_a h2_b h2_c h2_d" bash tools/gpu_pmc.sh > gpurun_out/pmc_h2.txt 2>&1 || { echo "pmc failed"; tail -20 gpurun_out/pmc_h2.txt; exit 1; }
tail -30 gpurun_out/pmc_h2.txt
