# A/B: raster group size (M-tiles per group) for the fq6 and f8v2 GEMMs; e2e Llama per_token
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=$R/gpurun_out/r2d; mkdir -p $O
for rep in 1 2; do
for g in 1 2 4 8; do
SQMP_GROUP_M=$g timeout -k 10 60 python tools/gemm_time.py fq 200 | sed "s/^/gm=$g /" || exit 1
SQMP_GROUP_M=$g timeout -k 10 60 python tools/gemm_time.py f8 200 | sed "s/^/gm=$g /" || exit 1
done
done
timeout -k 10 400 python bench_e2e.py --model llama2-7b --windows 4 --act per_token --group 128 --no-cpu > $O/e2e_llama_pt.json 2> $O/e2e_llama_pt.err || { echo "llama pt failed"; tail -20 $O/e2e_llama_pt.err; exit 1; }
cat $O/e2e_llama_pt.json
