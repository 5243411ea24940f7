# Round-5 evidence on one box: default bench, rocprof kernel stats of the bench, counter
# profiles (fqt7 per_group, f8 per_token, h2d fp32) of THIS library, the default-build Llama
# layer trace.  gpurun -- bash tools/gpu_r5_final.sh   (results -> gpurun_out/r5final/)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
export TAG=r5final
O="$R/gpurun_out/$TAG"
mkdir -p "$O"
bash tools/gpu.sh bench prof pmc:fqt pmc:f8 pmc:h2 trace:tools/layer_trace.py:30 || exit 1
python tools/layer_trace.py --parse "$O/kernel_trace_layer_trace.csv" > "$O/llama_layer_trace.txt" || exit 1
python tools/pmc_summary.py "$O/pmc" fqt 0 214000000 16 "$O/r05_pmc_gemm_fqt7_per_group.json" gemm_fq7 || exit 1
python tools/pmc_summary.py "$O/pmc" f8 0 237000000 32 "$O/r05_pmc_gemm_f8v2_per_token.json" gemm_f8 || exit 1
python tools/pmc_summary.py "$O/pmc" h2 0 640000000 16 "$O/r05_pmc_gemm_h2d_fp32.json" gemm_h2d || exit 1
tail -3 "$O/llama_layer_trace.txt"
# only the summaries travel back (gpurun merges <= 64 MiB): drop the raw counter / trace dirs
rm -rf "$O/pmc" "$O/prof" "$O/kernel_trace_layer_trace.csv"
du -sh "$O"
echo "final ok"
