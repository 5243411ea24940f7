set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
TAG=r5f bash tools/gpu.sh trace:tools/layer_trace.py:30 py:tools/knob_ab.py:h2,SQMP_H2D_GROUP_M,4/8/2/16,3,60 || exit 1
python tools/layer_trace.py --parse gpurun_out/r5f/kernel_trace_layer_trace.csv > gpurun_out/r5f/llama_layer_trace.txt || exit 1
cat gpurun_out/r5f/llama_layer_trace.txt
export TMPDIR=/tmp
for g in 4 8; do
  for c in FETCH_SIZE "WRITE_SIZE TCC_HIT_sum TCC_MISS_sum"; do
    tagc=$(echo $c | cut -c1-5)
    (cd /tmp && SQMP_H2D_GROUP_M=$g timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d "$R/gpurun_out/r5f/pmc_h2d_g${g}_$tagc" -o run -- python "$R/tools/gemm_only.py" h2 20 > "$R/gpurun_out/r5f/pmc_h2d_g${g}_$tagc.log" 2>&1) || exit 1
  done
done
echo pmc ok
