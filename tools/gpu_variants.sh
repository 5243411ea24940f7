# GEMM-only timing of the fq5 variants (one process each; the variant knob is read once).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for v in ${VARIANTS:-wm1 wm2 pf6 nowait}; do
  SQMP_FQ_VARIANT=$v timeout -k 10 240 python tools/gemm_time.py fq 50 2>gpurun_out/gv_$v.err | tee -a gpurun_out/gemm_variants.txt || { tail -5 gpurun_out/gv_$v.err; exit 1; }
done
