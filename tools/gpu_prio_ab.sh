# Interleaved GEMM timing of fq6 PRIO variants (diagnostics / tuning): VALS="0 12" bash tools/gpu_prio_ab.sh
set -o pipefail
cd $GRAFT_REPO_ROOT/tools
for rep in 1 2; do
for v in ${VALS:-0}; do
  SQMP_FQ6_PRIO=$v timeout -k 10 120 python gemm_time.py ${KIND:-fq} 50 | sed "s/^/prio=$v /" || exit 1
done
done
