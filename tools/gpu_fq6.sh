# Parity (GEMM-touching tests) under fq5 (default) and fq6, then GEMM timing of both.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for v in wm1 fq6; do
  SQMP_FQ_VARIANT=$v timeout -k 10 600 python -m pytest tests -m gpu -q --maxfail=5 -p no:cacheprovider > gpurun_out/pytest_$v.log 2>&1
  rc=$?
  tail -3 gpurun_out/pytest_$v.log
  [ $rc -ne 0 ] && { echo "tests failed ($v)"; grep -E "^(FAILED|ERROR)|differ" gpurun_out/pytest_$v.log | head -20; exit $rc; }
done
VARIANTS="wm1 fq6 wm1 fq6" bash tools/gpu_variants.sh
