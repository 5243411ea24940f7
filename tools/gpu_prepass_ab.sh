# Prepass A/B: GPU tests, then per-linear timings with and without an env knob
# (AB="SQMP_RANK_TABLE_OFF=1" by default).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
TESTS="${TESTS:-tests/test_gpu_quant_act.py}" bash tools/gpu_tests.sh || exit 1
for m in ${MODELS:-opt-1.3b llama2-7b}; do
  echo "== $m"; timeout -k 10 300 python tools/model_shapes.py $m || exit 1
  echo "== $m ${AB:-SQMP_RANK_TABLE_OFF=1}"; env ${AB:-SQMP_RANK_TABLE_OFF=1} timeout -k 10 300 python tools/model_shapes.py $m || exit 1
done
