# Kernel stats (avg us) of the GEMM + prepass loop under several env assignments:
# ENVS="SQMP_COLMAX_RPB=128 SQMP_COLMAX_RPB=512" bash tools/gpu_kstats_env.sh
set -o pipefail
for e in ${ENVS:-X=0}; do
  echo "== $e"
  env $e NAME=ks_${e//=/_} bash $GRAFT_REPO_ROOT/tools/gpu_kstats.sh || exit 1
done
