# Interleaved GEMM timing of env-selected variants: ENVS="SQMP_FQ6_PRIO=0 SQMP_FQ6_WM=2" bash tools/gpu_env_ab.sh
set -o pipefail
cd $GRAFT_REPO_ROOT/tools
for rep in 1 2; do
for e in ${ENVS:-X=0}; do
  env $e timeout -k 10 120 python gemm_time.py ${KIND:-fq} 50 | sed "s/^/$e /" || exit 1
done
done
