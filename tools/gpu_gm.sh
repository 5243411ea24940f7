set -o pipefail
cd $GRAFT_REPO_ROOT
for v in 4 1 2 8 16 4; do
  SQMP_GROUP_M=$v timeout -k 10 200 python tools/gemm_ab.py "GM=$v" || exit 1
done
