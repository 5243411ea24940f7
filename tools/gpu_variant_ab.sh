# A/B of GEMM variants selected by an env var, interleaved: VAR=name VALS="a b c" (gemm_matrix per value, twice).
set -o pipefail
cd $GRAFT_REPO_ROOT/tools
for rep in 1 2; do
for v in $VALS; do
  echo "== $VAR=$v (rep $rep)"
  env $VAR=$v timeout -k 10 300 python gemm_matrix.py || exit 1
done
done
