set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 200 python tools/gemm_ab.py "fq6" || exit 1
SQMP_FQ7=1 SQMP_FQ7_J=2 timeout -k 10 200 python tools/gemm_ab.py "fq7J2" || exit 1
SQMP_FQ7=1 SQMP_FQ7_J=4 timeout -k 10 200 python tools/gemm_ab.py "fq7J4" || exit 1
timeout -k 10 200 python tools/gemm_ab.py "fq6" || exit 1
