# fq7 timing diagnostics (SQMP_FQ7_DIAG variants, wrong results by design)
set -o pipefail
cd $GRAFT_REPO_ROOT
for d in 0 1 2 3 4 0; do echo -n "diag=$d "; SQMP_FQ7_DIAG=$d timeout -k 10 60 python tools/gemm_time.py fq7 300 || exit 1; done
timeout -k 10 60 python tools/gemm_time.py fq 300 || exit 1
