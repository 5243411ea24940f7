# same-box A/B of library builds on the act-order prepass (tools/prepass_split.py):
#   bash tools/ab_libs_prepass.sh ROUNDS LIB1 LIB2 ...
set -e
R=$1; shift
for r in $(seq $R); do for L in "$@"; do
  echo "== $L"
  SQMP_LIB_PATH=$L timeout -k 10 120 python tools/prepass_split.py 100 2>&1 | grep -v amdgpu.ids
done; done
