# Interleaved A/B of two builds of the library (ab_tmp/lib_<a|b>.so, built on the CPU side)
# on the GEMM timing matrix: LIBS="old new" (default), two rounds.
set -o pipefail
cd $GRAFT_REPO_ROOT
L=smoothquant-mixedprecision_amd/smoothquant/libsqmp_w4a4.so
cp $L ab_tmp/lib_keep.so
for rep in 1 2; do
for v in ${LIBS:-old new}; do
  echo "== $v (rep $rep)"
  cp ab_tmp/lib_$v.so $L
  (cd tools && timeout -k 10 300 python gemm_matrix.py) || { cp ab_tmp/lib_keep.so $L; exit 1; }
done
done
cp ab_tmp/lib_keep.so $L
