# Interleaved A/B of two library builds (ab_tmp/lib_<v>.so) on an arbitrary command: CMD.
set -o pipefail
cd $GRAFT_REPO_ROOT
L=smoothquant-mixedprecision_amd/smoothquant/libsqmp_w4a4.so
cp $L ab_tmp/lib_keep.so
for rep in 1 2; do
for v in ${LIBS:-old new}; do
  echo "== $v (rep $rep)"
  cp ab_tmp/lib_$v.so $L
  timeout -k 10 300 bash -c "$CMD" || { cp ab_tmp/lib_keep.so $L; exit 1; }
done
done
cp ab_tmp/lib_keep.so $L
