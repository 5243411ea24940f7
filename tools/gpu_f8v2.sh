# f8 v2 check: layout probe, f8 tests, A/B timing of the 32x32x64 (v1) and 16x16x128 (v2)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/f8v2; mkdir -p $O
timeout -k 5 60 ./tools/probe/mfma16_f8f6_probe > $O/probe.txt 2>&1 || { echo "probe failed"; cat $O/probe.txt; exit 1; }
cat $O/probe.txt
timeout -k 10 300 python -u -m pytest tests/test_gpu_f8.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for i in 1 2; do
SQMP_F8_V1=1 timeout -k 10 60 python tools/gemm_time.py f8 200 || exit 1
timeout -k 10 60 python tools/gemm_time.py f8 200 || exit 1
done
