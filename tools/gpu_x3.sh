# x3 (fp32 on the bf16 MFMA): parity tests, fp32 layer tests, OPT fp32 per-linear shapes.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/x3
O=gpurun_out/x3
timeout -k 10 300 python -u -m pytest tests/test_gpu_x3.py -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest_x3.log 2>&1 || { echo "x3 tests failed"; grep -E "FAILED|Error|assert" $O/pytest_x3.log | head -30; tail -30 $O/pytest_x3.log; exit 1; }
tail -3 $O/pytest_x3.log
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -k "fp32 or config or golden or models" --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest_f32.log 2>&1 || { echo "fp32 tests failed"; grep -E "FAILED|Error|assert" $O/pytest_f32.log | head -30; tail -30 $O/pytest_f32.log; exit 1; }
tail -3 $O/pytest_f32.log
timeout -k 10 200 python tools/model_shapes.py opt-1.3b 2048 fp32 > $O/shapes_opt32.txt 2>&1 || { tail -20 $O/shapes_opt32.txt; exit 1; }
cat $O/shapes_opt32.txt
