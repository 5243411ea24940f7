# Full GPU suite, then the OPT fp32 / Llama fp16 per-linear shapes.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/x3
O=gpurun_out/x3
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1 || { echo "gpu tests failed"; grep -E "FAILED|Error|assert" $O/pytest_gpu.log | head -30; tail -30 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
timeout -k 10 200 python tools/model_shapes.py opt-1.3b 2048 fp32 > $O/shapes_opt32.txt 2>&1 || { tail -20 $O/shapes_opt32.txt; exit 1; }
cat $O/shapes_opt32.txt
