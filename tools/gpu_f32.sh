# fp32 generic GEMM: parity tests (every fp32 case), then OPT-1.3B fp32 per-linear timings (8-wave vs 4-wave)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/f32; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider -k "fp32 or f32 or config or model" > $O/pytest.log 2>&1 || { echo "pytest failed"; grep -E "FAILED|Error|assert" $O/pytest.log | head -20; tail -5 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 150 python tools/model_shapes.py opt-1.3b 2048 fp32 || exit 1
SQMP_F32_WN2=1 timeout -k 10 150 python tools/model_shapes.py opt-1.3b 2048 fp32 || exit 1
