# fused output quant: GPU tests, then OPT-1.3B per-linear timings with and without fusion
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=$R/gpurun_out/r2e; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 || { echo "pytest failed"; grep -E "FAILED|Error|assert" $O/pytest.log | head -30; tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
SQMP_OQ_FUSE=0 timeout -k 10 120 python tools/model_shapes.py opt-1.3b | tail -6 || exit 1
timeout -k 10 120 python tools/model_shapes.py opt-1.3b | tail -6 || exit 1
