set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/lcab
timeout -k 10 300 python -u -m pytest tests/test_gpu_quant_act.py tests/test_gpu_parity.py tests/test_gpu_sweep.py tests/test_gpu_configs.py tests/test_gpu_models.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/lcab/pytest.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error|assert" gpurun_out/lcab/pytest.log | head; tail -20 gpurun_out/lcab/pytest.log; exit 1; }
tail -1 gpurun_out/lcab/pytest.log
for v in 0 1 0 1; do
  echo "SQMP_LC_RPL8=$v"
  SQMP_LC_RPL8=$v timeout -k 10 200 python tools/model_shapes.py llama2-7b 2048 fp16 2>&1 | grep -v amdgpu.ids || exit 1
done
