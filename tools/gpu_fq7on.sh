set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/fq7on
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/fq7on/pytest.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error|assert" gpurun_out/fq7on/pytest.log | head -20; tail -20 gpurun_out/fq7on/pytest.log; exit 1; }
tail -1 gpurun_out/fq7on/pytest.log
for v in 1 0; do
  echo "SQMP_FQ7=$v"
  SQMP_FQ7=$v timeout -k 10 200 python tools/model_shapes.py llama2-7b 2048 fp16 2>&1 | grep -v amdgpu.ids || exit 1
done
MODELS=llama2-7b bash tools/gpu_e2e.sh || exit 1
