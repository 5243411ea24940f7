set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/h2ab
timeout -k 10 300 python -u -m pytest tests/test_gpu_x3.py tests/test_gpu_configs.py tests/test_gpu_parity.py tests/test_gpu_quant_act.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/h2ab/pytest.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error|assert" gpurun_out/h2ab/pytest.log | head; tail -20 gpurun_out/h2ab/pytest.log; exit 1; }
tail -1 gpurun_out/h2ab/pytest.log
for v in 0 1 0 1; do
  echo "SQMP_H2_BK64=$v"
  SQMP_H2_BK64=$v timeout -k 10 200 python tools/model_shapes.py opt-1.3b 2048 fp32 2>&1 | grep -v amdgpu.ids || exit 1
  SQMP_H2_BK64=$v timeout -k 10 200 python bench.py --dtype fp32 --no-cpu --steps 100 --warmup 100 > gpurun_out/h2ab/bench_fp32_$v.json || exit 1
  python -c "import json;d=json.load(open('gpurun_out/h2ab/bench_fp32_$v.json'));print(d['value'],d['roofline']['avg_ms'],d['roofline']['achieved'])"
done
