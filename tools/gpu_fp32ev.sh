set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/round gpurun_out/e2e
timeout -k 10 300 python bench.py --dtype fp32 --no-cpu --steps 100 --warmup 100 > gpurun_out/round/bench_fp32.json 2> gpurun_out/round/bench_fp32.err || { tail -20 gpurun_out/round/bench_fp32.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/round/bench_fp32.json'));print(d['value'],d['roofline']['avg_ms'],d['roofline']['achieved'])"
MODELS=opt-1.3b E2E_ARGS="--windows 40" bash tools/gpu_e2e.sh || exit 1
