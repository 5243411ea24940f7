set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/settle
for v in 300 0 300 0; do
  timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu --settle-ms $v > gpurun_out/settle/b_$v.json || exit 1
  python -c "import json;d=json.load(open('gpurun_out/settle/b_$v.json'));print('settle=$v', d['value'], d['ms_per_step'], d['roofline']['avg_ms'])"
done
timeout -k 10 200 python bench.py --act per_token --no-cpu > gpurun_out/settle/pt.json || exit 1
python -c "import json;d=json.load(open('gpurun_out/settle/pt.json'));print('pt', d['value'], d['ms_per_step'], d['config']['kernel'], d['roofline']['avg_ms'])"
