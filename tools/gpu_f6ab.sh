set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/f6ab
for v in 1 0 1 0; do
  SQMP_F6=$v timeout -k 10 200 python bench.py --act per_token --no-cpu > gpurun_out/f6ab/pt_$v.json || exit 1
  python -c "import json;d=json.load(open('gpurun_out/f6ab/pt_$v.json'));print('F6=$v', d['value'], d['ms_per_step'], d['config']['kernel'], d['roofline']['avg_ms'], d['roofline']['achieved'], d['prepass']['avg_ms'])"
done
