set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/fqtab
for v in 1 0 1 0; do
  SQMP_FQT=$v timeout -k 10 200 python bench.py --no-cpu --steps 100 --warmup 100 > gpurun_out/fqtab/b_$v.json || exit 1
  python -c "import json;d=json.load(open('gpurun_out/fqtab/b_$v.json'));print('FQT=$v', d['value'], d['ms_per_step'], d['config']['kernel'], d['roofline']['avg_ms'], d['prepass']['avg_ms'])"
done
