# fqt7 tile-order group size A/B (SQMP_FQT7_GROUP_M) at config 2
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/fqt7gm
O=gpurun_out/fqt7gm
for g in ${GMS:-8 16 4 2 16 8}; do
  SQMP_FQT7_GROUP_M=$g timeout -k 10 200 python bench.py --steps 50 --warmup 10 --no-cpu > $O/b_$g.json 2> $O/b_$g.err || { echo "bench failed"; tail -20 $O/b_$g.err; exit 1; }
  python -c "import json;d=json.load(open('$O/b_$g.json'));print('GM=$g', d['value'], d['ms_per_step'], d['roofline']['avg_ms'])"
done
