# fqt7 (tile-major activation operands on fq7's structure) vs fqt on fq6: parity + bench A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/fqt7
O=gpurun_out/fqt7
timeout -k 10 300 python -u -m pytest tests/test_gpu_fqt.py -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 || { echo "pytest failed"; grep -E "FAILED|Error|assert" $O/pytest.log | head -30; tail -30 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
for v in 1 0 1 0; do
  SQMP_FQT7=$v timeout -k 10 200 python bench.py --steps 50 --warmup 10 > $O/bench_$v.json 2> $O/bench_$v.err || { echo "bench failed"; tail -20 $O/bench_$v.err; exit 1; }
  python -c "import json;d=json.load(open('$O/bench_$v.json'));print('FQT7=$v', d['value'], d['ms_per_step'], d['roofline']['avg_ms'], d['prepass']['avg_ms'])"
done
