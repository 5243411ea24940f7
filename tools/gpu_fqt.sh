# activation-order path: parity tests, then config-2 GEMM timings fqt vs fq
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/fqt; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_fqt.py -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 || { echo "pytest failed"; grep -E "FAILED|Error|assert" $O/pytest.log | head -20; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 60 python tools/gemm_time.py fqt 300 || exit 1
timeout -k 10 60 python tools/gemm_time.py fq 300 || exit 1
for g in 1 8 16; do echo -n "group_m=$g "; SQMP_GROUP_M=$g timeout -k 10 60 python tools/gemm_time.py fqt 300 || exit 1; done
timeout -k 10 300 python bench.py --no-cpu --steps 100 --warmup 100 > gpurun_out/fqt/bench.json 2> gpurun_out/fqt/bench.err || { echo "bench failed"; tail -5 gpurun_out/fqt/bench.err; exit 1; }
python -c "import json; d=json.loads(open('gpurun_out/fqt/bench.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['roofline']['avg_ms'], d['prepass'])"
cd /tmp && export TMPDIR=/tmp && timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/fqt/prof -o run -- python $GRAFT_REPO_ROOT/tools/gemm_only.py fqt 20 per_group prepass > $GRAFT_REPO_ROOT/gpurun_out/fqt/prof.log 2>&1 || { echo "prof failed"; exit 1; }
python - <<'PY'
import csv
for r in csv.DictReader(open('/root/repo/gpurun_out/fqt/prof/run_kernel_stats.csv')):
    print(r['Name'][:60], r['Calls'], round(float(r['AverageNs'])/1000, 1))
PY
