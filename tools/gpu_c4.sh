# fused C4 prepass: quantizer workgroups per CU sweep (kernel time from rocprof)
set -o pipefail
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
for v in 8 6 4 3 2; do
SQMP_C4_QPERCU=$v timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/c4/q$v -o run -- python $R/tools/gemm_only.py fqt 60 per_group prepass > $R/gpurun_out/c4_q.log 2>&1 || { echo "prof failed"; exit 1; }
python - $v <<'PY'
import csv, sys
for r in csv.DictReader(open(f'/root/repo/gpurun_out/c4/q{sys.argv[1]}/run_kernel_stats.csv')):
    if 'fused' in r['Name'] or 'gemm' in r['Name']:
        print('qpercu', sys.argv[1], r['Name'][:40], r['Calls'], round(float(r['AverageNs'])/1000, 1), round(float(r['MinNs'])/1000, 1))
PY
done
