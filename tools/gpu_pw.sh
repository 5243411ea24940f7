# perm_weight variants (kernel time from rocprof, prepass only)
set -o pipefail
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
for v in "2 0" "2 1"; do set -- $v
SQMP_PW_RB=$1 SQMP_PW_DIRECT=$2 timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/pw/v$1$2 -o run -- python $R/tools/gemm_only.py fqt 40 per_group prepass > $R/gpurun_out/pw_v.log 2>&1 || { echo "prof failed"; exit 1; }
python - $1$2 <<'PY'
import csv, sys
for r in csv.DictReader(open(f'/root/repo/gpurun_out/pw/v{sys.argv[1]}/run_kernel_stats.csv')):
    if 'perm_weight' in r['Name']:
        print('v', sys.argv[1], r['Name'][:60], r['Calls'], round(float(r['AverageNs'])/1000, 1))
PY
done
cd $R && SQMP_PW_DIRECT=1 timeout -k 10 200 python -u -m pytest tests/test_gpu_fqt.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "operands" 2>&1 | tail -1
