# Kernel-trace stats of a command's kernels (default: GEMM + prepass loop).
set -o pipefail
R=$GRAFT_REPO_ROOT
NAME=${NAME:-kstats}
mkdir -p $R/gpurun_out/$NAME
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/$NAME -o run -- python $R/tools/gemm_only.py ${KIND:-fq} 20 prepass > $R/gpurun_out/$NAME/log.txt 2>&1 || { tail -5 $R/gpurun_out/$NAME/log.txt; exit 1; }
python - <<'PY'
import csv, glob, os
R = os.environ["GRAFT_REPO_ROOT"] + "/gpurun_out/" + os.environ.get("NAME", "kstats")
f = glob.glob(R + "/*kernel_stats.csv")[0]
for r in csv.DictReader(open(f)):
    print(f"{r['Name'][:70]:70s} calls={r['Calls']:>4s} avg_us={float(r['AverageNs'])/1e3:9.1f}")
PY
