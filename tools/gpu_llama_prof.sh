# Llama-shape per-linear timing, host overhead, and kernel stats of a short Llama run.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out/llprof
timeout -k 10 300 python tools/llama_shapes.py > gpurun_out/llprof/shapes.txt 2>&1 || { tail -20 gpurun_out/llprof/shapes.txt; exit 1; }
cat gpurun_out/llprof/shapes.txt
timeout -k 10 300 python tools/host_overhead.py > gpurun_out/llprof/host.txt 2>&1 || { tail -20 gpurun_out/llprof/host.txt; exit 1; }
cat gpurun_out/llprof/host.txt
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/llprof/ks -o run -- python $R/bench_llama.py --layers 8 --windows 2 > $R/gpurun_out/llprof/ks.log 2>&1 || { tail -20 $R/gpurun_out/llprof/ks.log; exit 1; }
python - <<'PY'
import csv, glob, os
R = os.environ["GRAFT_REPO_ROOT"] + "/gpurun_out/llprof/ks"
f = glob.glob(R + "/**/*kernel_stats.csv", recursive=True)[0]
for r in list(csv.DictReader(open(f)))[:30]:
    print(f"{r['Name'][:90]:90s} calls={r['Calls']:>5s} avg_us={float(r['AverageNs'])/1e3:9.1f} pct={r['Percentage']}")
PY
