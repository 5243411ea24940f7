# Kernel durations (rocprofv3 kernel trace) of tools/model_shapes.py: MODEL (opt-1.3b),
# optional ENV="VAR=1" for an A/B leg.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/shp
cd /tmp && export TMPDIR=/tmp
for leg in base ${ENVB:+alt}; do
  if [ $leg = alt ]; then export $ENVB; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/shp/$leg -o run -- python $R/tools/model_shapes.py ${MODEL:-opt-1.3b} > $R/gpurun_out/shp/$leg.log 2>&1 || { tail -20 $R/gpurun_out/shp/$leg.log; exit 1; }
  python - "$R/gpurun_out/shp/$leg" <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True)[0]
print("==", sys.argv[1].split("/")[-1])
for r in list(csv.DictReader(open(f)))[:30]:
    print(f"  {r['Name'][:100]:100s} calls={r['Calls']:>6s} avg_us={float(r['AverageNs'])/1e3:8.2f} min_us={float(r['MinNs'])/1e3:8.2f}")
PY
done
