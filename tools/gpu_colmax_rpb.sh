# Column-max rows-per-block sweep at config 2 (kernel trace of the quantizer driver).
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/rpb
cd /tmp && export TMPDIR=/tmp
for rpb in ${RPBS:-32 64 128 256 512}; do
  SQMP_COLMAX_RPB=$rpb timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/rpb/$rpb -o run -- python $R/tools/prepass_only.py 16384 4096 128 per_group 300 > $R/gpurun_out/rpb/$rpb.log 2>&1 || { tail -20 $R/gpurun_out/rpb/$rpb.log; exit 1; }
  python - "$R/gpurun_out/rpb/$rpb" $rpb <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    if "colmax" in r["Name"] or "quant_lc" in r["Name"] or "rank_table" in r["Name"]:
        print(f"rpb={sys.argv[2]:>4s} {r['Name'][:40]:40s} avg_us={float(r['AverageNs'])/1e3:8.2f} min_us={float(r['MinNs'])/1e3:8.2f}")
PY
done
