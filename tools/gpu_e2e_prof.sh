# Kernel-time breakdown of the W4A4 end-to-end runs (fp16 leg + W4A4 leg, no reference legs).
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/e2eprof
cd /tmp && export TMPDIR=/tmp
for m in ${MODELS:-llama2-7b opt-1.3b}; do
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/e2eprof/$m -o run -- python $R/bench_e2e.py --model $m --windows 2 --no-ref > $R/gpurun_out/e2eprof/$m.log 2>&1 || { tail -20 $R/gpurun_out/e2eprof/$m.log; exit 1; }
python - "$R/gpurun_out/e2eprof/$m" <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True)[0]
rows = list(csv.DictReader(open(f)))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
print("==", sys.argv[1].split("/")[-1], f"total kernel time {tot/1e6:.1f} ms")
for r in rows[:25]:
    print(f"  {r['Name'][:80]:80s} calls={r['Calls']:>6s} avg_us={float(r['AverageNs'])/1e3:8.1f} tot_ms={float(r['TotalDurationNs'])/1e6:7.2f}")
PY
done
