# Kernel trace + counters of the activation quantizer alone.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/ppmc
cd /tmp && export TMPDIR=/tmp
for cfg in "16384 4096 128 per_group" "2048 4096 64 per_group" "2048 11008 64 per_group"; do
  tag=$(echo $cfg | tr ' ' '_')
  timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/ppmc/kt_$tag -o run -- python $R/tools/prepass_only.py $cfg 20 > $R/gpurun_out/ppmc/kt_$tag.log 2>&1 || { tail -5 $R/gpurun_out/ppmc/kt_$tag.log; exit 1; }
  timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU --output-format csv -d $R/gpurun_out/ppmc/a_$tag -o run -- python $R/tools/prepass_only.py $cfg 5 > $R/gpurun_out/ppmc/a_$tag.log 2>&1 || { tail -5 $R/gpurun_out/ppmc/a_$tag.log; exit 1; }
  timeout -s KILL 90 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM GRBM_GUI_ACTIVE --output-format csv -d $R/gpurun_out/ppmc/b_$tag -o run -- python $R/tools/prepass_only.py $cfg 5 > $R/gpurun_out/ppmc/b_$tag.log 2>&1 || { tail -5 $R/gpurun_out/ppmc/b_$tag.log; exit 1; }
done
python - <<'PY'
import csv, glob, os, collections
R = os.environ["GRAFT_REPO_ROOT"] + "/gpurun_out/ppmc"
for d in sorted(glob.glob(R + "/kt_*")):
    if not os.path.isdir(d): continue
    f = glob.glob(d + "/**/*kernel_stats.csv", recursive=True)[0]
    print("==", os.path.basename(d))
    for r in csv.DictReader(open(f)):
        if "sqmp" in r["Name"] or "fill" in r["Name"]:
            print(f"   {r['Name'][:60]:60s} calls={r['Calls']:>4s} avg_us={float(r['AverageNs'])/1e3:8.1f}")
for d in sorted(glob.glob(R + "/[ab]_*")):
    if not os.path.isdir(d): continue
    f = glob.glob(d + "/**/*counter_collection.csv", recursive=True)
    if not f: continue
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for r in csv.DictReader(open(f[0])):
        agg[r["Kernel_Name"][:40]][r["Counter_Name"]].append(float(r["Counter_Value"]))
    print("==", os.path.basename(d))
    for k, cs in agg.items():
        if "sqmp" not in k: continue
        print("  ", k, " ".join(f"{c}={sum(v)/len(v):.4g}" for c, v in cs.items()))
PY
