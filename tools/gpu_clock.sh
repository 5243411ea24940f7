# Effective clock of the fq GEMM: kernel trace + GRBM_GUI_ACTIVE in one pass (no sys/runtime
# trace).  clock = GRBM_GUI_ACTIVE / 8 / kernel duration (MI355X_MICROARCH.md, DVFS give-back).
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/clk
cd /tmp && export TMPDIR=/tmp
# ENVS="SQMP_FQ6_PRIO=0 SQMP_FQ6_PRIO=5": one pass per env assignment
for v in ${ENVS:-SQMP_FQ6_PRIO=0}; do
  env $v timeout -k 10 240 rocprofv3 --kernel-trace --pmc GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES --output-format csv -d $R/gpurun_out/clk/$v -o run -- python $R/tools/gemm_only.py fq 20 > $R/gpurun_out/clk/$v.log 2>&1 || { echo "clock $v failed"; tail -5 $R/gpurun_out/clk/$v.log; exit 1; }
done
python - <<'PY'
import csv, glob, os, collections
R = os.environ["GRAFT_REPO_ROOT"] + "/gpurun_out/clk"
for d in sorted(glob.glob(R + "/*/")):
    kt = glob.glob(d + "*kernel_trace.csv")
    cc = glob.glob(d + "*counter_collection.csv")
    if not kt or not cc:
        print(d, "missing csv"); continue
    dur = [int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in csv.DictReader(open(kt[0])) if "gemm" in r["Kernel_Name"]]
    agg = collections.defaultdict(list)
    for r in csv.DictReader(open(cc[0])):
        if "gemm" in r.get("Kernel_Name", ""):
            agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
    ns = sum(dur) / len(dur)
    g = sum(agg["GRBM_GUI_ACTIVE"]) / len(agg["GRBM_GUI_ACTIVE"])
    mb = sum(agg["SQ_VALU_MFMA_BUSY_CYCLES"]) / len(agg["SQ_VALU_MFMA_BUSY_CYCLES"])
    cyc = g / 8
    print(f"{os.path.basename(d.rstrip('/'))}: kernel {ns/1e3:.1f} us, clock {cyc/ns:.3f} GHz, MFMA busy {mb/(1024*cyc):.3f}")
PY
