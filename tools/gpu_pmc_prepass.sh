# Counter passes for the activation-quantization kernels (kernel trace + one PMC group per pass).
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/pmcq
cd /tmp && export TMPDIR=/tmp
run() {
  local name=$1; shift
  timeout -k 10 240 rocprofv3 --kernel-trace --pmc "$@" --output-format csv -d $R/gpurun_out/pmcq/$name -o run -- python $R/tools/gemm_only.py ${KIND:-fq} 5 prepass > $R/gpurun_out/pmcq/$name.log 2>&1 || { echo "pmc $name failed"; tail -5 $R/gpurun_out/pmcq/$name.log; return 1; }
}
run a SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_LDS_IDX_ACTIVE && \
run b SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE && \
run c FETCH_SIZE WRITE_SIZE
python - <<'PY'
import csv, glob, os, collections
R = os.environ["GRAFT_REPO_ROOT"] + "/gpurun_out/pmcq"
for d in sorted(glob.glob(R + "/*/")):
    cc = glob.glob(d + "*counter_collection.csv"); kt = glob.glob(d + "*kernel_trace.csv")
    if not cc: continue
    durs = collections.defaultdict(list)
    for r in csv.DictReader(open(kt[0])):
        durs[r["Kernel_Name"][:40]].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for r in csv.DictReader(open(cc[0])):
        agg[r["Kernel_Name"][:40]][r["Counter_Name"]].append(float(r["Counter_Value"]))
    print("==", os.path.basename(d.rstrip("/")))
    for k, cs in agg.items():
        if "sqmp" not in k: continue
        dd = durs.get(k, [0])
        print(f"  {k:40s} {sum(dd)/len(dd)/1e3:8.1f} us  " + "  ".join(f"{c}={sum(v)/len(v):.4g}" for c, v in cs.items()))
PY
