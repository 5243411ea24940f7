# Counter passes for the GEMM kernels (separate --pmc passes, kernel-trace only).
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/pmc
cd /tmp && export TMPDIR=/tmp
rocprofv3 -L > $R/gpurun_out/pmc/counters_list.txt 2>&1 || true
run() {  # name, counters...
  local name=$1; shift
  timeout -k 10 240 rocprofv3 --pmc "$@" --output-format csv -d $R/gpurun_out/pmc/$name -o run -- python $R/tools/gemm_only.py ${KIND:-fq} 20 > $R/gpurun_out/pmc/$name.log 2>&1 || { echo "pmc $name failed"; tail -5 $R/gpurun_out/pmc/$name.log; return 1; }
}
P=${PASSES:-fq_a fq_b fq_c fq_d i8_a i8_b i8_c}
for name in $P; do
  case $name in
    *_a) C="SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT" ;;
    *_b) C="SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE" ;;
    *_c) C="FETCH_SIZE" ;;
    *_d) C="WRITE_SIZE TCC_HIT_sum TCC_MISS_sum" ;;
    *_e) C="SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM SQ_BUSY_CU_CYCLES" ;;
  esac
  KIND=${name%%_*} run $name $C || exit 1
done
for d in $R/gpurun_out/pmc/*/; do f=$(ls $d/*counter_collection.csv 2>/dev/null | head -1); [ -n "$f" ] && echo "== $d" && python - "$f" <<'PY'
import csv, sys, collections
rows = list(csv.DictReader(open(sys.argv[1])))
agg = collections.defaultdict(list)
for r in rows:
    if "gemm" in r.get("Kernel_Name", ""):
        agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, v in agg.items():
    print(f"{k:32s} mean/dispatch {sum(v)/len(v):.4g}  (n={len(v)})")
PY
done
