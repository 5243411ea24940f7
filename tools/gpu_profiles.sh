# Round artifacts for profiles/: bench JSON lines (with the CPU baseline), rocprofv3 kernel
# stats of the bench command, PMC HBM traffic of the GEMM (FETCH_SIZE and WRITE_SIZE in
# separate passes; FETCH_SIZE x2 on gfx950, MI355X_MICROARCH.md §HBM).
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/prof
TAG=${TAG:-r01}
mkdir -p $O
cd $R
timeout -k 10 400 python bench.py > $O/${TAG}_bench_per_group.json 2> $O/bench_pg.err || { tail -5 $O/bench_pg.err; exit 1; }
timeout -k 10 400 python bench.py --act per_token > $O/${TAG}_bench_per_token.json 2> $O/bench_pt.err || { tail -5 $O/bench_pt.err; exit 1; }
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/ks -o run -- python $R/bench.py --no-cpu > $O/ks.log 2>&1 || { tail -5 $O/ks.log; exit 1; }
for act in per_group per_token; do
  kind=fq; [ $act = per_token ] && kind=f8   # the kernel W4A4Linear(kernel="auto") runs
  timeout -k 10 240 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d $O/f_$act -o run -- python $R/tools/gemm_only.py $kind 5 $act > $O/f_$act.log 2>&1 || { tail -5 $O/f_$act.log; exit 1; }
  timeout -k 10 240 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d $O/w_$act -o run -- python $R/tools/gemm_only.py $kind 5 $act > $O/w_$act.log 2>&1 || { tail -5 $O/w_$act.log; exit 1; }
done
python - <<'PY'
import csv, glob, json, os, shutil
R = os.environ["GRAFT_REPO_ROOT"]; O = R + "/gpurun_out/prof"; tag = os.environ.get("TAG", "r01")
ks = glob.glob(O + "/ks/*kernel_stats.csv")[0]
shutil.copy(ks, f"{O}/{tag}_bench_kernel_stats.csv")
def counter(d, name):
    f = glob.glob(d + "/*counter_collection.csv")[0]
    v = [float(r["Counter_Value"]) for r in csv.DictReader(open(f)) if "gemm" in r["Kernel_Name"] and r["Counter_Name"] == name]
    kt = glob.glob(d + "/*kernel_trace.csv")[0]
    du = [int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in csv.DictReader(open(kt)) if "gemm" in r["Kernel_Name"]]
    return sum(v) / len(v), sum(du) / len(du)
M, K, N = 16384, 4096, 4096
for act in ("per_group", "per_token"):
    kdt = "f16" if act == "per_group" else "f8"
    fetch_kb, dur = counter(f"{O}/f_{act}", "FETCH_SIZE")
    write_kb, _ = counter(f"{O}/w_{act}", "WRITE_SIZE")
    rd = 2 * fetch_kb * 1024
    wr = write_kb * 1024
    a_bytes = M * (4096 + 448) * 2 if kdt == "f16" else M * 4096 + M * 448 * 2 + M * 4
    b_bytes = 4096 * 2048 if kdt == "f16" else 4096 * 4096
    out = {"kernel": "sqmp::gemm_fq6_kernel<F16,1>" if kdt == "f16" else "sqmp::gemm_f8_kernel<F16>",
           "act": act, "config": "M=16384 K=N=4096 G=128 10% salient",
           "fetch_size_kb_raw": fetch_kb, "write_size_kb": write_kb,
           "hbm_read_bytes_per_launch": rd, "hbm_write_bytes_per_launch": wr,
           "hbm_bytes_per_launch": rd + wr, "profiled_kernel_ns": dur,
           "correction": "FETCH_SIZE x2 on gfx950 (MI355X_MICROARCH.md HBM); Infinity-Cache hits are counted",
           "algorithmic_bytes": {"A": a_bytes, "B_codes": b_bytes, "B_scales": 32 * 4096 * (2 if kdt == "f16" else 4),
                                 "B_salient": 4096 * 448 * 2, "Y": M * N * 2}}
    json.dump(out, open(f"{O}/pmc_gemm_{kdt}_{act}.json", "w"), indent=1)
    print(act, "read MB", rd / 1e6, "write MB", wr / 1e6)
for f in ("per_group", "per_token"):
    d = json.loads(open(f"{O}/{tag}_bench_{f}.json").read().strip().splitlines()[-1])
    print(f, d["value"], d["roofline"]["achieved"], d.get("cpu_baseline"))
PY
