# GPU parity tests and the per_group quick bench for each fq tile variant.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for wm in 1 2; do
  SQMP_FQ_WAVES_M=$wm timeout -k 10 600 python -m pytest tests -m gpu -q --maxfail=5 -p no:cacheprovider > gpurun_out/pytest_gpu_wm$wm.log 2>&1
  rc=$?
  tail -4 gpurun_out/pytest_gpu_wm$wm.log
  [ $rc -ne 0 ] && { echo "gpu tests failed (waves_m=$wm) rc=$rc"; grep -E "^(FAILED|ERROR)|Error|mismatch" gpurun_out/pytest_gpu_wm$wm.log | head -30; exit $rc; }
  SQMP_FQ_WAVES_M=$wm timeout -k 10 300 python bench.py --no-cpu > gpurun_out/bq_pg_wm$wm.json 2> gpurun_out/bq_pg_wm$wm.err || { tail -20 gpurun_out/bq_pg_wm$wm.err; exit 1; }
  python - gpurun_out/bq_pg_wm$wm.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r = d["roofline"]
print(sys.argv[1], "value", d["value"], "ms", d["ms_per_step"], "| gemm", r["achieved"], r["unit"], "frac", r["frac"], r["avg_ms"], "ms")
PY
done
