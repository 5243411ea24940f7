# Quick bench (no CPU leg, no profiler) for both act modes.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --no-cpu > gpurun_out/bq_pg.json 2> gpurun_out/bq_pg.err || { tail -20 gpurun_out/bq_pg.err; exit 1; }
timeout -k 10 300 python bench.py --no-cpu --act per_token > gpurun_out/bq_pt.json 2> gpurun_out/bq_pt.err || { tail -20 gpurun_out/bq_pt.err; exit 1; }
python - <<'PY'
import json
for f in ("gpurun_out/bq_pg.json", "gpurun_out/bq_pt.json"):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    r = d["roofline"]
    print(f, "value", d["value"], "ms", d["ms_per_step"], "| gemm", r["achieved"], r["unit"], "frac", r["frac"], r["avg_ms"], "ms | prepass", d["prepass"])
PY
