# One parameterised runner for every GPU-box step (replaces the per-experiment scripts).
#
#   gpurun -- bash tools/gpu.sh STEP [STEP ...]          (results -> gpurun_out/<tag>/)
#
# Steps (each under its own time limit; the first failure ends the run, nothing after it
# touches the GPU):
#   tests            pytest -m gpu (one process, per-test timeout)
#   tests:EXPR       pytest -m gpu -k EXPR
#   smoke            __graft_entry__.smoke()
#   bench            bench.py default (200 warm-up + 200 timed steps, CPU baseline leg)
#   bench20          bench.py --steps 20 --warmup 5 --no-cpu  (the driver's shape)
#   bench_pt         bench.py --act per_token --no-cpu
#   bench_fp32       bench.py --dtype fp32 --no-cpu --steps 100 --warmup 100
#   prof             rocprofv3 --kernel-trace --stats of bench.py --no-cpu
#   pmc:KIND         the four counter passes of tools/gemm_only.py KIND (fq|fqt|f8|h2|...);
#                    summarise with tools/pmc_summary.py
#   e2e              bench_e2e.py per model (MODELS, E2E_ARGS env; configs 3, 4)
#   sweep            bench_sweep.py (config 5)
#   layer            bench_e2e.py --model llama2-7b (config 4 end to end)
#   py:SCRIPT[:ARGS] python SCRIPT ARGS (comma-separated args)
#   profpy:SCRIPT[:ARGS]  the same under rocprofv3 --kernel-trace --stats
#   trace:SCRIPT[:ARGS]   the same under rocprofv3 --kernel-trace (per-dispatch CSV)
# TAG (env, default "run") names the output directory.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O="$R/gpurun_out/${TAG:-run}"
mkdir -p "$O"
export TMPDIR=/tmp

fail() { echo "FAILED: $1"; tail -25 "$2"; exit 1; }

step() {
  local s=$1
  case "$s" in
    tests|tests:*)
      local k=(); [ "$s" != tests ] && k=(-k "${s#tests:}")
      timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread \
        -p no:cacheprovider "${k[@]}" > "$O/pytest_gpu.log" 2>&1 || fail "$s" "$O/pytest_gpu.log"
      tail -1 "$O/pytest_gpu.log" ;;
    smoke)
      timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1 \
        || fail smoke "$O/smoke.log"
      tail -1 "$O/smoke.log" ;;
    bench)
      timeout -k 10 500 python bench.py > "$O/bench.json" 2> "$O/bench.err" || fail bench "$O/bench.err"
      cat "$O/bench.json" ;;
    bench20)
      timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu > "$O/bench20.json" 2> "$O/bench20.err" \
        || fail bench20 "$O/bench20.err"
      cat "$O/bench20.json" ;;
    bench_pt)
      timeout -k 10 300 python bench.py --act per_token --no-cpu > "$O/bench_pt.json" 2> "$O/bench_pt.err" \
        || fail bench_pt "$O/bench_pt.err"
      cat "$O/bench_pt.json" ;;
    bench_fp32)
      timeout -k 10 300 python bench.py --dtype fp32 --no-cpu --steps 100 --warmup 100 > "$O/bench_fp32.json" \
        2> "$O/bench_fp32.err" || fail bench_fp32 "$O/bench_fp32.err"
      cat "$O/bench_fp32.json" ;;
    prof)
      (cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof" -o run \
        -- python "$R/bench.py" --no-cpu > "$O/prof.log" 2>&1) || fail prof "$O/prof.log"
      f=$(ls "$O"/prof/*/run_kernel_stats.csv "$O"/prof/run_kernel_stats.csv 2>/dev/null | head -1)
      [ -n "$f" ] && cp "$f" "$O/kernel_stats.csv" && rm -rf "$O/prof" && head -6 "$O/kernel_stats.csv" | cut -c1-160 ;;
    pmc:*)
      # PMC_TAG (env): a suffix of the pass directories (knob sweeps: SQMP_...=v PMC_TAG=v);
      # PMC_PASSES (env, default "a b c d"): the passes to run
      local kind=${s#pmc:}
      local pa="SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT"
      local pb="SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE"
      local pc="FETCH_SIZE"
      local pd="WRITE_SIZE TCC_HIT_sum TCC_MISS_sum"
      for p in ${PMC_PASSES:-a b c d}; do
        local C; eval C=\$p$p
        local D="$O/pmc${PMC_TAG:+_$PMC_TAG}/${kind}_$p"
        mkdir -p "$(dirname "$D")"
        (cd /tmp && timeout -s KILL 120 rocprofv3 --pmc $C --output-format csv -d "$D" -o run \
          -- python "$R/tools/gemm_only.py" $kind 20 > "$D.log" 2>&1) || fail "pmc $kind $p" "$D.log"
      done
      echo "pmc $kind ok" ;;
    e2e)
      for m in ${MODELS:-opt-1.3b llama2-7b}; do
        timeout -k 10 600 python bench_e2e.py --model $m $E2E_ARGS > "$O/e2e_$m.json" 2> "$O/e2e_$m.err" \
          || fail "e2e $m" "$O/e2e_$m.err"
        cat "$O/e2e_$m.json"
      done ;;
    sweep)
      timeout -k 10 900 python bench_sweep.py > "$O/sweep.jsonl" 2> "$O/sweep.err" || fail sweep "$O/sweep.err"
      tail -2 "$O/sweep.jsonl" ;;
    layer)
      timeout -k 10 400 python bench_e2e.py --model llama2-7b > "$O/layer.json" 2> "$O/layer.err" || fail layer "$O/layer.err"
      cat "$O/layer.json" ;;
    profpy:*)
      local rest=${s#profpy:}; local script=${rest%%:*}; local args=""
      [ "$rest" != "$script" ] && args=$(echo "${rest#*:}" | tr ',' ' ')
      local name=$(basename "$script" .py)
      (cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof_$name" -o run \
        -- python "$R/$script" $args > "$O/prof_$name.log" 2>&1) || fail "$s" "$O/prof_$name.log"
      f=$(ls "$O"/prof_$name/*/run_kernel_stats.csv "$O"/prof_$name/run_kernel_stats.csv 2>/dev/null | head -1)
      [ -n "$f" ] && cp "$f" "$O/kernel_stats_$name.csv" && rm -rf "$O/prof_$name" && cut -d, -f1-4 "$O/kernel_stats_$name.csv" | cut -c1-150 ;;
    trace:*)
      local rest=${s#trace:}; local script=${rest%%:*}; local args=""
      [ "$rest" != "$script" ] && args=$(echo "${rest#*:}" | tr ',' ' ')
      local name=$(basename "$script" .py)
      (cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d "$O/trace_$name" -o run \
        -- python "$R/$script" $args > "$O/trace_$name.log" 2>&1) || fail "$s" "$O/trace_$name.log"
      f=$(ls "$O"/trace_$name/*/run_kernel_trace.csv "$O"/trace_$name/run_kernel_trace.csv 2>/dev/null | head -1)
      [ -n "$f" ] && cp "$f" "$O/kernel_trace_$name.csv" && rm -rf "$O/trace_$name" && echo "trace $name ok" ;;
    py:*)
      local rest=${s#py:}; local script=${rest%%:*}; local args=""
      [ "$rest" != "$script" ] && args=$(echo "${rest#*:}" | tr ',' ' ')
      local name=$(basename "$script" .py)
      timeout -k 10 600 python -u "$script" $args > "$O/$name.out" 2> "$O/$name.err" || fail "$s" "$O/$name.err"
      tail -40 "$O/$name.out" ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
}

for s in "$@"; do step "$s"; done
echo "all steps ok"
