# Kernel-level profile of a short e2e run (MODEL, default opt-1.3b): W4A4 + unquantized.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/e2ep
O=$R/gpurun_out/e2ep
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_${MODEL:-opt-1.3b} -o run -- python $R/bench_e2e.py --model ${MODEL:-opt-1.3b} --layers 4 --windows 2 --no-ref --no-cpu --rounds 1 > $O/prof_${MODEL:-opt-1.3b}.log 2>&1 || { echo "rocprof failed"; tail -30 $O/prof_${MODEL:-opt-1.3b}.log; exit 1; }
tail -2 $O/prof_${MODEL:-opt-1.3b}.log
