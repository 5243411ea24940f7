# Per-linear shapes (Llama fp16, OPT fp32) and a kernel-level profile of a 4-layer Llama e2e run.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out/e2ep
O=$R/gpurun_out/e2ep
timeout -k 10 200 python tools/model_shapes.py llama2-7b 2048 fp16 > $O/shapes_llama.txt 2>&1 || { tail -20 $O/shapes_llama.txt; exit 1; }
cat $O/shapes_llama.txt
timeout -k 10 200 python tools/model_shapes.py opt-1.3b 2048 fp32 > $O/shapes_opt32.txt 2>&1 || { tail -20 $O/shapes_opt32.txt; exit 1; }
cat $O/shapes_opt32.txt
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python $R/bench_e2e.py --model llama2-7b --layers 4 --windows 2 --no-ref --no-cpu --rounds 1 > $O/prof.log 2>&1 || { echo "rocprof failed"; tail -30 $O/prof.log; exit 1; }
tail -3 $O/prof.log
