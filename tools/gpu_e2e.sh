# End-to-end benches (configs 3 and 4) -> gpurun_out/e2e
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/e2e
O=gpurun_out/e2e
for m in ${MODELS:-opt-1.3b llama2-7b}; do
  timeout -k 10 500 python bench_e2e.py --model $m $E2E_ARGS > $O/e2e_$m.json 2> $O/e2e_$m.err || { echo "$m failed"; tail -20 $O/e2e_$m.err; exit 1; }
  cat $O/e2e_$m.json
done
