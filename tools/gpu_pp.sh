set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/pp
cd /tmp && export TMPDIR=/tmp
for cfg in ${CFGS:-"2048 4096 4096 fp16 64" "2048 11008 4096 fp16 64"}; do
  n=$(echo $cfg | tr ' ' '_')
  timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/pp/$n -o run -- python $R/tools/prepass_prof.py $cfg > $R/gpurun_out/pp/$n.log 2>&1 || { echo "fail $n"; tail -5 $R/gpurun_out/pp/$n.log; exit 1; }
done
