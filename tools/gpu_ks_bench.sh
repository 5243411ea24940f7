set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/prof2
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/ks -o run -- python $R/bench.py --no-cpu > $O/ks.log 2>&1 || { tail -5 $O/ks.log; exit 1; }
tail -1 $O/ks.log
