set -o pipefail
cd $GRAFT_REPO_ROOT
for m in 4096 8192; do
  for v in 0 1; do
    echo "M=$m SQMP_FQT=$v"
    SQMP_FQT=$v timeout -k 10 200 python tools/model_shapes.py llama2-7b $m fp16 2>&1 | grep -v amdgpu.ids || exit 1
  done
done
