set -o pipefail
cd $GRAFT_REPO_ROOT
for v in 0 1 2 4 0; do
  echo "SQMP_LC_PERCU=$v"
  if [ $v = 0 ]; then unset SQMP_LC_PERCU; else export SQMP_LC_PERCU=$v; fi
  timeout -k 10 200 python tools/model_shapes.py llama2-7b 2048 fp16 2>&1 | grep -v amdgpu.ids || exit 1
done
