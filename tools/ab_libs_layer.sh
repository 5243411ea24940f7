# same-box A/B of library builds on bench.py's llama_layer leg (Llama-2-7B decoder layer
# linears at 2048 tokens vs hipBLASLt fp16) and the config-2 prepass:
#   bash tools/ab_libs_layer.sh ROUNDS LIB1 LIB2 ...
set -e
R=$1; shift
for r in $(seq $R); do for L in "$@"; do
  SQMP_LIB_PATH=$L timeout -k 10 120 python -c "
import sys, torch; sys.path[:0] = ['.', 'smoothquant-mixedprecision_amd']
import bench
d = bench.llama_layer(torch.device('cuda'))
print('$L', 'layer', d['w4a4_ms'], 'fp16', d['fp16_linear_ms'], 'ratio', d['w4a4_over_fp16_speed'],
      {g: v['w4a4_ms'] for g, v in d['per_group'].items()})
" 2>&1 | grep -v amdgpu.ids
done; done
