# same-box A/B of library builds and / or knob settings on bench.py's llama_layer leg
# (Llama-2-7B decoder layer linears at 2048 tokens vs hipBLASLt fp16):
#   bash tools/ab_libs_layer.sh ROUNDS SPEC1 SPEC2 ...     SPEC = LIB.so[@VAR=value[,VAR=value]]
set -e
R=$1; shift
for r in $(seq $R); do for S in "$@"; do
  L=${S%%@*}; E=""; [ "$S" != "$L" ] && E=$(echo "${S#*@}" | tr ',' ' ')
  env SQMP_LIB_PATH=$L $E timeout -k 10 120 python -c "
import sys, torch; sys.path[:0] = ['.', 'smoothquant-mixedprecision_amd']
import bench
d = bench.llama_layer(torch.device('cuda'))
print('$S', 'layer', d['w4a4_ms'], 'fp16', d['fp16_linear_ms'], 'ratio', d['w4a4_over_fp16_speed'],
      {g: v['w4a4_ms'] for g, v in d['per_group'].items()})
" 2>&1 | grep -v amdgpu.ids
done; done
