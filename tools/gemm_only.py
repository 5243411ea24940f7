"""Run only the W4A4 GEMM (and optionally the prepass) of BASELINE config 2 -- a target
for rocprofv3 counter passes.  python tools/gemm_only.py [fq|fqt|f8|h2|c4] [iters] [per_group|per_token] [prepass]
(c4: the activation-order prepass alone -- column max, rank table, fused quantizer + permutation)"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "smoothquant-mixedprecision_amd")]
import torch  # noqa: E402

import bench  # noqa: E402
from smoothquant import ops  # noqa: E402

kind = sys.argv[1] if len(sys.argv) > 1 else "fq"
iters = int(sys.argv[2]) if len(sys.argv) > 2 else 10
extra = sys.argv[3:]
prepass = "prepass" in extra
dev = torch.device("cuda")
act = next((a for a in extra if a.startswith("per_")), "per_group" if kind in ("fq", "fqt", "c4") else "per_token")
q, x, lin = bench.make_layer(dev, act, seed=1,
                             dtype=torch.float32 if kind == "h2" else torch.float16)
pw = q.packed()
if kind == "h2" and not ops.h2_planes_ok(pw, act, x.shape[0]):
    kind = "fq"  # the fp32 layer's gemm_fq runs sqmp_gemm_h2
if kind == "h2":  # the fp32 forward's path: quantizer -> f16 planes -> sqmp_gemm_h2d
    a2 = ops.quant_act_fp(x, pw, act, 4, bench.G, h2=True)
    for _ in range(iters):
        if prepass:
            ops.quant_act_fp(x, pw, act, 4, bench.G, h2=True)
        ops.gemm_h2_planes(a2, pw, lin.bias)
elif kind == "fq":
    a = ops.quant_act_fp(x, pw, act, 4, bench.G)
    for _ in range(iters):
        if prepass:
            ops.quant_act_fp(x, pw, act, 4, bench.G)
        ops.gemm_fq(a, pw, lin.bias)
elif kind == "fqt":
    c4 = ops.quant_act_c4(x, pw, act, 4, bench.G)
    for _ in range(iters):
        if prepass:
            ops.quant_act_c4(x, pw, act, 4, bench.G)
        ops.gemm_fqt(*c4, pw, lin.bias, bench.G)
elif kind == "c4":
    for _ in range(iters):
        ops.quant_act_c4(x, pw, act, 4, bench.G)
elif kind == "f8":
    a8, sa, xs = ops.quant_act_f8(x, pw, act, 4)
    for _ in range(iters):
        if prepass:
            ops.quant_act_f8(x, pw, act, 4)
        ops.gemm_f8(a8, sa, xs, pw, lin.bias)
else:
    raise SystemExit(f"unknown kind {kind}")
torch.cuda.synchronize()
print("done", kind, iters)
