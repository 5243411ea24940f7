"""Prepass kernels of one linear (for rocprofv3 --stats): quant_act_fp and the in-place output
quantizer, 20 calls each.  python tools/prepass_prof.py M K N dtype [G] [act]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "smoothquant-mixedprecision_amd")]
import torch  # noqa: E402

from smoothquant import ops  # noqa: E402
from smoothquant.fake_quant import W4A4Linear  # noqa: E402

M, K, N = (int(v) for v in sys.argv[1:4])
DT = {"fp16": torch.float16, "fp32": torch.float32, "bf16": torch.bfloat16}[sys.argv[4]]
G = int(sys.argv[5]) if len(sys.argv) > 5 else 128
act = sys.argv[6] if len(sys.argv) > 6 else "per_group"
dev = torch.device("cuda")
g = torch.Generator(device=dev).manual_seed(0)
lin = torch.nn.Linear(K, N).to(dev, DT)
x = torch.randn(M, K, generator=g, device=dev).to(DT)
q = W4A4Linear.from_float(lin, weight_quant="per_group", act_quant=act, quantize_output=K == N,
                          importance=x.float().abs().mean(0).cpu(), salient_prop=0.05, group_size=G)
pw = q.packed()
y = torch.randn(M, N, generator=g, device=dev).to(DT)
for _ in range(20):
    ops.quant_act_fp(x, pw, act, 4, G)
    ops.fake_quant_inplace(y, act, 4, G, pw.amap_fq, pw.nonsal, pw.S)
for _ in range(20):
    q(x)
torch.cuda.synchronize()
print("done")
