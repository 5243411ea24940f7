"""Drive only the activation quantizer (for rocprofv3 kernel traces / counters).
python tools/prepass_only.py M K G act iters"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "smoothquant-mixedprecision_amd")]
import torch  # noqa: E402

from smoothquant import ops  # noqa: E402
from smoothquant.fake_quant import W4A4Linear  # noqa: E402

M, K, G = (int(a) for a in sys.argv[1:4])
act = sys.argv[4]
iters = int(sys.argv[5])
dev = torch.device("cuda")
g = torch.Generator(device=dev).manual_seed(0)
lin = torch.nn.Linear(K, 4096, bias=False).to(dev, torch.float16)
with torch.no_grad():
    lin.weight.copy_(torch.randn(4096, K, generator=g, device=dev) * 0.02)
x = torch.randn(M, K, generator=g, device=dev)
x[:, torch.randperm(K, generator=g, device=dev)[: K // 100]] *= 30
x = x.half()
q = W4A4Linear.from_float(lin, weight_quant="per_group", act_quant=act,
                          importance=x.float().abs().mean(0).cpu(), salient_prop=0.05 if K != 4096 or M != 16384 else 0.10,
                          group_size=G)
pw = q.packed()
for _ in range(iters):
    ops.quant_act_fp(x, pw, act, 4, G)
torch.cuda.synchronize()
