"""GEMM-only timings (int4 + salient tail) of the faithful kernels at the benchmark shapes:
fq (packed order) at every shape, fqt (activation order) at config 2.  One line per shape;
run it under different env knobs to A/B a kernel variant.  python tools/gemm_ab.py [label]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "smoothquant-mixedprecision_amd"), os.path.join(ROOT, "tools")]
import torch  # noqa: E402

from gemm_matrix import SHAPES, t_ms  # noqa: E402
from smoothquant import ops  # noqa: E402

label = sys.argv[1] if len(sys.argv) > 1 else ""
dev = torch.device("cuda")
out = []
for (M, K, N, G, p) in SHAPES:
    g = torch.Generator(device=dev).manual_seed(0)
    w = (torch.randn(N, K, generator=g, device=dev) * 0.02).half()
    x = torch.randn(M, K, generator=g, device=dev).half()
    sal = torch.argsort(x.float().abs().mean(0), descending=True)[: int(p * K)].cpu()
    pw = ops.pack_weight(w, "per_group", 4, G, sal)
    a = ops.quant_act_fp(x, pw, "per_group", 4, G)
    fl = 2.0 * M * N * K
    ms = t_ms(lambda: ops.gemm_fq(a, pw, None), it=100, warm_ms=300)
    out.append(f"fq {M}x{K}x{N} {ms*1e3:7.1f}us {fl / ms / 1e9:7.1f}TF")
    if M >= 8192:
        c4 = ops.quant_act_c4(x, pw, "per_group", 4, G)
        ms = t_ms(lambda: ops.gemm_fqt(*c4, pw, None, G), it=100, warm_ms=300)
        out.append(f"fqt {M}x{K}x{N} {ms*1e3:7.1f}us {fl / ms / 1e9:7.1f}TF")
print(label, " | ".join(out), flush=True)
