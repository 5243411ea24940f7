"""Probe: GEMM time vs salient-tail width (int4 and dense main parts), M=16384, K=N=4096."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "smoothquant-mixedprecision_amd")]
import torch  # noqa: E402

from smoothquant import ops  # noqa: E402
from gemm_matrix import t_ms  # noqa: E402

M, K, N, G = int(sys.argv[1]) if len(sys.argv) > 1 else 16384, 4096, 4096, 128
dev = torch.device("cuda")
g = torch.Generator(device=dev).manual_seed(0)
w = (torch.randn(N, K, generator=g, device=dev) * 0.02).half()
x = torch.randn(M, K, generator=g, device=dev).half()
for mode in ("per_group", "none", "per_group", "none"):
    base = None
    for p in (0.0, 0.02, 0.05, 0.10, 0.20):
        sal = None
        if p > 0:
            sal = torch.argsort(x.float().abs().mean(0), descending=True)[: int(p * K)].cpu()
        pw = ops.pack_weight(w, mode, 4, G, sal)
        a = ops.quant_act_fp(x, pw, "per_token", 4, G)
        ms = t_ms(lambda: ops.gemm_fq(a, pw, None), it=200, warm_ms=300)
        if base is None:
            base = ms
        nd = pw.S_pad // 32
        extra = (ms - base) * 1e3
        print(f"{mode:9s} p={p:.2f} S_pad={pw.S_pad:4d}: {ms*1e3:7.1f} us  (+{extra:6.1f} us, "
              f"{extra / max(nd, 1):5.2f} us per 32-col dense stage per tile-row... )", flush=True)
