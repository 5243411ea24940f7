"""The packed-order per_group quantizer (sqmp_quant_act_v2 OUT_FP: column max + rank table +
lane-contiguous quantizer) at K = 4096 / 11008 over M = 1024 .. 16384 rows, and the same call
with the statistics reused (table + quantizer only): whether the 2048-token Llama calls are
latency- or throughput-bound.  python tools/quant_scaling.py [VAR=v1/v2 ...]"""
import itertools
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "smoothquant-mixedprecision_amd")]
import torch  # noqa: E402

import bench  # noqa: E402
from smoothquant import ops  # noqa: E402

axes = [(kv.split("=")[0], kv.split("=")[1].split("/")) for kv in sys.argv[1:]]
dev = torch.device("cuda")
stream = torch.cuda.current_stream(dev)
for K, N in ((4096, 4096), (11008, 4096)):
    g = torch.Generator(device=dev).manual_seed(0)
    w = (torch.randn(N, K, generator=g, device=dev) * 0.02).half()
    xf = torch.randn(16384, K, generator=g, device=dev).half()
    sal = torch.argsort(xf[:512].float().abs().mean(0), descending=True)[: int(0.05 * K)].cpu()
    pw = ops.pack_weight(w, "per_group", 4, 64, sal)
    pw2 = ops.pack_weight(w.flip(0), "per_group", 4, 64, sal)  # a sibling (same salient set)
    for combo in itertools.product(*[v for _, v in axes]) if axes else [()]:
        for (k, _), v in zip(axes, combo):
            os.environ[k] = v
            __import__("smoothquant._lib", fromlist=["_lib"]).reload_knobs()  # (knobs are read once at load)
        tag = " ".join(f"{k}={v}" for (k, _), v in zip(axes, combo))
        line = []
        for M in (1024, 2048, 4096, 8192, 16384):
            x = xf[:M]
            full = lambda: ops.quant_act_fp(x, pw, "per_group", 4, 64)  # noqa: E731

            def sib():
                ops.quant_act_fp(x, pw, "per_group", 4, 64)
                ops.quant_act_fp(x, pw2, "per_group", 4, 64)   # reuses the statistics
            tf = bench.time_events(full, 50, stream) * 1e3
            ts = bench.time_events(sib, 50, stream) * 1e3 - tf
            line.append(f"M={M}: {tf:6.1f} / sib {ts:6.1f} us")
        print(f"K={K} {tag}: " + " | ".join(line), flush=True)
