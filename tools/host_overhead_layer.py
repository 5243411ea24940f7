"""Host (CPU) time to enqueue one Llama-layer pass of bench.llama_layer's 7 W4A4 linears vs
the GPU time of the pass: when the enqueue is slower, the GPU waits for the host.  Also a
cProfile of the enqueue (top functions by cumulative time)."""
import cProfile
import os
import pstats
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "smoothquant-mixedprecision_amd")]
import torch  # noqa: E402

import bench  # noqa: E402
from smoothquant.fake_quant import W4A4Linear, link_siblings  # noqa: E402

dev = torch.device("cuda")
gen = torch.Generator(device=dev).manual_seed(7)
xs = {}
for name, K in (("attn", 4096), ("o", 4096), ("mlp", 4096), ("down", 11008)):
    x = torch.randn(bench.LLAMA_T, K, generator=gen, device=dev)
    xs[name] = x.half()
layers = []
for name, K, N, src in bench.LLAMA_LINEARS:
    lin = torch.nn.Linear(K, N, bias=False).to(dev, torch.float16)
    imp = xs[src][:512].float().abs().mean(0).cpu()
    q = W4A4Linear.from_float(lin, weight_quant="per_group", act_quant="per_group",
                              importance=imp, salient_prop=bench.LLAMA_P, group_size=bench.LLAMA_G)
    layers.append((q, xs[src]))
link_siblings(*[layers[i][0] for i in (0, 1, 2)])
link_siblings(*[layers[i][0] for i in (4, 5)])


def run():
    for q, x in layers:
        q(x)


for _ in range(10):
    run()
torch.cuda.synchronize()
n = 40
t0 = time.perf_counter()
for _ in range(n):
    run()
t1 = time.perf_counter()
torch.cuda.synchronize()
t2 = time.perf_counter()
print(f"host enqueue per pass {1e6 * (t1 - t0) / n:.1f} us; wall per pass {1e6 * (t2 - t0) / n:.1f} us")
pr = cProfile.Profile()
pr.enable()
for _ in range(20):
    run()
pr.disable()
torch.cuda.synchronize()
pstats.Stats(pr).sort_stats("tottime").print_stats(18)
