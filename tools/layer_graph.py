"""The Llama-2-7B decoder layer's 7 linears at 2048 tokens (bench.llama_layer's layer) run
eagerly and replayed from a HIP graph (torch.cuda.graph), W4A4 and fp16 F.linear alike:
per-pass GPU time (HIP events over 40 back-to-back passes, median of interleaved rounds).
python tools/layer_graph.py [rounds]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "smoothquant-mixedprecision_amd")]
import torch  # noqa: E402

import bench  # noqa: E402
from smoothquant.fake_quant import W4A4Linear, link_siblings  # noqa: E402

rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 5
dev = torch.device("cuda")
gen = torch.Generator(device=dev).manual_seed(7)
xs = {}
for name, K in (("attn", 4096), ("o", 4096), ("mlp", 4096), ("down", 11008)):
    x = torch.randn(bench.LLAMA_T, K, generator=gen, device=dev)
    x[:, torch.randperm(K, generator=gen, device=dev)[: K // 100]] *= 30.0
    xs[name] = x.half()
layers = []
for name, K, N, src in bench.LLAMA_LINEARS:
    lin = torch.nn.Linear(K, N, bias=False).to(dev, torch.float16)
    with torch.no_grad():
        lin.weight.copy_((torch.randn(N, K, generator=gen, device=dev) * 0.02).half())
    imp = xs[src][:512].float().abs().mean(0).cpu()
    q = W4A4Linear.from_float(lin, weight_quant="per_group", act_quant="per_group", importance=imp,
                              salient_prop=bench.LLAMA_P, group_size=bench.LLAMA_G)
    layers.append((q, lin.weight.detach(), xs[src]))
link_siblings(*[layers[i][0] for i in (0, 1, 2)])
link_siblings(*[layers[i][0] for i in (4, 5)])


def w4a4():
    return [q(x) for q, _, x in layers]


def fp16():
    return [torch.nn.functional.linear(x, w) for _, w, x in layers]


def graph_of(fn):
    s = torch.cuda.Stream(dev)
    s.wait_stream(torch.cuda.current_stream(dev))
    with torch.cuda.stream(s):
        for _ in range(3):
            fn()
    torch.cuda.current_stream(dev).wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        fn()
    return g.replay


with torch.no_grad():
    variants = {"w4a4 eager": w4a4, "fp16 eager": fp16, "w4a4 graph": graph_of(w4a4),
                "fp16 graph": graph_of(fp16)}
    stream = torch.cuda.current_stream(dev)
    res = {k: [] for k in variants}
    for r in range(rounds):
        for k, fn in variants.items():
            for _ in range(5):
                fn()
            res[k].append(bench.time_events(fn, 40, stream) * 1e3)
    med = {k: sorted(v)[len(v) // 2] for k, v in res.items()}
    for k, v in med.items():
        print(f"{k:12s} {v:7.1f} us per layer pass", flush=True)
    print(f"ratio fp16 / w4a4: eager {med['fp16 eager'] / med['w4a4 eager']:.4f}, "
          f"graph {med['fp16 graph'] / med['w4a4 graph']:.4f}")
