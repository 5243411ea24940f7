"""Prepass of the Llama-2-7B decoder-layer linears at 2048 tokens (bench.py llama_layer's
shapes: G = 64, 5 % salient, per_group sorted activations, fp16) with the per-launch tuning
variables swept: one ops.quant_act_fp call (column max + rank table + quantizer) per input
width, HIP events, ITERS calls each.

    python tools/llama_prepass.py [ITERS] [VAR=v1/v2/... ...]     (e.g. SQMP_RT_TPO=4/8/16/32)
"""
import itertools
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "smoothquant-mixedprecision_amd")]
import torch  # noqa: E402

import bench  # noqa: E402
from smoothquant import ops  # noqa: E402
from smoothquant.fake_quant import W4A4Linear  # noqa: E402

iters = int(sys.argv[1]) if len(sys.argv) > 1 else 50
axes = [(kv.split("=")[0], kv.split("=")[1].split("/")) for kv in sys.argv[2:]]
dev = torch.device("cuda")
gen = torch.Generator(device=dev).manual_seed(7)
cases = []
for K, N in ((4096, 4096), (11008, 4096)):
    x = torch.randn(bench.LLAMA_T, K, generator=gen, device=dev)
    x[:, torch.randperm(K, generator=gen, device=dev)[: K // 100]] *= 30.0
    x = x.to(torch.float16)
    lin = torch.nn.Linear(K, N, bias=False).to(dev, torch.float16)
    with torch.no_grad():
        lin.weight.copy_((torch.randn(N, K, generator=gen, device=dev) * 0.02).half())
    imp = x[:512].float().abs().mean(0).cpu()
    q = W4A4Linear.from_float(lin, weight_quant="per_group", act_quant="per_group",
                              importance=imp, salient_prop=bench.LLAMA_P,
                              group_size=bench.LLAMA_G)
    cases.append((K, x, q.packed()))
stream = torch.cuda.current_stream(dev)

for combo in itertools.product(*[v for _, v in axes]) if axes else [()]:
    for (k, _), v in zip(axes, combo):
        os.environ[k] = v
        __import__("smoothquant._lib", fromlist=["_lib"]).reload_knobs()  # (knobs are read once at load)
    tag = " ".join(f"{k}={v}" for (k, _), v in zip(axes, combo)) or "default"
    res = []
    for K, x, pw in cases:
        ref = ops.quant_act_fp(x, pw, "per_group", 4, bench.LLAMA_G).clone()
        fn = lambda: ops.quant_act_fp(x, pw, "per_group", 4, bench.LLAMA_G)  # noqa: E731
        for _ in range(5):
            fn()
        ok = torch.equal(fn().view(torch.int16), ref.view(torch.int16))
        res.append(f"K={K}: {bench.time_events(fn, iters, stream) * 1e3:6.1f} us{'' if ok else ' MISMATCH'}")
    print(f"{tag:32s} " + "  ".join(res), flush=True)
