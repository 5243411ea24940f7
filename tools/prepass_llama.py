"""Prepass kernels of the Llama-2-7B 2048-token inputs, one segment per (input, variant), for
`rocprofv3 --kernel-trace` + tools/seg_trace.py: the sibling-group quantizer (q/k/v: 3
outputs, gate/up: 2) and the single-layer quantizer (o: K = 4096, down: K = 11008), each with
the tuning variables given as VAR=v1/v2 (read per launch, e.g. SQMP_LC_PERCU=1/2/4/8).
Prints the segment labels (SEG ...) in order; also M sweeps with M=... (e.g. M=1024/2048/4096).

    python tools/prepass_llama.py [ITERS] [VAR=v1/v2 ...] > labels.txt
"""
import itertools
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "smoothquant-mixedprecision_amd"), os.path.join(ROOT, "tests"),
                os.path.join(ROOT, "tools")]
import torch  # noqa: E402

import bench  # noqa: E402
from seg_trace import mark  # noqa: E402
from smoothquant import ops  # noqa: E402
from test_gpu_sibling import _siblings  # noqa: E402

iters = int(sys.argv[1]) if len(sys.argv) > 1 and "=" not in sys.argv[1] else 10
axes = [(kv.split("=")[0], kv.split("=")[1].split("/")) for kv in sys.argv[1:] if "=" in kv]
Ms = [int(v) for k, vs in axes if k == "M" for v in vs] or [bench.LLAMA_T]
axes = [(k, v) for k, v in axes if k != "M"]
dev = torch.device("cuda")
G = bench.LLAMA_G
cases = []
for name, K, Ns in (("qkv", 4096, (4096, 4096, 4096)), ("o", 4096, (4096,)),
                    ("gate_up", 4096, (11008, 11008)), ("down", 11008, (4096,))):
    layers, x = _siblings(dev, max(Ms), K, Ns, G, bench.LLAMA_P, torch.float16, seed=2)
    cases.append((name, [q.packed() for q in layers], x))
for combo in itertools.product(*[v for _, v in axes]) if axes else [()]:
    for (k, _), v in zip(axes, combo):
        os.environ[k] = v
        __import__("smoothquant._lib", fromlist=["_lib"]).reload_knobs()  # (knobs are read once at load)
    tag = " ".join(f"{k}={v}" for (k, _), v in zip(axes, combo)) or "default"
    for M in Ms:
        for name, pws, x in cases:
            xm = x[:M].contiguous()
            mark()
            print(f"SEG {name} M={M} {tag}", flush=True)
            for _ in range(iters):
                if len(pws) > 1:
                    ops.quant_act_fp_group(xm, pws, "per_group", 4, G)
                else:
                    ops.quant_act_fp(xm, pws[0], "per_group", 4, G)
mark()
