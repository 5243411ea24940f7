"""Same-process A/B of the grouped sibling GEMM (sqmp_gemm_fq7_group) at the Llama-2-7B
2048-token shapes: q/k/v (3 x 4096 -> 4096) and gate/up (2 x 4096 -> 11008), each launch
variant given as VAR=v1/v2/... (read per launch, e.g. SQMP_FQ7G_TM=128/256 SQMP_FQ7_OPT=3/8),
interleaved rounds, median of ITERS launches per round; the sum of the members' own
sqmp_gemm_fq7 launches for comparison.

    python tools/group_ab.py [ITERS] [VAR=v1/v2 ...]
"""
import itertools
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "smoothquant-mixedprecision_amd"), os.path.join(ROOT, "tests")]
import torch  # noqa: E402

import bench  # noqa: E402
from smoothquant import ops  # noqa: E402
from test_gpu_sibling import _siblings  # noqa: E402

iters = int(sys.argv[1]) if len(sys.argv) > 1 and "=" not in sys.argv[1] else 50
axes = [(kv.split("=")[0], kv.split("=")[1].split("/")) for kv in sys.argv[1:] if "=" in kv]
dev = torch.device("cuda")
stream = torch.cuda.current_stream(dev)
cases = []
for name, Ns in (("qkv", (4096, 4096, 4096)), ("gate_up", (11008, 11008))):
    layers, x = _siblings(dev, bench.LLAMA_T, 4096, Ns, bench.LLAMA_G, bench.LLAMA_P,
                          torch.float16, seed=1)
    pws = [q.packed() for q in layers]
    a = ops.quant_act_fp_group(x, pws, "per_group", 4, bench.LLAMA_G)
    cases.append((name, pws, a))
combos = list(itertools.product(*[v for _, v in axes])) if axes else [()]
res = {}
for rnd in range(3):
    for name, pws, a in cases:
        for combo in combos:
            for (k, _), v in zip(axes, combo):
                os.environ[k] = v
                __import__("smoothquant._lib", fromlist=["_lib"]).reload_knobs()  # (knobs are read once at load)
            tag = " ".join(f"{k}={v}" for (k, _), v in zip(axes, combo)) or "default"
            fn = lambda: ops.gemm_fq7_group(a, pws, [None] * len(pws))  # noqa: E731
            for _ in range(3):
                fn()
            res.setdefault((name, tag), []).append(bench.time_events(fn, iters, stream) * 1e3)
        for k, _ in axes:
            os.environ.pop(k, None)
            __import__("smoothquant._lib", fromlist=["_lib"]).reload_knobs()  # (knobs are read once at load)
        own = lambda: [ops.gemm_fq7(ai, pw, None) for ai, pw in zip(a, pws)]  # noqa: E731
        for _ in range(3):
            own()
        res.setdefault((name, "members alone (sum)"), []).append(
            bench.time_events(own, iters, stream) * 1e3)
for (name, tag), v in res.items():
    print(f"{name:8s} {tag:40s} median {statistics.median(v):7.1f} us  all "
          + ", ".join(f"{t:.1f}" for t in v), flush=True)
