"""Same-box A/B of the grouped packed-order GEMM's schedules (sqmp_gemm_fq7_group_ws):
SQMP_FQ7_SK = 0 (data-parallel tiles, the launch's own tile height) / 0 with 256-row tiles /
1 (stream-K where the tiles are not whole rounds) / 2 (stream-K forced) / 3 (a remainder of
half a round cut into K halves).  The single layers (o_proj, down_proj: 128 tiles) also run
their standalone launch (sqmp_gemm_fq7, "alone").  HIP events, median of interleaved rounds.
python tools/sk_ab.py [rounds] [iters]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "smoothquant-mixedprecision_amd"), os.path.join(ROOT, "tests")]
import torch  # noqa: E402

import bench  # noqa: E402
from smoothquant import _lib, ops  # noqa: E402
from test_gpu_sibling import _siblings  # noqa: E402

rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 5
iters = int(sys.argv[2]) if len(sys.argv) > 2 else 30
dev = torch.device("cuda")
stream = torch.cuda.current_stream(dev)
SHAPES = [("qkv", 2048, 4096, (4096, 4096, 4096), 64, 0.05),
          ("gate_up", 2048, 4096, (11008, 11008), 64, 0.05),
          ("whole_512", 2048, 4096, (8192, 8192), 64, 0.05),
          ("o", 2048, 4096, (4096,), 64, 0.05),
          ("down", 2048, 11008, (4096,), 64, 0.05)]
VARIANTS = [("dp", {"SQMP_FQ7_SK": "0"}), ("dp256", {"SQMP_FQ7_SK": "0", "SQMP_FQ7G_TM": "256"}),
            ("sk", {"SQMP_FQ7_SK": "1"}), ("sk_forced", {"SQMP_FQ7_SK": "2"}),
            ("sk_halves", {"SQMP_FQ7_SK": "3"})]


def setenv(env):
    for k in ("SQMP_FQ7_SK", "SQMP_FQ7G_TM"):
        os.environ.pop(k, None)
    os.environ.update(env)
    _lib.reload_knobs()


for name, M, K, Ns, G, p in SHAPES:
    layers, x = _siblings(dev, M, K, Ns, G, p, torch.float16, seed=21)
    pws = [q.packed() for q in layers]
    a = (ops.quant_act_fp_group(x, pws, "per_group", 4, G) if len(pws) > 1
         else [ops.quant_act_fp(x, pws[0], "per_group", 4, G)])
    biases = [q.bias.reshape(-1) for q in layers]
    variants = VARIANTS + ([("alone", {})] if len(pws) == 1 else [])
    res = {v: [] for v, _ in variants}
    plans = {}
    for r in range(rounds):
        for v, env in variants:
            setenv(env)
            if v == "alone":
                plans[v] = ops.fq7_plan(pws, M, group=False)
                f = lambda: ops.gemm_fq7(a[0], pws[0], biases[0])  # noqa: E731
            else:
                plans[v] = ops.fq7_plan(pws, M, group=True)
                f = lambda: ops.gemm_fq7_group(a, pws, biases)  # noqa: E731
            for _ in range(3):
                f()
            res[v].append(bench.time_events(f, iters, stream) * 1e3)
    for v, _ in variants:
        t = sorted(res[v])
        print(f"{name:10s} {v:10s} plan {plans[v]}: median {t[len(t) // 2]:7.1f} us  min {t[0]:7.1f}", flush=True)
