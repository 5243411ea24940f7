"""Same-box A/B of the grouped packed-order GEMM's row-tile height (SQMP_FQ7G_TM 128 / 256,
with the launch's own OPT) on the Llama-2-7B sibling shapes at 2048 tokens; HIP events,
interleaved rounds.  python tools/group_tm_ab.py [rounds] [iters]"""
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
SHAPES = [("qkv", 2048, 4096, (4096, 4096, 4096)), ("gate_up", 2048, 4096, (11008, 11008))]
for name, M, K, Ns in SHAPES:
    layers, x = _siblings(dev, M, K, Ns, 64, 0.05, torch.float16, seed=21)
    pws = [q.packed() for q in layers]
    a = ops.quant_act_fp_group(x, pws, "per_group", 4, 64)
    biases = [q.bias.reshape(-1) for q in layers]
    res, plans = {}, {}
    for r in range(rounds):
        for tm in ("128", "256"):
            os.environ["SQMP_FQ7G_TM"] = tm
            _lib.reload_knobs()
            plans[tm] = ops.fq7_plan(pws, M, group=True)
            f = lambda: ops.gemm_fq7_group(a, pws, biases)  # noqa: E731
            for _ in range(3):
                f()
            res.setdefault(tm, []).append(bench.time_events(f, iters, stream) * 1e3)
    os.environ.pop("SQMP_FQ7G_TM")
    _lib.reload_knobs()
    for tm, t in res.items():
        t = sorted(t)
        print(f"{name:8s} TM {tm} plan {plans[tm]}: median {t[len(t) // 2]:7.1f} us  min {t[0]:7.1f}",
              flush=True)
