"""In-process A/B of whole config-2 steps (W4A4Linear.forward, the bench.py step) under
per-launch tuning variables: interleaved rounds, HIP events, y bit-identical across variants.

    python tools/step_ab.py ENV=v1/v2/... [rounds] [iters] [act] [fp16|fp32]
                                                   (e.g. SQMP_NT_STORES=0/1 4 100 per_token)
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "smoothquant-mixedprecision_amd")]
import torch  # noqa: E402

import bench  # noqa: E402

var, vals = sys.argv[1].split("=")
vals = vals.split("/")
rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 4
iters = int(sys.argv[3]) if len(sys.argv) > 3 else 100
dev = torch.device("cuda")
act = sys.argv[4] if len(sys.argv) > 4 else "per_group"
dt = torch.float32 if len(sys.argv) > 5 and sys.argv[5] == "fp32" else torch.float16
q, x, lin = bench.make_layer(dev, act, seed=1, dtype=dt)
stream = torch.cuda.current_stream(dev)
ref = None
for v in vals:
    os.environ[var] = v
    __import__("smoothquant._lib", fromlist=["_lib"]).reload_knobs()  # (knobs are read once at load)
    y = q(x)
    torch.cuda.synchronize()
    if ref is None:
        ref = y.clone()
    assert torch.equal(y.view(torch.int16), ref.view(torch.int16)), f"{var}={v} changed y"
res = {v: [] for v in vals}
flops = 2.0 * bench.M * bench.N * bench.K
for _ in range(rounds):
    for v in vals:
        os.environ[var] = v
        __import__("smoothquant._lib", fromlist=["_lib"]).reload_knobs()  # (knobs are read once at load)
        for _ in range(20):
            q(x)
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(stream)
        for _ in range(iters):
            q(x)
        b.record(stream)
        b.synchronize()
        res[v].append(a.elapsed_time(b) / iters * 1e3)
for v in vals:
    t = sorted(res[v])
    print(f"{act} {dt}: {var}={v}: step median {t[len(t) // 2]:7.1f} us  min {t[0]:7.1f} us  "
          f"({flops / t[len(t) // 2] / 1e6:7.1f} TFLOP/s)  all {[round(u, 1) for u in res[v]]}")
