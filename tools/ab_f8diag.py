"""Timing diagnostics of the FP8 per_token GEMM at config 2 (SQMP_F8_DIAG, diagnostics
library only: SQMP_DIAG_LIB=1 after SQMP_DIAG=1 python smoothquant-mixedprecision_amd/build_ext.py).
Wrong results by design for every value but 0: no equality check.
    SQMP_DIAG_LIB=1 python tools/ab_f8diag.py [values, '+'-separated] [rounds] [iters] [ENV]
ENV (default SQMP_F8_DIAG) names the per-launch variable: SQMP_F8_OPT A/Bs the product
variants on the product library (y checked equal across them)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "smoothquant-mixedprecision_amd")]
import torch  # noqa: E402

import bench  # noqa: E402
from smoothquant import ops  # noqa: E402

vals = (sys.argv[1] if len(sys.argv) > 1 else "0+1+2+3").split("+")
rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 4
iters = int(sys.argv[3]) if len(sys.argv) > 3 else 100
ENV = sys.argv[4] if len(sys.argv) > 4 else "SQMP_F8_DIAG"
dev = torch.device("cuda")
q, x, lin = bench.make_layer(dev, "per_token", seed=1)
pw = q.packed()
a8, sa, xs = ops.quant_act_f8(x, pw, "per_token", 4)
stream = torch.cuda.current_stream(dev)
res = {v: [] for v in vals}
ref = None
if ENV != "SQMP_F8_DIAG":  # product variants: identical outputs
    for v in vals:
        os.environ[ENV] = v
        __import__("smoothquant._lib", fromlist=["_lib"]).reload_knobs()  # (knobs are read once at load)
        y = ops.gemm_f8(a8, sa, xs, pw, lin.bias)
        torch.cuda.synchronize()
        if ref is None:
            ref = y.clone()
        assert torch.equal(y, ref), f"{ENV}={v}: y differs"
for _ in range(rounds):
    for v in vals:
        os.environ[ENV] = v
        __import__("smoothquant._lib", fromlist=["_lib"]).reload_knobs()  # (knobs are read once at load)
        for _ in range(10):
            ops.gemm_f8(a8, sa, xs, pw, lin.bias)
        t0, t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0.record(stream)
        for _ in range(iters):
            ops.gemm_f8(a8, sa, xs, pw, lin.bias)
        t1.record(stream)
        t1.synchronize()
        res[v].append(t0.elapsed_time(t1) / iters * 1e3)
for v in vals:
    r = sorted(res[v])
    print(f"{ENV}={v}: median {r[len(r) // 2]:7.1f} us  all {[round(t, 1) for t in res[v]]}", flush=True)
