"""Time the W4A4 GEMM alone on BASELINE config 2 (HIP events, GEMM on torch's current
stream).  python tools/gemm_time.py [fq|fq7|fqt|f8] [iters]  -> one line: kind, avg ms, TFLOP/s."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "smoothquant-mixedprecision_amd")]
import torch  # noqa: E402

import bench  # noqa: E402
from smoothquant import ops  # noqa: E402

kind = sys.argv[1] if len(sys.argv) > 1 else "fq"
iters = int(sys.argv[2]) if len(sys.argv) > 2 else 50
dev = torch.device("cuda")
act = "per_group" if kind in ("fq", "fq7", "fqt") else "per_token"
q, x, lin = bench.make_layer(dev, act, seed=1)
pw = q.packed()
if kind == "fq":
    a = ops.quant_act_fp(x, pw, act, 4, bench.G)
    ops.FQ7_AUTO = False
    run = lambda: ops.gemm_fq(a, pw, lin.bias)  # noqa: E731
elif kind == "fqt":
    c4 = ops.quant_act_c4(x, pw, act, 4, bench.G)
    run = lambda: ops.gemm_fqt(*c4, pw, lin.bias, bench.G)  # noqa: E731
elif kind == "fq7":
    a = ops.quant_act_fp(x, pw, act, 4, bench.G)
    run = lambda: ops.gemm_fq7(a, pw, lin.bias)  # noqa: E731
elif kind == "f8":
    a8, sa, xs = ops.quant_act_f8(x, pw, act, 4)
    run = lambda: ops.gemm_f8(a8, sa, xs, pw, lin.bias)  # noqa: E731
else:
    raise SystemExit(f"unknown kind {kind}")
t_end = __import__("time").perf_counter() + 2.0  # settle the clock
while __import__("time").perf_counter() < t_end:
    for _ in range(10):
        run()
    torch.cuda.synchronize()
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(iters):
    run()
e1.record()
torch.cuda.synchronize()
ms = e0.elapsed_time(e1) / iters
M, K, N = x.shape[0], x.shape[1], lin.out_features
print(f"{kind} variant={os.environ.get('SQMP_FQ_VARIANT', 'default')} avg_ms={ms:.4f} "
      f"TFLOP/s={2 * M * N * K / ms / 1e9:.1f}")
