"""Same-box A/B of one launch knob on one config-2 GEMM: interleaved rounds, HIP events on the
launch stream, outputs checked bit-identical across the values.

    python tools/knob_ab.py KIND KNOB v1/v2/... [rounds] [iters]
    KIND: fqt (act per_group, the activation-order GEMM) | f8 (act per_token) | h2 (fp32 layer,
          sqmp_gemm_h2d on the quantizer's planes)
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "smoothquant-mixedprecision_amd")]
import torch  # noqa: E402

import bench  # noqa: E402
from smoothquant import ops  # noqa: E402
from smoothquant._lib import reload_knobs  # noqa: E402

kind, knob, vals = sys.argv[1], sys.argv[2], sys.argv[3].split("/")
rounds = int(sys.argv[4]) if len(sys.argv) > 4 else 4
iters = int(sys.argv[5]) if len(sys.argv) > 5 else 100
dev = torch.device("cuda")
act = "per_token" if kind == "f8" else "per_group"
q, x, lin = bench.make_layer(dev, act, seed=1,
                             dtype=torch.float32 if kind == "h2" else torch.float16)
pw = q.packed()
if kind == "h2":
    a2 = ops.quant_act_fp(x, pw, act, 4, bench.G, h2=True)
    gemm = lambda: ops.gemm_h2_planes(a2, pw, lin.bias)  # noqa: E731
elif kind == "f8":
    a8, sa, xs = ops.quant_act_f8(x, pw, act, 4)
    gemm = lambda: ops.gemm_f8(a8, sa, xs, pw, lin.bias)  # noqa: E731
else:
    c4 = ops.quant_act_c4(x, pw, act, 4, bench.G)
    gemm = lambda: ops.gemm_fqt(*c4, pw, lin.bias, bench.G)  # noqa: E731


def use(v):
    os.environ[knob] = v
    reload_knobs()


def timed(n):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(n):
        gemm()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / n * 1e3


ref = None
for v in vals:
    use(v)
    y = gemm()
    torch.cuda.synchronize()
    if ref is None:
        ref = y.clone()
    assert torch.equal(y.view(torch.int16 if y.dtype != torch.float32 else torch.int32),
                       ref.view(torch.int16 if y.dtype != torch.float32 else torch.int32)), v
    timed(30)
res = {v: [] for v in vals}
for r in range(rounds):
    for v in vals:
        use(v)
        res[v].append(timed(iters))
    print(f"round {r}: " + "  ".join(f"{knob}={v} {t[-1]:.1f}" for v, t in res.items()), flush=True)
for v, t in res.items():
    print(f"{kind} {knob}={v}: median {sorted(t)[len(t) // 2]:.1f} us  min {min(t):.1f}")
