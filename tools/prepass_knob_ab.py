"""Same-box A/B of one launch knob on a prepass (quantizer) launch at config 2 or a Llama
shape: interleaved rounds, HIP events, outputs checked bit-identical across the values.

    python tools/prepass_knob_ab.py KIND KNOB v1/v2/... [rounds] [iters]
    KIND: f8 (per_token e4m3 quantizer, config 2) | c4 (act-order quantizer + permutation,
          config 2) | fp (packed-order per_group quantizer, 2048 x 11008 Llama down_proj) |
          fp4k (the same at 2048 x 4096, Llama o_proj)
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
if kind in ("fp", "fp4k"):
    from smoothquant.fake_quant import W4A4Linear
    KK = 11008 if kind == "fp" else 4096
    g = torch.Generator(device=dev).manual_seed(0)
    x = torch.randn(2048, KK, generator=g, device=dev)
    x[:, torch.randperm(KK, generator=g, device=dev)[:KK // 100]] *= 30.0
    x = x.half()
    lin = torch.nn.Linear(KK, 4096, bias=False).to(dev, torch.float16)
    q = W4A4Linear.from_float(lin, weight_quant="per_group", act_quant="per_group",
                              importance=x[:512].float().abs().mean(0).cpu(), salient_prop=0.05,
                              group_size=64)
    pw = q.packed()
    run = lambda: [ops.quant_act_fp(x, pw, "per_group", 4, 64)]  # noqa: E731
else:
    q, x, lin = bench.make_layer(dev, "per_token" if kind == "f8" else "per_group", seed=1)
    pw = q.packed()
    if kind == "f8":
        run = lambda: list(ops.quant_act_f8(x, pw, "per_token", 4))  # noqa: E731
    else:
        run = lambda: list(ops.quant_act_c4(x, pw, "per_group", 4, bench.G))  # noqa: E731


def use(v):
    os.environ[knob] = v
    reload_knobs()


def bits(t):
    return t.contiguous().view(torch.uint8)


def timed(n):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(n):
        run()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / n * 1e3


ref = None
for v in vals:
    use(v)
    out = [bits(t).clone() for t in run() if torch.is_tensor(t)]
    torch.cuda.synchronize()
    if ref is None:
        ref = out
    assert all(torch.equal(a, b) for a, b in zip(out, ref)), f"{knob}={v} changed the output"
    timed(20)
res = {v: [] for v in vals}
for r in range(rounds):
    for v in vals:
        use(v)
        res[v].append(timed(iters))
    print(f"round {r}: " + "  ".join(f"{knob}={v} {t[-1]:.1f}" for v, t in res.items()), flush=True)
for v, t in res.items():
    print(f"{kind} {knob}={v}: median {sorted(t)[len(t) // 2]:.1f} us  min {min(t):.1f}")
