"""Same-box A/B of the activation-order GEMMs at config 2 (M=16384, K=N=4096, G=128, 10 %
salient): fqt7 (wp by LDS-DMA, act codes decoded per wave in registers) against fqa (act codes
decoded once per workgroup into LDS, wp in registers), interleaved rounds, HIP events on the
launch stream; then the DENSE core: sqmp_gemm_fqa with Kq = 0 (plain f16 operands, the act
tile by LDS-DMA, W in registers) on 16384 x 4160 -> 4096 against hipBLASLt's F.linear on the
same operands.

    python tools/fqa_ab.py [rounds] [iters]
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "smoothquant-mixedprecision_amd")]
import torch  # noqa: E402

import bench  # noqa: E402
from smoothquant import ops  # noqa: E402
from smoothquant._lib import load, check  # noqa: E402

rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 4
iters = int(sys.argv[2]) if len(sys.argv) > 2 else 200
dev = torch.device("cuda")
q, x, lin = bench.make_layer(dev, "per_group", seed=1)
pw = q.packed()
G = bench.G


def c4(fqa):
    ops.FQA = fqa
    return ops.quant_act_c4(x, pw, "per_group", 4, G)


ops_c4 = {"fqt7": c4(False), "fqa": c4(True)}
ys = {k: ops.gemm_fqt(*v, pw, lin.bias, G) for k, v in ops_c4.items()}
d = float((ys["fqa"].float() - ys["fqt7"].float()).norm() / ys["fqt7"].float().norm())
print(f"rel(fqa, fqt7) = {d:.2e}", flush=True)
assert d < 1e-3


def timed(fn, n):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(n):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / n * 1e3  # us


runs = {
    "fqt7 gemm": lambda: ops.gemm_fqt(*ops_c4["fqt7"], pw, lin.bias, G),
    "fqa gemm": lambda: ops.gemm_fqt(*ops_c4["fqa"], pw, lin.bias, G),
    "fqt7 prepass": lambda: c4(False),
    "fqa prepass": lambda: c4(True),
}
# dense core
lib = load()
M, L, N = 16384, 4160, 4096
g = torch.Generator(device=dev).manual_seed(3)
xs = torch.randn(M, L, generator=g, device=dev).half()
W = (torch.randn(N, L, generator=g, device=dev) * 0.02).half()
wpt = torch.empty(lib.sqmp_fqa_wpt_elems(N, L, 0), dtype=torch.float16, device=dev)
check(lib.sqmp_pack_wpt(ops._p(W), ops._dtype_code(torch.float16), N, L, ops._p(wpt),
                        ops._stream(W)), "pack_wpt")
yd = torch.empty(M, N, dtype=torch.float16, device=dev)


def dense_core():
    check(lib.sqmp_gemm_fqa(None, None, ops._p(xs), ops._p(wpt), None, ops._p(yd),
                            ops._dtype_code(torch.float16), M, N, 0, L, 64, M, None,
                            ops._stream(xs)), "gemm_fqa dense")


dense_core()
yr = torch.nn.functional.linear(xs, W)
print(f"dense core rel vs F.linear = {float((yd.float() - yr.float()).norm() / yr.float().norm()):.2e}",
      flush=True)
x4 = xs[:, :4096].contiguous()
W4 = W[:, :4096].contiguous()
runs["dense core 4160"] = dense_core
runs["hipBLASLt 4160"] = lambda: torch.nn.functional.linear(xs, W)
runs["hipBLASLt 4096"] = lambda: torch.nn.functional.linear(x4, W4)

for fn in runs.values():  # warm-up, ~2 s of clock settling
    timed(fn, 50)
res = {k: [] for k in runs}
for r in range(rounds):
    for k, fn in runs.items():
        res[k].append(timed(fn, iters))
    print(f"round {r}: " + "  ".join(f"{k} {v[-1]:.1f}" for k, v in res.items()), flush=True)
flop = 2 * 16384 * 4096 * 4096
for k, v in res.items():
    med = sorted(v)[len(v) // 2]
    extra = f"  {flop / med / 1e6:.1f} TFLOP/s (2MNK at K=4096)" if "gemm" in k else ""
    print(f"{k:18s} median {med:8.1f} us  min {min(v):8.1f}{extra}")
