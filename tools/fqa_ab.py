"""Same-box A/B of the activation-order GEMMs at config 2 (M=16384, K=N=4096, G=128, 10 %
salient), interleaved rounds, HIP events on the launch stream:

  fqt7                       wp by LDS-DMA, act codes decoded per wave in registers (default)
  fqa:RB=r[,DIAG=d]          act codes decoded once per workgroup into LDS, wp in registers
                             (SQMP_FQA_RB = 4: 128 tokens x 512 rows; 2: 256 x 256); DIAG = the
                             timing diagnostics of a SQMP_DIAG=1 build (wrong results by design)
  dense:RB=r                 sqmp_gemm_fqa with Kq = 0: the same core on plain f16 operands
                             (16384 x 4160 -> 4096), against hipBLASLt's F.linear
  prepass:fqt7 / prepass:fqa the quantizer + permutation launch of either path

    [SQMP_DIAG_LIB=1] python tools/fqa_ab.py [rounds] [iters] [variant ...]
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "smoothquant-mixedprecision_amd")]
import torch  # noqa: E402

import bench  # noqa: E402
from smoothquant import ops  # noqa: E402
from smoothquant._lib import load, check, reload_knobs  # noqa: E402

rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 4
iters = int(sys.argv[2]) if len(sys.argv) > 2 else 200
variants = sys.argv[3:] or ["fqt7", "fqa:RB=4", "fqa:RB=2", "dense:RB=4", "dense:RB=2",
                            "hipblaslt:4160", "hipblaslt:4096", "prepass:fqt7", "prepass:fqa"]
dev = torch.device("cuda")
q, x, lin = bench.make_layer(dev, "per_group", seed=1)
pw = q.packed()
G = bench.G


def knobs(spec):
    kv = dict(a.split("=") for a in spec.split(",") if "=" in a) if spec else {}
    for k in ("RB", "DIAG"):
        if k in kv:
            os.environ["SQMP_FQA_" + k] = kv[k]
        else:
            os.environ.pop("SQMP_FQA_" + k, None)
    reload_knobs()
    return kv


def c4(fqa):
    ops.FQA = fqa
    return ops.quant_act_c4(x, pw, "per_group", 4, G)


ops_c4 = {"fqt7": c4(False), "fqa": c4(True)}
knobs("")
y7 = ops.gemm_fqt(*ops_c4["fqt7"], pw, lin.bias, G)

lib = load()
M, L, N = 16384, 4160, 4096
g = torch.Generator(device=dev).manual_seed(3)
xs = torch.randn(M, L, generator=g, device=dev).half()
W = (torch.randn(N, L, generator=g, device=dev) * 0.02).half()
wpt = torch.empty(lib.sqmp_fqa_wpt_elems(N, L, 0), dtype=torch.float16, device=dev)
check(lib.sqmp_pack_wpt(ops._p(W), ops._dtype_code(torch.float16), N, L, ops._p(wpt),
                        ops._stream(W)), "pack_wpt")
yd = torch.empty(M, N, dtype=torch.float16, device=dev)
x4, W4 = xs[:, :4096].contiguous(), W[:, :4096].contiguous()


def dense_core():
    check(lib.sqmp_gemm_fqa(None, None, ops._p(xs), ops._p(wpt), None, ops._p(yd),
                            ops._dtype_code(torch.float16), M, N, 0, L, 64, M, None,
                            ops._stream(xs)), "gemm_fqa dense")


def runner(v):
    kind, _, spec = v.partition(":")
    if kind == "fqt7":
        return lambda: ops.gemm_fqt(*ops_c4["fqt7"], pw, lin.bias, G), ""
    if kind == "fqa":
        return lambda: ops.gemm_fqt(*ops_c4["fqa"], pw, lin.bias, G), spec
    if kind == "dense":
        return dense_core, spec
    if kind == "hipblaslt":
        return ((lambda: torch.nn.functional.linear(xs, W)) if spec == "4160"
                else (lambda: torch.nn.functional.linear(x4, W4))), ""
    if kind == "prepass":
        return (lambda: c4(spec == "fqa")), ""
    raise ValueError(v)


def timed(fn, n):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(n):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / n * 1e3  # us


# correctness of every non-diagnostic variant first
yr = torch.nn.functional.linear(xs, W)
for v in variants:
    fn, spec = runner(v)
    kv = knobs(spec)
    if "DIAG" in kv:
        continue
    if v.startswith("fqa"):
        y = fn()
        d = float((y.float() - y7.float()).norm() / y7.float().norm())
        print(f"{v}: rel vs fqt7 {d:.2e}", flush=True)
        assert d < 1e-3
    if v.startswith("dense"):
        fn()
        d = float((yd.float() - yr.float()).norm() / yr.float().norm())
        print(f"{v}: rel vs F.linear {d:.2e}", flush=True)
        assert d < 1e-3

for v in variants:  # warm-up, clock settling
    fn, spec = runner(v)
    knobs(spec)
    timed(fn, 50)
res = {v: [] for v in variants}
for r in range(rounds):
    for v in variants:
        fn, spec = runner(v)
        knobs(spec)
        res[v].append(timed(fn, iters))
    print(f"round {r}: " + "  ".join(f"{k} {t[-1]:.1f}" for k, t in res.items()), flush=True)
flop = 2 * 16384 * 4096 * 4096
for k, t in res.items():
    med = sorted(t)[len(t) // 2]
    extra = f"  {flop / med / 1e6:.1f} TFLOP/s (2MNK at K=4096)" if k.startswith(("fqt7", "fqa")) else ""
    print(f"{k:24s} median {med:8.1f} us  min {min(t):8.1f}{extra}")
