"""The config-2 activation-order prepass split into its kernels (for rocprofv3 --stats and
HIP-event timing): the fused quant_act_c4 (column max + rank table + C4 quantizer with the
weight permutation in one launch), then the quantizer alone (sqmp_quant_act_v2 OUT_C4) and
the permutation alone (sqmp_perm_weight_c4), each ITERS times.

    python tools/prepass_split.py [ITERS] [VAR=v1/v2/... [VAR=...]]

The optional further arguments sweep the permutation's per-launch tuning variables
(SQMP_PW_RB, SQMP_C4_QPERCU, SQMP_LC_PERCU): every combination is timed (fused and perm alone).
"""
import itertools
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "smoothquant-mixedprecision_amd")]
import torch  # noqa: E402

import bench  # noqa: E402
from smoothquant import _lib, ops  # noqa: E402
from smoothquant._lib import check, load  # noqa: E402

iters = int(sys.argv[1]) if len(sys.argv) > 1 else 50
dev = torch.device("cuda")
q, x, lin = bench.make_layer(dev, "per_group", seed=1)
pw = q.packed()
G, M, K = bench.G, bench.M, bench.K
lib = load()
stream = torch.cuda.current_stream(dev)


def t_us(fn, n=iters):
    for _ in range(5):
        fn()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record(stream)
    for _ in range(n):
        fn()
    b.record(stream)
    b.synchronize()
    return a.elapsed_time(b) / n * 1e3


fused = lambda: ops.quant_act_c4(x, pw, "per_group", 4, G)  # noqa: E731
c4 = fused()
codes, scales, xs, wp = c4
Kq = codes.shape[1] * 2
ngq = scales.shape[1]
e = ops._act_ws(dev, stream.cuda_stream, K, pw.Kp, ops._ws_bytes(M, K, pw.Kp))


def quant_only():
    st = lib.sqmp_quant_act_v2(ops._p(x), ops._dtype_code(x.dtype), M, K, ops.ACT_MODES["per_group"],
                               4, G, ops._p(pw.amap), pw.Kp, ops._p(pw.nonsal), ops._p(pw.salient),
                               pw.S, pw.S_pad, ops._p(pw.posmap),
                               _lib.QA_CLEAN_WS | _lib.QA_TILED, _lib.OUT_C4, ops._p(codes),
                               ops._p(scales), ops._p(xs), ops._p(e["buf"]), e["buf"].numel(),
                               ctypes.c_void_p(stream.cuda_stream))
    check(st, "quant_act_v2 C4")


def perm_only():
    st = lib.sqmp_perm_weight_c4(ops._p(e["buf"]), pw.K, pw.Kp, pw.S, pw.S_pad, ops._p(pw.codes),
                                 ops._p(pw.wscale), ops._p(pw.wsal), ops._dtype_code(pw.dtype),
                                 pw.N, pw.Gw, pw.ngw, ops._p(wp), ctypes.c_void_p(stream.cuda_stream))
    check(st, "perm_weight_c4")


wp_ref = wp.clone()
quant_only()
perm_only()
torch.cuda.synchronize()
assert torch.equal(wp.view(torch.int16), wp_ref.view(torch.int16))
xbytes = M * K * 2
qbytes = xbytes + codes.numel() + M * ngq * 2 + M * pw.S_pad * 2
pbytes = pw.N * pw.Kp // 2 + pw.N * (Kq + pw.S_pad) * 2
tf = t_us(fused)
tq = t_us(quant_only)
tp = t_us(perm_only)
print(f"fused quant_act_c4 (colmax + rank + quant|perm): {tf:7.1f} us")
print(f"quant_act_v2 OUT_C4 (colmax + rank + quant):     {tq:7.1f} us   quant bytes {qbytes/1e6:.1f} MB")
print(f"perm_weight_c4 alone:                             {tp:7.1f} us   {pbytes/1e6:.1f} MB = {pbytes/tp/1e3:.0f} GB/s")

if len(sys.argv) > 2:
    axes = [(kv.split("=")[0], kv.split("=")[1].split("/")) for kv in sys.argv[2:]]
    for combo in itertools.product(*[v for _, v in axes]):
        for (k, _), v in zip(axes, combo):
            os.environ[k] = v
            __import__("smoothquant._lib", fromlist=["_lib"]).reload_knobs()  # (knobs are read once at load)
        wp.zero_()
        perm_only()
        torch.cuda.synchronize()
        ok = torch.equal(wp.view(torch.int16), wp_ref.view(torch.int16))
        tf, tq, tp = t_us(fused), t_us(quant_only), t_us(perm_only)
        tag = " ".join(f"{k}={v}" for (k, _), v in zip(axes, combo))
        print(f"{tag:40s} fused {tf:7.1f} us  quant {tq:7.1f} us  perm {tp:7.1f} us ({pbytes/tp/1e3:.0f} GB/s)"
              f"{'' if ok else '  MISMATCH'}")
