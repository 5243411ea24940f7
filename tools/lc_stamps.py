"""Where the lane-contiguous quantizer's time goes: per-workgroup real-time stamps (100 MHz)
of the diagnostics build (SQMP_DIAG=1 build_ext.py; quant_lc_body's LC_STAMP points: entry,
prologue done, first pair interleaved / gathered / quantized / done, exit), for the Llama-2-7B
layer's quantizers at 2048 tokens and the config-2 C4 quantizer.

    SQMP_LIB_PATH=ab_tmp/diag.so python tools/lc_stamps.py

Per case: the launch's span (first entry -> last exit), the spread of workgroup entries, and
per phase the median / 90th percentile of each workgroup's time in it (µs)."""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "smoothquant-mixedprecision_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from smoothquant import ops  # noqa: E402
from smoothquant._lib import load  # noqa: E402
from smoothquant.fake_quant import W4A4Linear, link_siblings  # noqa: E402

lib = load()
f = lib.sqmp_diag_lc_stamps
f.argtypes = [ctypes.c_void_p, ctypes.c_int]
f.restype = ctypes.c_int
dev = torch.device("cuda")
PH = ["prologue", "interleave", "gather+stats", "quantize", "store", "rest pairs"]


def stamps():
    buf = np.zeros((8192, 8), dtype=np.uint64)
    assert f(buf.ctypes.data, 8192) == 0
    b = buf[buf[:, 0] > 0].astype(np.int64)
    return b


def report(name, run):
    for _ in range(5):
        run()
    torch.cuda.synchronize()
    assert f(None, 8192) == 0
    torch.cuda.synchronize()
    run()
    torch.cuda.synchronize()
    b = stamps()
    t0 = b[:, 0].min()
    span = (b[:, 6].max() - t0) / 100.0
    ent = (b[:, 0] - t0) / 100.0
    print(f"{name}: {len(b)} workgroups, span {span:.2f} us, entries spread "
          f"median {np.median(ent):.2f} max {ent.max():.2f} us, exits median "
          f"{np.median((b[:, 6] - t0) / 100.0):.2f} us")
    d = (b[:, 7] - b[:, 0]) / 100.0
    if d.min() > 0:
        print(f"   {'x + mask in':12s} median {np.median(d):6.2f}  p90 {np.percentile(d, 90):6.2f}  max {d.max():6.2f} us")
    for k in range(6):
        d = (b[:, k + 1] - b[:, k]) / 100.0
        print(f"   {PH[k]:12s} median {np.median(d):6.2f}  p90 {np.percentile(d, 90):6.2f}  max {d.max():6.2f} us")


def layer(K, N, M=2048, G=64, p=0.05, seed=0):
    g = torch.Generator(device=dev).manual_seed(seed)
    x = torch.randn(M, K, generator=g, device=dev)
    x[:, torch.randperm(K, generator=g, device=dev)[: K // 100]] *= 30.0
    x = x.half()
    lin = torch.nn.Linear(K, N, bias=False).to(dev, torch.float16)
    with torch.no_grad():
        lin.weight.copy_((torch.randn(N, K, generator=g, device=dev) * 0.02).half())
    imp = x[:512].float().abs().mean(0).cpu()
    q = W4A4Linear.from_float(lin, weight_quant="per_group", act_quant="per_group",
                              importance=imp, salient_prop=p, group_size=G)
    return q, x


with torch.no_grad():
    q, x = layer(4096, 4096)
    report("o_proj 2048x4096 (quantizer + GEMM forward)", lambda: q(x))
    q, x = layer(11008, 4096)
    report("down_proj 2048x11008", lambda: q(x))
    qs = [layer(4096, 4096, seed=s)[0] for s in (1, 2, 3)]
    _, xq = layer(4096, 4096, seed=1)
    link_siblings(*qs)
    report("q/k/v group 2048x4096", lambda: qs[0](xq.clone()))
    qc, xc, _ = bench.make_layer(dev, "per_group", seed=1)
    pw = qc.packed()
    report("config-2 C4 fused quantizer 16384x4096", lambda: ops.quant_act_c4(xc, pw, "per_group", 4, bench.G))
