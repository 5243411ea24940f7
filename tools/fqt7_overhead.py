"""Fixed per-tile cost of the activation-order GEMM (fqt7): HIP-event time of the config-2
GEMM (M=16384, N=4096, G=128, 10 % salient) at K = 2048 / 4096 / 8192; the K-linear part is
the steady-state stage cost, the intercept the per-round fixed cost (prologue, epilogue,
workgroup turnover) times the 4 rounds of 256 tiles.

    python tools/fqt7_overhead.py [iters]
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "smoothquant-mixedprecision_amd")]
import torch  # noqa: E402

from smoothquant import ops  # noqa: E402

iters = int(sys.argv[1]) if len(sys.argv) > 1 else 100
dev = torch.device("cuda")
res = []
for K in (2048, 4096, 8192):
    g = torch.Generator(device=dev).manual_seed(0)
    w = (torch.randn(4096, K, generator=g, device=dev) * 0.02).half()
    x = torch.randn(16384, K, generator=g, device=dev).half()
    sal = torch.argsort(x.float().abs().mean(0), descending=True)[: int(0.1 * K)].cpu()
    pw = ops.pack_weight(w, "per_group", 4, 128, sal)
    c4 = ops.quant_act_c4(x, pw, "per_group", 4, 128)
    run = lambda: ops.gemm_fqt(*c4, pw, None, 128)  # noqa: E731
    for _ in range(20):
        run()
    ts = []
    for _ in range(3):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(iters):
            run()
        b.record()
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b) / iters * 1e3)
    pos = pw.Kp - 0 + pw.S_pad
    res.append((K, sorted(ts)[1], c4[0].shape, pw.S_pad))
    print(f"K={K}: {sorted(ts)[1]:.1f} us  (codes {tuple(c4[0].shape)}, S_pad {pw.S_pad})", flush=True)
(k1, t1, _, _), (k2, t2, _, _), (k3, t3, _, _) = res
slope = (t3 - t2) / (k3 - k2)
print(f"per 1024 K positions {slope * 1024:.1f} us; intercept at K=0 {t2 - slope * k2:.1f} us "
      f"(= 4 rounds of fixed cost); K=2048 check: predicted {t2 - slope * (k2 - k1):.1f} vs {t1:.1f}")
