"""In-process A/B of the packed-order fq7 GEMM at the 2048-token Llama-2-7B shapes (and config
2) under a per-launch variable: interleaved rounds, HIP events, y bit-identical across variants.

    python tools/ab_fq7.py ENV=v1/v2/... [rounds] [iters]        (e.g. SQMP_FQ7_OPT=0/1/2/3)
    AB_STRICT=0: y within 1e-3 (relative Frobenius) instead of bit-identical (the K split)
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "smoothquant-mixedprecision_amd")]
import torch  # noqa: E402

from smoothquant import ops  # noqa: E402

var, vals = sys.argv[1].split("=")
vals = vals.split("/")
rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 4
iters = int(sys.argv[3]) if len(sys.argv) > 3 else 100
SHAPES = [(2048, 4096, 4096, 64, 0.05), (2048, 4096, 11008, 64, 0.05),
          (2048, 11008, 4096, 64, 0.05), (16384, 4096, 4096, 128, 0.10)]
dev = torch.device("cuda")
stream = torch.cuda.current_stream(dev)
for (M, K, N, G, p) in SHAPES:
    g = torch.Generator(device=dev).manual_seed(0)
    w = (torch.randn(N, K, generator=g, device=dev) * 0.02).half()
    x = torch.randn(M, K, generator=g, device=dev).half()
    sal = torch.argsort(x.float().abs().mean(0), descending=True)[: int(p * K)].cpu()
    pw = ops.pack_weight(w, "per_group", 4, G, sal)
    a = ops.quant_act_fp(x, pw, "per_group", 4, G)
    run = lambda: ops.gemm_fq(a, pw, None)  # noqa: E731
    ref = None
    for v in vals:
        os.environ[var] = v
        __import__("smoothquant._lib", fromlist=["_lib"]).reload_knobs()  # (knobs are read once at load)
        y = run()
        torch.cuda.synchronize()
        if ref is None:
            ref = y.clone()
        if os.environ.get("AB_STRICT", "1") == "1":
            assert torch.equal(y.view(torch.int16), ref.view(torch.int16)), f"{var}={v} changed y"
        else:  # (variants that add partial sums in another order: the K split, OPT bit 4)
            d = float((y.float() - ref.float()).norm() / ref.float().norm())
            assert d < 1e-3, f"{var}={v}: rel {d}"
    res = {v: [] for v in vals}
    for _ in range(rounds):
        for v in vals:
            os.environ[var] = v
            __import__("smoothquant._lib", fromlist=["_lib"]).reload_knobs()  # (knobs are read once at load)
            for _ in range(10):
                run()
            a0, b0 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a0.record(stream)
            for _ in range(iters):
                run()
            b0.record(stream)
            b0.synchronize()
            res[v].append(a0.elapsed_time(b0) / iters * 1e3)
    line = " | ".join(f"{var}={v}: {sorted(res[v])[len(res[v]) // 2]:7.1f} us" for v in vals)
    print(f"fq7 {M}x{K}->{N}: {line}", flush=True)
