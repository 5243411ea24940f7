"""Vendor reference points at config 2's shape (M=16384, K=N=4096): hipBLASLt fp16 F.linear
and, where torch exposes it, the FP8 e4m3 GEMM (torch._scaled_mm, per-tensor scales) -- the
rates our f16 and FP8 MFMA kernels are compared with.  python tools/vendor_gemm.py [iters]"""
import sys

import torch

M, K, N = 16384, 4096, 4096
iters = int(sys.argv[1]) if len(sys.argv) > 1 else 100
dev = torch.device("cuda")
stream = torch.cuda.current_stream(dev)
g = torch.Generator(device=dev).manual_seed(0)


def timeit(fn):
    for _ in range(20):
        fn()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    res = []
    for _ in range(3):
        a.record(stream)
        for _ in range(iters):
            fn()
        b.record(stream)
        b.synchronize()
        res.append(a.elapsed_time(b) / iters * 1e3)
    return sorted(res)[1]


flops = 2.0 * M * N * K
x = torch.randn(M, K, generator=g, device=dev).half()
w = (torch.randn(N, K, generator=g, device=dev) * 0.02).half()
t = timeit(lambda: torch.nn.functional.linear(x, w))
print(f"fp16 F.linear: {t:7.1f} us  {flops / t / 1e6:7.1f} TFLOP/s")
for name in ("float8_e4m3fn", "float8_e4m3fnuz"):
    if not hasattr(torch, name):
        continue
    try:
        f8 = getattr(torch, name)
        a8 = (torch.randint(-7, 8, (M, K), generator=g, device=dev)).to(f8)
        b8 = (torch.randint(-7, 8, (N, K), generator=g, device=dev)).to(f8)
        one = torch.ones((), device=dev)
        fn = lambda: torch._scaled_mm(a8, b8.t(), scale_a=one, scale_b=one,  # noqa: E731
                                      out_dtype=torch.float16)
        fn()
        t = timeit(fn)
        print(f"{name} _scaled_mm: {t:7.1f} us  {flops / t / 1e6:7.1f} TFLOP/s")
    except Exception as e:  # noqa: BLE001
        print(f"{name} _scaled_mm unavailable: {type(e).__name__}: {str(e)[:200]}")
