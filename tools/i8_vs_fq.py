"""Is the integer GEMM (kernel="i8": int8 act codes x int4 weight codes on the i8 MFMA) the
fastest path for any shape?  It is the only exact route that factors the scales out for
8-bit per_token activations (the W4A8 idiom with per_token acts); "auto" takes the faithful
fq GEMM there.  Times whole forwards (quantizer + GEMM, HIP events) of kernel="i8" against
kernel="auto" (fq / fq7) for 8-bit and 4-bit per_token activations at config 2 and the
Llama-2-7B 2048-token shapes.  python tools/i8_vs_fq.py"""
import os
import sys
from functools import partial

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "smoothquant-mixedprecision_amd")]
import torch  # noqa: E402

import bench  # noqa: E402
from smoothquant import fake_quant as FQ  # noqa: E402
from smoothquant.fake_quant import W4A4Linear  # noqa: E402

dev = torch.device("cuda")
stream = torch.cuda.current_stream(dev)
for M, K, N, G, p in ((16384, 4096, 4096, 128, 0.10), (2048, 4096, 4096, 64, 0.05),
                      (2048, 4096, 11008, 64, 0.05), (2048, 11008, 4096, 64, 0.05)):
    gen = torch.Generator(device=dev).manual_seed(1)
    x = torch.randn(M, K, generator=gen, device=dev).half()
    lin = torch.nn.Linear(K, N).to(dev, torch.float16)
    with torch.no_grad():
        lin.weight.copy_((torch.randn(N, K, generator=gen, device=dev) * 0.02).half())
    imp = x[:512].float().abs().mean(0).cpu()
    q = W4A4Linear.from_float(lin, weight_quant="per_group", act_quant="per_token",
                              importance=imp, salient_prop=p, group_size=G)
    for bits in (8, 4):
        q.act_quant = partial(FQ.quantize_activation_per_token_absmax, n_bits=bits)
        res = {}
        for kern in ("auto", "i8"):
            q.kernel = kern
            f = lambda: q(x)  # noqa: E731
            for _ in range(5):
                f()
            torch.cuda.synchronize()
            res[kern] = min(bench.time_events(f, 50, stream) for _ in range(3))
        print(f"{M}x{K}->{N} per_token {bits}-bit: auto {res['auto'] * 1e3:7.1f} us, "
              f"i8 {res['i8'] * 1e3:7.1f} us ({res['auto'] / res['i8']:.2f}x)", flush=True)
