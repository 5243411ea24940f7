"""Per-shape timing of the W4A4 linear at Llama-2-7B prefill shapes (M = 2048 tokens):
prepass (activation quant) + GEMM of this repo vs the PyTorch fp16 F.linear (hipBLASLt)
on the same shape.  python tools/llama_shapes.py [M] [group] [act]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "smoothquant-mixedprecision_amd")]
import torch  # noqa: E402

from smoothquant import ops  # noqa: E402
from smoothquant.fake_quant import W4A4Linear  # noqa: E402

M = int(sys.argv[1]) if len(sys.argv) > 1 else 2048
G = int(sys.argv[2]) if len(sys.argv) > 2 else 64
act = sys.argv[3] if len(sys.argv) > 3 else "per_group"
dev = torch.device("cuda")


def t_ms(fn, it=50):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(it):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / it


tot = {"pre": 0.0, "gemm": 0.0, "fwd": 0.0, "fp16": 0.0}
for name, K, N, count in [("qkvo", 4096, 4096, 4), ("gate_up", 4096, 11008, 2), ("down", 11008, 4096, 1)]:
    g = torch.Generator(device=dev).manual_seed(0)
    lin = torch.nn.Linear(K, N, bias=False).to(dev, torch.float16)
    with torch.no_grad():
        lin.weight.copy_(torch.randn(N, K, generator=g, device=dev) * 0.02)
    x = torch.randn(M, K, generator=g, device=dev).half()
    imp = x.float().abs().mean(0).cpu()
    q = W4A4Linear.from_float(lin, weight_quant="per_group", act_quant=act, importance=imp,
                              salient_prop=0.05, quant_bits=4, group_size=G)
    pw = q.packed()
    a = ops.quant_act_fp(x, pw, act, 4, G)
    pre = t_ms(lambda: ops.quant_act_fp(x, pw, act, 4, G))
    gemm = t_ms(lambda: ops.gemm_fq(a, pw, None))
    fwd = t_ms(lambda: q(x))
    w = lin.weight.detach()
    fp16 = t_ms(lambda: torch.nn.functional.linear(x, w))
    fl = 2 * M * N * K
    print(f"{name:8s} M={M} K={K} N={N}: prepass {pre*1e3:7.1f} us  gemm {gemm*1e3:7.1f} us "
          f"({fl/gemm/1e9:6.1f} TF/s)  forward {fwd*1e3:7.1f} us  fp16 {fp16*1e3:7.1f} us ({fl/fp16/1e9:6.1f} TF/s)")
    for k, v in (("pre", pre), ("gemm", gemm), ("fwd", fwd), ("fp16", fp16)):
        tot[k] += count * v
print(f"per decoder layer (7 linears): prepass {tot['pre']*1e3:.1f} us, gemm {tot['gemm']*1e3:.1f} us, "
      f"W4A4 forward {tot['fwd']*1e3:.1f} us, fp16 {tot['fp16']*1e3:.1f} us")
