"""Per-linear timing at a model's prefill shapes (M = 2048 tokens): prepass, GEMM, output
quantization (OPT q/k/v with quantize_bmm_input), the whole W4A4Linear.forward, and the
fp16 F.linear (hipBLASLt).  python tools/model_shapes.py [llama2-7b|opt-1.3b] [M] [fp16|fp32]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "smoothquant-mixedprecision_amd")]
import torch  # noqa: E402

from smoothquant import ops  # noqa: E402
from smoothquant.fake_quant import W4A4Linear  # noqa: E402

model = sys.argv[1] if len(sys.argv) > 1 else "llama2-7b"
M = int(sys.argv[2]) if len(sys.argv) > 2 else 2048
DT = {"fp16": torch.float16, "fp32": torch.float32, "bf16": torch.bfloat16}[sys.argv[3] if len(sys.argv) > 3 else "fp16"]
if model == "llama2-7b":
    G, LIN = 64, [("qkvo", 4096, 4096, 4, False), ("gate_up", 4096, 11008, 2, False),
                  ("down", 11008, 4096, 1, False)]
else:
    G, LIN = 128, [("qkv", 2048, 2048, 3, True), ("out", 2048, 2048, 1, False),
                   ("fc1", 2048, 8192, 1, False), ("fc2", 8192, 2048, 1, False)]
dev = torch.device("cuda")


def t_ms(fn, it=30):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(it):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / it


tot = {"pre": 0.0, "gemm": 0.0, "oq": 0.0, "fwd": 0.0, "fp16": 0.0}
for name, K, N, count, oq in LIN:
    g = torch.Generator(device=dev).manual_seed(0)
    lin = torch.nn.Linear(K, N, bias=True).to(dev, DT)
    with torch.no_grad():
        lin.weight.copy_(torch.randn(N, K, generator=g, device=dev) * 0.02)
    x = torch.randn(M, K, generator=g, device=dev).to(DT)
    q = W4A4Linear.from_float(lin, weight_quant="per_group", act_quant="per_group",
                              quantize_output=oq, importance=x.float().abs().mean(0).cpu(),
                              salient_prop=0.05, group_size=G)
    pw = q.packed()
    a = ops.quant_act_fp(x, pw, "per_group", 4, G)
    bias = q.bias.reshape(-1)
    pre = t_ms(lambda: ops.quant_act_fp(x, pw, "per_group", 4, G))
    gemm = t_ms(lambda: ops.gemm_fq(a, pw, bias))
    y = ops.gemm_fq(a, pw, bias)
    oqt = t_ms(lambda: ops.fake_quant_inplace(y, "per_group", 4, G, pw.amap_fq, pw.nonsal, pw.S)) if oq else 0.0
    fwd = t_ms(lambda: q(x))
    w = lin.weight.detach()
    fp16 = t_ms(lambda: torch.nn.functional.linear(x, w, lin.bias))
    fl = 2 * M * N * K
    print(f"{name:8s} M={M} K={K} N={N}: prepass {pre*1e3:6.1f} us  gemm {gemm*1e3:6.1f} us "
          f"({fl/gemm/1e9:6.1f} TF/s)  outq {oqt*1e3:6.1f} us  forward {fwd*1e3:6.1f} us  "
          f"fp16 {fp16*1e3:6.1f} us ({fl/fp16/1e9:6.1f} TF/s)", flush=True)
    for k, v in (("pre", pre), ("gemm", gemm), ("oq", oqt), ("fwd", fwd), ("fp16", fp16)):
        tot[k] += count * v
print(f"{model} per decoder layer: prepass {tot['pre']*1e3:.1f} us, gemm {tot['gemm']*1e3:.1f} us, "
      f"output quant {tot['oq']*1e3:.1f} us, W4A4 forward {tot['fwd']*1e3:.1f} us, fp16 {tot['fp16']*1e3:.1f} us")
