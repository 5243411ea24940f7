"""Locate fq7 mismatches: per case, the output columns / rows that differ from the fp32
product of the operands (debug aid)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "smoothquant-mixedprecision_amd"), os.path.join(ROOT, "tests")]
import torch  # noqa: E402

from test_gpu_fq7 import _layer, _ref  # noqa: E402
from smoothquant import ops  # noqa: E402

dev = torch.device("cuda")
cases = [(100, 1100, 520, 64, 0.1), (100, 1152, 520, 64, 0.1), (100, 1100, 512, 64, 0.1),
         (100, 1100, 520, 128, 0.1), (100, 1100, 520, 64, 0.0), (64, 512, 1024, 128, 0.1),
         (100, 1100, 256, 64, 0.1)]
for (M, K, N, Gs, p) in cases:
    q, lin, x = _layer(dev, M, K, N, Gs, p, torch.float16)
    pw = q.packed()
    a = ops.quant_act_fp(x, pw, "per_group", 4, Gs)
    y = torch.full((M, N), float("nan"), dtype=torch.float16, device=dev)
    y7 = ops.gemm_fq7(a, pw, lin.bias)
    ref = _ref(a, pw, lin.bias)
    bad = ~((y7.float() - ref).abs() <= 1e-2 * ref.abs().clamp_min(1.0))
    cols = bad.any(0).nonzero().flatten().tolist()
    rows = bad.any(1).nonzero().flatten().tolist()
    print(f"M{M} K{K} N{N} G{Gs} p{p} Kp{pw.Kp} S_pad{pw.S_pad} ngw{pw.ngw}: bad {int(bad.sum())} "
          f"cols {cols[:24]}{'...' if len(cols) > 24 else ''} ({len(cols)}) rows {rows[:12]} ({len(rows)})",
          flush=True)
