"""Seeded inputs of the config-5 sweep golden cases that are stored by DIGEST (the wide
cases added in round 3: K up to 11008, G up to 1024), shared by the generator
(tests/golden/gen_golden_sweep.py, run against the reference in the survey container) and
the tests (tests/test_oracle_sweep.py, tests/test_gpu_sweep.py): the weight, bias,
activation and importance are re-drawn from torch's CPU generator (same seed, same torch
build on both sides), so the fixture holds only the reference's outputs -- sha256 digests
of W_hat and q_x and the small y -- instead of megabytes of random floats.
"""
from __future__ import annotations

import hashlib

import numpy as np
import torch

TORCH_DT = {"fp32": torch.float32, "fp16": torch.float16, "bf16": torch.bfloat16}


def _x(gen, shape, K, n_outlier, dt):
    x = torch.randn(*shape, K, generator=gen)
    if n_outlier:
        idx = torch.randperm(K, generator=gen)[:n_outlier]
        x[..., idx] *= 30.0
    return x.to(TORCH_DT[dt])


def case_inputs(i, case):
    """(W [N, K], b [N] or None, x [*x_shape, K], importance [K] fp32) of sweep case i,
    all in the case dtype except the importance (the generator's draw order)."""
    dt, sort, abits, p, G, xshape, K, N, bias = case
    gen = torch.Generator().manual_seed(5000 + i)
    w = (torch.randn(N, K, generator=gen) * 0.02).to(TORCH_DT[dt])
    b = (torch.randn(N, generator=gen) * 0.01).to(TORCH_DT[dt]) if bias else None
    n_out = max(1, K // 64)
    x = _x(gen, tuple(xshape), K, n_out, dt)
    imp = _x(gen, (64,), K, n_out, "fp32").abs().mean(0)
    return w, b, x, imp


def digest(a) -> str:
    """sha256 of the values as float32 bytes, -0.0 folded to +0.0 (a packed integer code 0
    dequantizes to +0.0 where the reference's fake quantizer may give -0.0)."""
    if isinstance(a, torch.Tensor):
        a = a.detach().cpu().float().numpy()
    a = np.ascontiguousarray(np.asarray(a, dtype=np.float32) + np.float32(0.0))
    return hashlib.sha256(a.tobytes()).hexdigest()
