"""Golden fixtures for BASELINE config 5 (W4A8 and the sort sweep), from the REFERENCE.

The reference has one `quant_bits` for both operands and wires only max-sorted groups, so
config 5 is expressed the way a user of the reference composes it:
  * W4A8:      from_float(quant_bits=4), then
               q.act_quant = partial(quantize_activation_per_group_absmax_sort, n_bits=8, ...)
  * sort=none: W_hat = quantize_weight_per_group_absmax(W) (fake_quant.py:29-53) with the
               salient columns restored (as from_float does, :347/:363-365), assigned to
               q.weight, and q.act_quant = partial(quantize_activation_per_group_absmax, ...)
               (:77-101).
The mean+3sigma sort exists only in the README, so it has no reference fixture (parity
unpinned; the oracle defines it).

Loads fake_quant.py by file path exactly like gen_golden.py (argsort pinned stable) and
writes tests/golden/sweep_golden.npz (plain arrays + JSON metadata, no pickles).

Usage:  python tests/golden/gen_golden_sweep.py   (needs /root/reference)
"""
from __future__ import annotations

import json
import os
import sys
from functools import partial

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gen_golden import TORCH_DT, load_reference, make_x, to_np  # noqa: E402
import sweep_inputs as SI  # noqa: E402

OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "sweep_golden.npz")

# cases from this index on are stored by digest (inputs re-drawn: tests/sweep_inputs.py)
DIGEST_FROM = 8
# dtype, sort (max|none), act_bits, salient_prop, G, x_shape, K, N, bias
CASES = [
    ("fp16", "max", 8, 0.05, 64, (48,), 256, 128, True),
    ("fp16", "none", 4, 0.05, 64, (48,), 256, 128, True),
    ("fp16", "none", 8, 0.10, 32, (2, 24), 192, 160, False),
    ("fp32", "none", 4, 0.10, 32, (40,), 160, 96, True),
    ("fp32", "max", 8, 0.10, 128, (40,), 320, 96, True),
    ("bf16", "max", 8, 0.05, 64, (48,), 256, 128, True),
    ("bf16", "none", 4, 0.05, 64, (48,), 256, 128, False),
    ("fp16", "max", 8, 0.0, 64, (48,), 256, 128, True),
    # round 3: the sweep's larger groups (run_experiments.py:262 goes to 1024), including
    # the Llama-2-7B down_proj width K = 11008 at G = 1024 (11 act groups, the weight's
    # last group padded by 256 zero columns) for W4A8, sort=none and W4A4 max
    ("fp16", "max", 8, 0.05, 256, (64,), 1024, 96, True),
    ("fp16", "none", 4, 0.05, 256, (64,), 1024, 96, True),
    ("fp16", "none", 8, 0.05, 256, (48,), 1000, 64, False),
    ("fp16", "max", 8, 0.05, 1024, (16,), 11008, 16, True),
    ("fp16", "none", 4, 0.05, 1024, (16,), 11008, 16, True),
    ("fp16", "max", 4, 0.05, 1024, (16,), 11008, 16, True),
    ("bf16", "none", 8, 0.05, 1024, (16,), 11008, 16, True),
    ("fp32", "max", 8, 0.05, 256, (40,), 1024, 64, True),
    ("fp16", "none", 8, 0.0, 1024, (24,), 4096, 32, False),
]


def gen_case(ref, arrays, meta, i, case):
    dt, sort, abits, p, G, xshape, K, N, bias = case
    if i >= DIGEST_FROM:
        # inputs re-drawn by the tests from the same seed (tests/sweep_inputs.py)
        w0, b0, x, imp = SI.case_inputs(i, case)
        lin = torch.nn.Linear(K, N, bias=bias).to(TORCH_DT[dt])
        with torch.no_grad():
            lin.weight.copy_(w0)
            if bias:
                lin.bias.copy_(b0)
    else:
        gen = torch.Generator().manual_seed(5000 + i)
        lin = torch.nn.Linear(K, N, bias=bias)
        with torch.no_grad():
            lin.weight.copy_(torch.randn(N, K, generator=gen) * 0.02)
            if bias:
                lin.bias.copy_(torch.randn(N, generator=gen) * 0.01)
        lin = lin.to(TORCH_DT[dt])
        n_out = max(1, K // 64)
        x = make_x(gen, xshape, K, n_out, dt)
        imp = make_x(gen, (64,), K, n_out, "fp32").abs().mean(0)
    w_in = lin.weight.detach().clone()
    b_in = lin.bias.detach().clone() if bias else None
    q = ref.W4A4Linear.from_float(lin, weight_quant="per_group", act_quant="per_group",
                                  importance=imp if p > 0 else None, salient_prop=p,
                                  quant_bits=4, group_size=G)
    if sort == "none":
        w = w_in.clone()
        sal = q.salient_indices
        keep = w[:, sal].clone() if sal is not None else None
        w_hat = ref.quantize_weight_per_group_absmax(w, n_bits=4, group_size=G)
        if sal is not None:
            w_hat[:, sal] = keep
        q.weight = w_hat
        act_fn = ref.quantize_activation_per_group_absmax
    else:
        act_fn = ref.quantize_activation_per_group_absmax_sort
    q.act_quant = partial(act_fn, n_bits=abits, group_size=G)
    x2 = x.clone().reshape(-1, K)
    if q.salient_indices is not None:
        mask = torch.ones(K, dtype=torch.bool)
        mask[q.salient_indices] = False
        qx = x2.clone()
        qx[:, mask] = q.act_quant(x2[:, mask])
    else:
        qx = q.act_quant(x2.clone())
    y = q(x.clone())
    key = f"sweep{i}"
    sal = q.salient_indices
    if i >= DIGEST_FROM:
        arrays[key + "_y"] = to_np(y, dt)
        arrays[key + "_sal"] = (sal.numpy().astype(np.int64) if sal is not None
                                else np.zeros((0,), np.int64))
        meta.append(dict(key=key, dtype=dt, sort=sort, w_bits=4, act_bits=abits,
                         salient_prop=p, group_size=G, x_shape=list(x.shape), K=K, N=N,
                         bias=bias, has_salient=sal is not None, index=i,
                         case=[dt, sort, abits, p, G, list(xshape), K, N, bias],
                         what_sha256=SI.digest(q.weight), qx_sha256=SI.digest(qx)))
        return
    arrays[key + "_W"] = to_np(w_in, dt)
    arrays[key + "_x"] = to_np(x, dt)
    arrays[key + "_imp"] = imp.numpy().astype(np.float32)
    if bias:
        arrays[key + "_b"] = to_np(b_in, dt)
    arrays[key + "_What"] = to_np(q.weight, dt)
    arrays[key + "_qx"] = to_np(qx, dt)
    arrays[key + "_y"] = to_np(y, dt)
    arrays[key + "_sal"] = (sal.numpy().astype(np.int64) if sal is not None
                            else np.zeros((0,), np.int64))
    meta.append(dict(key=key, dtype=dt, sort=sort, w_bits=4, act_bits=abits, salient_prop=p,
                     group_size=G, x_shape=list(x.shape), K=K, N=N, bias=bias,
                     has_salient=sal is not None))


def main():
    ref = load_reference()
    torch.set_num_threads(4)
    arrays, meta = {}, []
    for i, c in enumerate(CASES):
        gen_case(ref, arrays, meta, i, c)
    info = dict(source="adithyab100/smoothquant-mixedprecision @ 2024-12-20, "
                       "smoothquant/fake_quant.py (loaded by path, CPU)",
                torch=torch.__version__, argsort="stable=True (ties -> lower index)",
                bf16_storage="uint16 bit patterns", cases=meta)
    arrays["meta_json"] = np.frombuffer(json.dumps(info).encode(), dtype=np.uint8)
    np.savez_compressed(OUT, **arrays)
    print(f"wrote {OUT}: {os.path.getsize(OUT) / 1e6:.2f} MB, {len(meta)} cases")


if __name__ == "__main__":
    main()
