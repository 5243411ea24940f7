"""Generate the golden fixtures from the REFERENCE implementation itself.

Runs only in the survey/build container, where the read-only reference checkout lives
at /root/reference.  It loads `smoothquant/fake_quant.py` by file path (no bytecode is
written, nothing is copied), runs its quantizers and `W4A4Linear` on seeded synthetic
inputs on the CPU, and writes inputs + outputs as plain arrays to
`tests/golden/fake_quant_golden.npz` (no pickles; metadata is a JSON string).

Tie pinning: the reference calls `torch.argsort(...)` without `stable=True`; CPU
torch's unstable sort orders tied fp16/bf16 column maxima arbitrarily.  For
reproducible fixtures the reference module's `torch` global is wrapped so that every
`argsort` it makes is `stable=True` (ties -> lower index first).  That is the rule the
oracle and the HIP kernels implement; it is recorded in the metadata.

Usage:  python tests/golden/gen_golden.py      (refuses to run without /root/reference)
"""
from __future__ import annotations

import importlib.util
import json
import os
import sys

import numpy as np
import torch

REF = "/root/reference/smoothquant/fake_quant.py"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "fake_quant_golden.npz")

TORCH_DT = {"fp32": torch.float32, "fp16": torch.float16, "bf16": torch.bfloat16}


class _StableTorch:
    """Proxy for the `torch` module inside the reference: argsort is pinned stable."""

    def __init__(self, real):
        self._real = real

    def argsort(self, input, dim=-1, descending=False, stable=False):  # noqa: A002
        return self._real.argsort(input, dim=dim, descending=descending, stable=True)

    def __getattr__(self, name):
        return getattr(self._real, name)


def load_reference():
    if not os.path.exists(REF):
        raise SystemExit("gen_golden.py needs the reference checkout at /root/reference")
    sys.dont_write_bytecode = True
    spec = importlib.util.spec_from_file_location("_ref_fake_quant", REF)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    mod.torch = _StableTorch(torch)
    return mod


def to_np(t: torch.Tensor, dt: str):
    t = t.detach().cpu()
    if dt == "bf16":
        return t.view(torch.int16).numpy().view(np.uint16)
    return t.numpy()


def from_np(a: np.ndarray, dt: str) -> torch.Tensor:
    if dt == "bf16":
        return torch.from_numpy(a.view(np.int16).copy()).view(torch.bfloat16)
    return torch.from_numpy(a.copy())


def make_x(gen, shape, K, n_outlier, dt):
    x = torch.randn(*shape, K, generator=gen)
    if n_outlier:
        idx = torch.randperm(K, generator=gen)[:n_outlier]
        x[..., idx] *= 30.0
    return x.to(TORCH_DT[dt])


PRIM_CASES = [
    # name, fn, kind, dtype, shape, n_bits, group_size, special
    ("w_per_channel", "quantize_weight_per_channel_absmax", "w", "fp32", (24, 40), 4, None, None),
    ("w_per_channel_h", "quantize_weight_per_channel_absmax", "w", "fp16", (24, 40), 4, None, "zero_row"),
    ("w_per_tensor_b", "quantize_weight_per_tensor_absmax", "w", "bf16", (24, 40), 4, None, None),
    ("w_per_group", "quantize_weight_per_group_absmax", "w", "fp16", (16, 100), 4, 32, None),
    ("w_per_group_sort", "quantize_weight_per_group_absmax_sort", "w", "fp32", (16, 100), 4, 32, None),
    ("w_per_group_sort_h", "quantize_weight_per_group_absmax_sort", "w", "fp16", (16, 100), 4, 16, "ties"),
    ("w_per_group_sort_b", "quantize_weight_per_group_absmax_sort", "w", "bf16", (16, 130), 4, 64, "ties"),
    ("w_per_group_sort_8b", "quantize_weight_per_group_absmax_sort", "w", "fp16", (16, 96), 8, 32, None),
    ("a_per_token", "quantize_activation_per_token_absmax", "a", "fp16", (3, 5, 40), 4, None, "zero_row"),
    ("a_per_tensor", "quantize_activation_per_tensor_absmax", "a", "fp32", (12, 40), 4, None, None),
    ("a_per_group", "quantize_activation_per_group_absmax", "a", "bf16", (12, 70), 4, 32, None),
    ("a_per_group_sort", "quantize_activation_per_group_absmax_sort", "a", "fp32", (20, 100), 4, 32, None),
    ("a_per_group_sort_h", "quantize_activation_per_group_absmax_sort", "a", "fp16", (20, 100), 4, 16, "zero_col"),
    ("a_per_group_sort_hties", "quantize_activation_per_group_absmax_sort", "a", "fp16", (20, 100), 4, 32, "ties"),
    ("a_per_group_sort_b", "quantize_activation_per_group_absmax_sort", "a", "bf16", (2, 10, 130), 4, 64, "ties"),
    ("a_per_group_sort_8b", "quantize_activation_per_group_absmax_sort", "a", "fp16", (20, 96), 8, 32, None),
]

# dtype, weight_quant, act_quant, salient_prop, quantize_output, bits, G, x_shape, K, N, bias
LAYER_CASES = [
    ("fp32", "per_group", "per_group", 0.10, False, 4, 32, (40,), 160, 96, True),
    ("fp32", "per_group", "per_token", 0.10, False, 4, 64, (2, 20), 160, 96, True),
    ("fp32", "per_channel", "per_token", 0.0, False, 4, 128, (40,), 160, 96, True),
    ("fp32", "per_tensor", "per_tensor", 0.05, False, 4, 128, (40,), 160, 96, False),
    ("fp32", "per_group", "per_group", 0.10, True, 4, 32, (40,), 128, 128, True),
    ("fp32", "per_group", "per_group", 0.0, True, 4, 32, (40,), 128, 128, True),
    ("fp16", "per_group", "per_group", 0.10, False, 4, 32, (2, 24), 192, 128, True),
    ("fp16", "per_group", "per_group", 0.05, False, 4, 64, (48,), 192, 160, False),
    ("fp16", "per_group", "per_token", 0.10, False, 4, 64, (48,), 192, 128, True),
    ("fp16", "per_group", "per_tensor", 0.10, False, 4, 64, (48,), 192, 128, True),
    ("fp16", "per_channel", "per_token", 0.0, False, 4, 128, (48,), 192, 128, True),
    ("fp16", "per_channel", "per_group", 0.10, False, 4, 64, (48,), 192, 128, True),
    ("fp16", "per_group", "per_group", 0.10, True, 4, 32, (1, 32), 128, 128, True),
    ("fp16", "per_group", "per_group", 0.10, False, 8, 64, (48,), 192, 128, True),
    ("fp16", "per_tensor", "per_group", 0.0, False, 4, 64, (48,), 192, 128, True),
    ("bf16", "per_group", "per_group", 0.10, False, 4, 64, (2, 24), 192, 128, True),
    ("bf16", "per_group", "per_token", 0.05, False, 4, 32, (48,), 192, 128, False),
    ("bf16", "per_channel", "per_tensor", 0.0, True, 4, 128, (48,), 128, 128, True),
]


def gen_prim(ref, arrays, meta, i, case):
    name, fn, kind, dt, shape, bits, G, special = case
    gen = torch.Generator().manual_seed(100 + i)
    t = torch.randn(*shape, generator=gen) * (0.02 if kind == "w" else 1.0)
    if special == "zero_row":
        t.reshape(-1, shape[-1])[1].zero_()
    if special == "zero_col":
        t[..., 3] = 0
        t[..., 7] = 0
    if special == "ties":
        # repeat a handful of magnitudes so many columns share their column absmax
        levels = torch.tensor([0.5, 1.0, 2.0, 4.0]) * (0.02 if kind == "w" else 1.0)
        cols = shape[-1]
        pick = torch.randint(0, 4, (cols,), generator=gen)
        t = t.clamp(-1e-3, 1e-3) if kind == "w" else t.clamp(-0.1, 0.1)
        t2 = t.reshape(-1, cols)
        t2[0] = levels[pick] * torch.where(torch.rand(cols, generator=gen) > 0.5, 1.0, -1.0)
        t = t2.reshape(shape)
    t = t.to(TORCH_DT[dt])
    kw = {"n_bits": bits}
    if G is not None:
        kw["group_size"] = G
    out = getattr(ref, fn)(t.clone(), **kw)
    key = f"prim{i}"
    arrays[key + "_in"] = to_np(t, dt)
    arrays[key + "_out"] = to_np(out.reshape(shape) if out.numel() == t.numel() else out, dt)
    meta.append(dict(key=key, name=name, fn=fn, dtype=dt, shape=list(shape), n_bits=bits,
                     group_size=G, special=special, out_shape=list(out.shape)))


def gen_layer(ref, arrays, meta, i, case):
    dt, wq, aq, p, qo, bits, G, xshape, K, N, bias = case
    tdt = TORCH_DT[dt]
    gen = torch.Generator().manual_seed(1000 + i)
    lin = torch.nn.Linear(K, N, bias=bias)
    with torch.no_grad():
        lin.weight.copy_(torch.randn(N, K, generator=gen) * 0.02)
        if bias:
            lin.bias.copy_(torch.randn(N, generator=gen) * 0.01)
    lin = lin.to(tdt)
    w_in = lin.weight.detach().clone()
    b_in = lin.bias.detach().clone() if bias else None
    n_out = max(1, K // 64)
    x = make_x(gen, xshape, K, n_out, dt)
    imp = make_x(gen, (64,), K, n_out, "fp32").abs().mean(0)
    q = ref.W4A4Linear.from_float(lin, weight_quant=wq, act_quant=aq, quantize_output=qo,
                                  importance=imp if p > 0 else None, salient_prop=p,
                                  quant_bits=bits, group_size=G)
    # q_x exactly as forward builds it (fake_quant.py:291-304), via the reference's own
    # bound act quantizer.
    x2 = x.clone().reshape(-1, K)
    if q.salient_indices is not None:
        mask = torch.ones(K, dtype=torch.bool)
        mask[q.salient_indices] = False
        qx = x2.clone()
        qx[:, mask] = q.act_quant(x2[:, mask])
    else:
        qx = q.act_quant(x2.clone())
    y = q(x.clone())
    key = f"layer{i}"
    arrays[key + "_W"] = to_np(w_in, dt)
    arrays[key + "_x"] = to_np(x, dt)
    arrays[key + "_imp"] = imp.numpy().astype(np.float32)
    if bias:
        arrays[key + "_b"] = to_np(b_in, dt)
    arrays[key + "_What"] = to_np(q.weight, dt)
    arrays[key + "_qx"] = to_np(qx, dt)
    arrays[key + "_y"] = to_np(y, dt)
    sal = q.salient_indices
    arrays[key + "_sal"] = (sal.numpy().astype(np.int64) if sal is not None
                            else np.zeros((0,), np.int64))
    meta.append(dict(key=key, dtype=dt, weight_quant=wq, act_quant=aq, salient_prop=p,
                     quantize_output=qo, n_bits=bits, group_size=G, x_shape=list(x.shape),
                     K=K, N=N, bias=bias, has_salient=sal is not None))


def main():
    ref = load_reference()
    torch.set_num_threads(4)
    arrays, prim_meta, layer_meta = {}, [], []
    for i, c in enumerate(PRIM_CASES):
        gen_prim(ref, arrays, prim_meta, i, c)
    for i, c in enumerate(LAYER_CASES):
        gen_layer(ref, arrays, layer_meta, i, c)
    meta = dict(source="adithyab100/smoothquant-mixedprecision @ 2024-12-20, "
                       "smoothquant/fake_quant.py (loaded by path, CPU)",
                torch=torch.__version__, argsort="stable=True (ties -> lower index)",
                bf16_storage="uint16 bit patterns", prims=prim_meta, layers=layer_meta)
    arrays["meta_json"] = np.frombuffer(json.dumps(meta).encode(), dtype=np.uint8)
    np.savez_compressed(OUT, **arrays)
    print(f"wrote {OUT}: {os.path.getsize(OUT) / 1e6:.2f} MB, "
          f"{len(prim_meta)} primitive KATs, {len(layer_meta)} layer goldens")


if __name__ == "__main__":
    main()
