"""The bucketed rank kernel (rank_bucket_kernel, SQMP_RT_BUCKET=1) against the all-pairs rank
table kernel: the sorted per_group quantizer's operand must be bit-identical whichever builds
the rank table (the stable argsort of fake_quant.py:113, ties to the lower list index) --
random keys, heavy ties (quantized inputs: few distinct column maxima), all columns equal,
zero columns, and the Llama shapes, through the single-layer and the sibling-group
quantizers, every owner lane count."""
import os

import pytest
import torch

from test_gpu_sibling import _dev, _siblings

pytestmark = pytest.mark.gpu


def _inputs(kind, x):
    if kind == "ties":      # column maxima from a handful of values
        return (x * 4).round() / 4
    if kind == "equal":     # every column the same maximum
        return torch.ones_like(x) * torch.where(torch.rand_like(x.float()) > 0.5, 1.0, -1.0).to(x.dtype)
    if kind == "zeros":     # a third of the columns zero
        y = x.clone()
        y[:, ::3] = 0
        return y
    return x


@pytest.mark.parametrize("btpo", ["1", "4", "16"])
@pytest.mark.parametrize("kind", ["random", "ties", "equal", "zeros"])
@pytest.mark.parametrize("M,K,Ns,G,p,dt", [
    (256, 1024, (512,), 64, 0.05, torch.float16),
    (2048, 4096, (4096, 4096, 4096), 64, 0.05, torch.float16),
    (300, 11008, (4096,), 64, 0.05, torch.float16),
    (129, 768, (768, 768), 128, 0.10, torch.bfloat16),
])
def test_bucketed_rank_bit_identical(M, K, Ns, G, p, dt, kind, btpo, monkeypatch):
    dev = _dev()
    from smoothquant import ops
    layers, x = _siblings(dev, M, K, Ns, G, p, dt, seed=5)
    x = _inputs(kind, x).contiguous()
    pws = [q.packed() for q in layers]
    monkeypatch.setenv("SQMP_RT_BTPO", btpo)
    __import__("smoothquant._lib", fromlist=["_lib"]).reload_knobs()  # (knobs are read once at load)
    outs = {}
    for on in ("0", "1"):
        monkeypatch.setenv("SQMP_RT_BUCKET", on)
        __import__("smoothquant._lib", fromlist=["_lib"]).reload_knobs()  # (knobs are read once at load)
        if len(pws) > 1:
            outs[on] = [a.clone() for a in ops.quant_act_fp_group(x, pws, "per_group", 4, G)]
        else:
            outs[on] = [ops.quant_act_fp(x, pws[0], "per_group", 4, G).clone()]
        torch.cuda.synchronize()
    for a, b in zip(outs["0"], outs["1"]):
        assert torch.equal(a.view(torch.int16), b.view(torch.int16))


@pytest.mark.parametrize("kind", ["random", "ties", "equal", "zeros"])
@pytest.mark.parametrize("M,K,Ns,G,p,dt", [
    (256, 1024, (512,), 64, 0.05, torch.float16),
    (2048, 4096, (4096, 4096, 4096), 64, 0.05, torch.float16),
    (300, 11008, (4096,), 64, 0.05, torch.float16),
    (129, 768, (768, 768), 128, 0.10, torch.bfloat16),
    (64, 192, (64,), 64, 0.05, torch.float16),
    (96, 16384, (256,), 128, 0.30, torch.float16),
])
def test_dense_rank_staging_bit_identical(M, K, Ns, G, p, dt, kind, monkeypatch):
    """The rank table with every column's key staged by coalesced loads and the salient
    columns masked (ties broken by column order = list order): the default 16-bit f16 / bf16
    key patterns ranked by a histogram of the keys (rank_hist16_kernel), the same keys compared
    two per packed op (SQMP_RT_HIST=0), and the 32-bit variant SQMP_RT_K16=0, against
    the list gather (SQMP_RT_DENSE=0): bit-identical operands, ragged K, a salient list longer than
    the first staging batch (30 % of 16384 columns)."""
    dev = _dev()
    from smoothquant import ops
    lib = __import__("smoothquant._lib", fromlist=["_lib"])
    layers, x = _siblings(dev, M, K, Ns, G, p, dt, seed=9)
    x = _inputs(kind, x).contiguous()
    pws = [q.packed() for q in layers]
    outs = {}
    # gather | dense 16-bit keys, histogram rank (default) | dense 16-bit keys, all-pairs
    # compares | dense 32-bit keys
    for on in ("0", "1", "a16", "k32"):
        monkeypatch.setenv("SQMP_RT_DENSE", "0" if on == "0" else "1")
        monkeypatch.setenv("SQMP_RT_K16", "0" if on == "k32" else "1")
        monkeypatch.setenv("SQMP_RT_HIST", "0" if on == "a16" else "1")
        lib.reload_knobs()
        if len(pws) > 1:
            outs[on] = [a.clone() for a in ops.quant_act_fp_group(x, pws, "per_group", 4, G)]
        else:
            outs[on] = [ops.quant_act_fp(x, pws[0], "per_group", 4, G).clone()]
        torch.cuda.synchronize()
    for v in ("1", "a16", "k32"):
        for a, b in zip(outs["0"], outs[v]):
            assert torch.equal(a.view(torch.int16), b.view(torch.int16))
