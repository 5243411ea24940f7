"""Packed-format persistence without a GPU: the state plumbing of
W4A4Linear (buffers + `_extra_state`), the safe loader and the model-level swap."""
import os

import pytest
import torch
import torch.nn as nn

from smoothquant.checkpoint import FORMAT, load_quantized, save_quantized
from smoothquant.fake_quant import W4A4Linear, _PACKED_BUFFERS


def _fake_packed(K=64, N=32, S=3):
    """A W4A4Linear whose packed state is filled by hand (packing itself needs the GPU)."""
    q = W4A4Linear(K, N, bias=True, act_quant="per_group", quantize_output=False,
                   importance=torch.arange(K, dtype=torch.float32), salient_prop=S / K,
                   quant_bits=4, group_size=16)
    g = torch.Generator().manual_seed(0)
    Kp, S_pad, Np = 128, 128, 256
    q.w_codes = torch.randint(0, 255, (Np, Kp // 2), generator=g, dtype=torch.uint8)
    q.w_scale = torch.randn(Kp // 16, Np, generator=g).half()
    q.w_salient = torch.randn(N, S_pad, generator=g).half()
    q.w_perm = torch.randperm(Kp, generator=g).int()
    q.w_amap = q.w_perm.clone()
    q.w_amap_fq = torch.arange(K, dtype=torch.int32)
    q.w_nonsal = torch.arange(K - S, dtype=torch.int32)
    q.salient_i32 = q.salient_indices.int()
    q.bias = torch.randn(N, generator=g).half()
    q._meta = dict(N=N, K=K, S=S, S_pad=S_pad, Kp=Kp, Gw=16, ngw=Kp // 16, n_bits=4, wmode=2,
                   dtype=torch.float16)
    q.weight_quant_name = "per_group"
    q._random_init = False
    return q


def _same(a, b):
    sa, sb = a.state_dict(), b.state_dict()
    assert set(sa) == set(sb)
    for k in sa:
        if k.endswith("_extra_state"):
            ea, eb = sa[k], sb[k]
            assert {x: v for x, v in ea.items() if x != "salient_indices"} == \
                   {x: v for x, v in eb.items() if x != "salient_indices"}
            assert torch.equal(ea["salient_indices"], eb["salient_indices"])
        else:
            assert torch.equal(sa[k], sb[k]), k


def test_layer_state_roundtrip(tmp_path):
    q = _fake_packed()
    sd = q.state_dict()
    for name in _PACKED_BUFFERS:
        if getattr(q, name) is not None:
            assert name in sd
    assert "_extra_state" in sd and sd["_extra_state"]["format"] == W4A4Linear.EXTRA_FORMAT
    p = os.path.join(tmp_path, "layer.pt")
    torch.save(sd, p)
    sd2 = torch.load(p, weights_only=True)          # no pickled code in the checkpoint
    fresh = W4A4Linear(64, 32, bias=True)           # defaults differ from the saved layer
    fresh.load_state_dict(sd2, strict=True)
    _same(q, fresh)
    assert fresh.act_quant_name == "per_group" and fresh.weight_quant_name == "per_group"
    assert fresh.group_size == 16 and fresh._meta["dtype"] == torch.float16
    assert torch.equal(fresh.salient_indices, q.salient_indices)
    assert repr(fresh) == repr(q)


def test_model_checkpoint_swaps_linears(tmp_path):
    model = nn.Sequential(nn.Linear(64, 32), nn.ReLU(), nn.Linear(32, 8))
    model[0] = _fake_packed()
    p = os.path.join(tmp_path, "model.pt")
    save_quantized(model, p)
    target = nn.Sequential(nn.Linear(64, 32), nn.ReLU(), nn.Linear(32, 8))
    load_quantized(target, p)
    assert isinstance(target[0], W4A4Linear) and isinstance(target[2], nn.Linear)
    _same(model[0], target[0])
    assert torch.equal(target[2].weight, model[2].weight)


def test_checkpoint_rejects_foreign_files(tmp_path):
    p = os.path.join(tmp_path, "x.pt")
    torch.save({"format": "something-else"}, p)
    with pytest.raises(RuntimeError):
        load_quantized(nn.Linear(2, 2), p)
    assert FORMAT.startswith("sqmp-")


def test_loaded_bias_follows_the_checkpoint_device():
    """The packed buffers take the checkpoint's device; the bias must follow them, not the
    fresh module's construction device (a host bias pointer handed to the GEMM is a GPU
    memory fault).  The meta device stands in for the GPU here."""
    sd = {k: (v.to("meta") if isinstance(v, torch.Tensor) else v)
          for k, v in _fake_packed().state_dict().items()}
    fresh = W4A4Linear(64, 32, bias=True)
    assert fresh.bias.device.type == "cpu"
    fresh.load_state_dict(sd, strict=True)
    assert fresh.bias.device.type == "meta" and fresh.w_codes.device.type == "meta"


def test_host_operands_are_refused():
    from smoothquant import ops
    with pytest.raises(RuntimeError, match="on the GPU"):
        ops._p(torch.zeros(4))
    assert ops._p(None) is None
