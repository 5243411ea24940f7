"""GPU: sibling layers computed together (fake_quant.SiblingGroup).  q/k/v and gate/up quantize
the same input with the same salient set and act mode (fake_quant.py:291-304 depends only on x,
the salient set and the act mode; each weight keeps its own packed order, :157-207), so one
quantizer pass can write every sibling's operand (sqmp_quant_act_group) and one launch can run
every sibling's GEMM (sqmp_gemm_fq7_group).  Each must equal the sibling's own path bit for
bit; the module-level group must return exactly what the members compute alone."""
import os

import pytest
import torch

from test_gpu_sibling import _siblings

pytestmark = pytest.mark.gpu


def _dev():
    if not torch.cuda.is_available():
        pytest.skip("no ROCm device")
    return torch.device("cuda")


def _bits(t):
    return t.view(torch.int16)


@pytest.mark.parametrize("M,K,Ns,G,p,dt,mode", [
    (2048, 4096, (4096, 4096, 4096), 64, 0.05, torch.float16, "per_group"),   # Llama q/k/v
    (2048, 4096, (11008, 11008), 64, 0.05, torch.float16, "per_group"),       # Llama gate/up
    (333, 1024, (512, 256, 256), 128, 0.10, torch.float16, "per_group"),      # ragged M, GQA-like
    (300, 768, (768, 768, 768), 64, 0.10, torch.bfloat16, "per_group"),
    (128, 2048, (1024, 1024), 256, 0.05, torch.float16, "per_group_mean3std"),
    (64, 512, (256, 256), 16, 0.0, torch.float16, "per_group"),               # no salient, G=16
])
def test_group_quantizer_equals_own(M, K, Ns, G, p, dt, mode):
    dev = _dev()
    from smoothquant import ops
    layers, x = _siblings(dev, M, K, Ns, G, p, dt)
    pws = [q.packed() for q in layers]
    got = ops.quant_act_fp_group(x, pws, mode, 4, G)
    old = ops.SIB_REUSE
    try:
        ops.SIB_REUSE = False
        own = [ops.quant_act_fp(x.clone(), pw, mode, 4, G) for pw in pws]
    finally:
        ops.SIB_REUSE = old
    for a, b in zip(got, own):
        assert torch.equal(_bits(a), _bits(b))
    # the workspace is left clean: a following single call on another input is unaffected
    x2 = torch.randn_like(x)
    a1 = ops.quant_act_fp(x2, pws[1], mode, 4, G)
    a2 = ops.quant_act_fp(x2.clone(), pws[1], mode, 4, G)
    assert torch.equal(_bits(a1), _bits(a2))


@pytest.mark.parametrize("tm", ["128", "256"])
@pytest.mark.parametrize("M,K,Ns,G,p,dt", [
    (2048, 4096, (4096, 4096, 4096), 64, 0.05, torch.float16),
    (2048, 4096, (11008, 11008), 64, 0.05, torch.float16),
    (333, 1024, (512, 256, 256), 128, 0.10, torch.float16),
    (300, 768, (768, 768, 768), 64, 0.10, torch.bfloat16),
])
def test_group_gemm_equals_own(tm, M, K, Ns, G, p, dt, monkeypatch):
    """The grouped launch computes each member's tiles exactly as the member's own launch of
    the same kernel variant (the K split, SQMP_FQ7_KS, off here: a one-tile-per-CU member
    alone takes the split kernel by default, whose fp32 partial sums add in another order --
    test_gpu_fq7.py::test_fq7_ksplit bounds that difference)."""
    dev = _dev()
    from smoothquant import ops
    monkeypatch.setenv("SQMP_FQ7_KS", "0")
    monkeypatch.setenv("SQMP_FQ7G_TM", tm)
    __import__("smoothquant._lib", fromlist=["_lib"]).reload_knobs()  # (knobs are read once at load)
    layers, x = _siblings(dev, M, K, Ns, G, p, dt, seed=5)
    pws = [q.packed() for q in layers]
    a = ops.quant_act_fp_group(x, pws, "per_group", 4, G)
    biases = [q.bias.reshape(-1) for q in layers]
    ys = ops.gemm_fq7_group(a, pws, biases)
    for ai, pw, b, y in zip(a, pws, biases, ys):
        ref = ops.gemm_fq7(ai, pw, b)
        assert torch.equal(_bits(y), _bits(ref))


def test_linked_modules_forward():
    """link_siblings: the members return what they compute alone; the first call's stash is
    handed out once per input; an input changed in place, or another tensor, is computed
    again; calling a member twice on one input recomputes it."""
    dev = _dev()
    from smoothquant import ops
    from smoothquant.fake_quant import link_siblings
    layers, x = _siblings(dev, 512, 2048, (2048, 1024, 1024), 64, 0.05, torch.float16, seed=3)
    alone = [q(x) for q in layers]
    g = link_siblings(*layers)
    assert g is not None and all(q.__dict__["_sqmp_group"] is g for q in layers)
    x3 = x.view(1, 512, 2048)
    calls = []
    orig = ops.gemm_fq7_group

    def counting(*a, **k):
        calls.append(1)
        return orig(*a, **k)

    ops.gemm_fq7_group = counting
    try:
        ys = [q(x3) for q in layers]             # one grouped computation
        assert len(calls) == 1
        for y, r in zip(ys, alone):
            assert y.shape == (1, 512, r.shape[1])
            assert torch.equal(_bits(y.view(512, -1)), _bits(r))
        y0 = layers[0](x3)
        x3.mul_(0.5)                              # in place: k must not reuse the stash
        y1 = layers[1](x3)
        assert len(calls) == 3
        for m in layers:
            m.__dict__.pop("_sqmp_group")
        y1_ref = layers[1](x3)
        assert torch.equal(_bits(y1), _bits(y1_ref))
        assert torch.equal(_bits(y0.view(512, -1)), _bits(alone[0]))
    finally:
        ops.gemm_fq7_group = orig


def test_group_falls_back_when_not_covered():
    """A member with output quantization (or a rebound act quantizer that differs) makes the
    whole group compute alone -- same results as unlinked modules."""
    dev = _dev()
    from functools import partial

    from smoothquant import fake_quant as fq
    layers, x = _siblings(dev, 256, 1024, (512, 512), 64, 0.05, torch.float16, seed=9)
    layers[1].act_quant = partial(fq.quantize_activation_per_group_absmax_sort, n_bits=8,
                                  group_size=64)
    alone = [q(x) for q in layers]
    fq.link_siblings(*layers)
    assert layers[0].__dict__["_sqmp_group"]._plan(x) is None
    for q, r in zip(layers, alone):
        assert torch.equal(_bits(q(x)), _bits(r))


def test_stash_not_returned_after_member_changes():
    """after q_proj ran the group on x, rebinding k_proj's act quantizer
    (the reference's W4A8 idiom, fake_quant.py:246-263 partials), its output quantizer or its
    weight makes k_proj compute its own output -- never the stashed one."""
    dev = _dev()
    from functools import partial

    from smoothquant import fake_quant as fq
    layers, x = _siblings(dev, 256, 1024, (512, 512, 512), 64, 0.05, torch.float16, seed=11)
    fq.link_siblings(*layers)
    # (1) k's act quantizer rebound to 8 bits after q's call
    layers[0](x)
    layers[1].act_quant = partial(fq.quantize_activation_per_group_absmax_sort, n_bits=8,
                                  group_size=64)
    y1 = layers[1](x)
    for m in layers:
        m.__dict__.pop("_sqmp_group")
    assert torch.equal(_bits(y1), _bits(layers[1](x)))
    # (2) v's weight replaced after q's call
    layers2, x2 = _siblings(dev, 256, 1024, (512, 512, 512), 64, 0.05, torch.float16, seed=12)
    fq.link_siblings(*layers2)
    layers2[0](x2)
    layers2[2].weight = torch.randn(512, 1024, device=dev, dtype=torch.float16) * 0.02
    y2 = layers2[2](x2)
    for m in layers2:
        m.__dict__.pop("_sqmp_group")
    assert torch.equal(_bits(y2), _bits(layers2[2](x2)))
    # (3) output quantization switched on for k after q's call
    # (N == K: with salient channels the reference's output quantizer indexes y's columns by
    # the input's salient mask, fake_quant.py:311-314)
    layers3, x3 = _siblings(dev, 256, 1024, (1024, 1024, 1024), 64, 0.05, torch.float16, seed=13)
    fq.link_siblings(*layers3)
    layers3[0](x3)
    layers3[1].output_quant = layers3[1].act_quant
    y3 = layers3[1](x3)
    for m in layers3:
        m.__dict__.pop("_sqmp_group")
    assert torch.equal(_bits(y3), _bits(layers3[1](x3)))


def test_empty_batch_linked_and_fp32():
    """an empty batch through linked siblings (group_eligible refuses M == 0, each
    member computes alone) and through an fp32 layer (h2_planes_ok refuses M == 0) returns an
    empty output instead of raising."""
    dev = _dev()
    from smoothquant import fake_quant as fq
    from smoothquant import ops
    layers, x = _siblings(dev, 64, 512, (256, 256), 64, 0.05, torch.float16, seed=14)
    fq.link_siblings(*layers)
    x0 = x[:0]
    assert not ops.group_eligible([q.packed() for q in layers], "per_group", 4, 64, 0)
    for q in layers:
        y = q(x0)
        assert y.shape == (0, 256)
    lin = torch.nn.Linear(512, 256).to(dev, torch.float32)
    q32 = fq.W4A4Linear.from_float(lin, weight_quant="per_group", act_quant="per_group",
                                   importance=torch.rand(512), salient_prop=0.05, group_size=64)
    y = q32(torch.zeros(0, 512, device=dev))
    assert y.shape == (0, 256) and y.dtype == torch.float32
