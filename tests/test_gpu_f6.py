"""GPU: the FP6 (e2m3) path for per_token / per_tensor 4-bit activations (weight groups of
whole 128-position blocks).

* operands: the f6-packed act codes (SQMP_OUT_F6) decode to exactly the integer codes of the
  e4m3 path (SQMP_OUT_F8, pinned against the oracle's q_x in test_gpu_f8); the f6-packed
  weight codes (sqmp_pack_f6) to exactly the e4m3 weight codes (sqmp_pack_f8).
* y: gemm_f6 computes the same exact integer block sums with the same fp32 fold order as
  gemm_f8, so its output is BIT-IDENTICAL to gemm_f8's (which test_gpu_f8 checks against
  the oracle), on ragged shapes, without and with the salient tail, fp16 and bf16."""
import zlib

import numpy as np
import pytest
import torch

from oracle import fake_quant_oracle as O
from test_gpu_f8 import e4m3_to_float
from test_gpu_parity import TOL_I8, _dev, _rand_inputs, make_layer, rel, to_np, to_t

pytestmark = pytest.mark.gpu

E2M3 = {0: 0.0, 8: 1.0, 16: 2.0, 20: 3.0, 24: 4.0, 26: 5.0, 28: 6.0, 30: 7.0}


def f6_unpack(b):
    """[R, Kp * 3 / 4] f6-packed bytes -> [R, Kp] float values (e2m3, every pattern)."""
    b = np.asarray(b, np.uint8)
    R, W = b.shape
    blocks = b.reshape(R, W // 24, 24).astype(np.uint64)
    out = np.zeros((R, W // 24, 32), np.int64)
    # 192-bit little-endian block as three 64-bit words
    words = [sum(blocks[:, :, 8 * w + i] << np.uint64(8 * i) for i in range(8)) for w in range(3)]
    for e in range(32):
        bit = 6 * e
        w, sh = bit // 64, bit % 64
        v = (words[w] >> np.uint64(sh)) & np.uint64(63)
        if sh > 58:
            v |= (words[w + 1] << np.uint64(64 - sh)) & np.uint64(63)
        out[:, :, e] = v.astype(np.int64)
    codes = out.reshape(R, -1)
    s = np.where(codes & 32, -1.0, 1.0)
    e = (codes >> 3) & 3
    m = codes & 7
    val = np.where(e == 0, m / 8.0, (1 + m / 8.0) * 2.0 ** (e - 1))
    return s * val


CASES = [
    # dtype, act, weight_quant, p, G, M, K, N, bias
    ("fp16", "per_token", "per_group", 0.10, 128, 1000, 4096, 640, True),
    ("fp16", "per_token", "per_group", 0.05, 256, 257, 2048, 300, False),
    ("fp16", "per_tensor", "per_group", 0.05, 128, 128, 1024, 512, True),
    ("fp16", "per_token", "per_group", 0.0, 128, 300, 1024, 256, True),    # no salient tail
    ("fp16", "per_token", "per_group", 0.10, 128, 1, 1024, 256, True),     # one row
    ("fp16", "per_token", "per_channel", 0.05, 128, 513, 1536, 768, True),  # Gw = K
    ("bf16", "per_token", "per_group", 0.10, 128, 512, 2048, 1024, True),
    ("bf16", "per_tensor", "per_group", 0.02, 128, 77, 1024, 128, False),
]


def _layer(case):
    dev = _dev()
    dt, aq, wq, p, Gs, M, K, N, bias = case
    D = O.DT(dt)
    W, x, imp, b = _rand_inputs(zlib.crc32(repr(case).encode()), M, K, N, bias)
    W, x = D.rnd(W), D.rnd(x)
    b = D.rnd(b) if b is not None else None
    q = make_layer(W, b, dt, dev, weight_quant=wq, act_quant=aq,
                   importance=torch.from_numpy(imp), salient_prop=p, quant_bits=4, group_size=Gs)
    return q, to_t(x, dt, dev), (W, x, imp, b, D)


@pytest.mark.parametrize("case", CASES, ids=[f"{c[0]}-{c[1]}-{c[2]}-p{c[3]}-G{c[4]}-{c[5]}x{c[6]}x{c[7]}" for c in CASES])
@torch.no_grad()
def test_f6_operands_and_gemm_match_f8(case):
    from smoothquant import ops
    q, xt, (W, x, imp, b, D) = _layer(case)
    dt, aq = case[0], case[1]
    pw = q.packed()
    assert ops.f6_eligible(pw, aq, 4)
    a6, sa6, xs6 = ops.quant_act_f6(xt, pw, aq, 4)
    a8, sa8, xs8 = ops.quant_act_f8(xt, pw, aq, 4)
    assert a6.shape[1] == pw.Kp // 32 * 24
    assert np.array_equal(f6_unpack(a6.cpu().numpy()), e4m3_to_float(a8.cpu().numpy()))
    assert torch.equal(sa6, sa8)
    if pw.S:
        assert torch.equal(xs6[:, :pw.S], xs8[:, :pw.S])
    w6, _ = ops.f6_operands(pw)
    w8, _ = ops.f8_operands(pw)
    assert np.array_equal(f6_unpack(w6[:pw.N].cpu().numpy()), e4m3_to_float(w8[:pw.N].cpu().numpy()))
    bias = None if q.bias is None else q.bias.reshape(-1)
    y6 = ops.gemm_f6(a6, sa6, xs6, pw, bias)
    y8 = ops.gemm_f8(a8, sa8, xs8, pw, bias)
    assert torch.equal(y6.view(torch.int16), y8.view(torch.int16))
    # and the module's auto path takes f6 and agrees with the oracle product
    sal = O.select_salient(imp, case[3])
    w_hat = O.w4a4_from_float(W, case[2], 4, case[4], sal, D)
    want = D.f32(O.linear(O.quantize_input(x, aq, 4, case[4], sal, D), w_hat, b, D))
    y = q(xt.clone())
    assert torch.equal(y.view(torch.int16), y8.view(torch.int16))
    assert rel(to_np(y), want) < TOL_I8[dt]


@torch.no_grad()
def test_f6_full_size_config2_bit_identical_to_f8():
    """BASELINE config 2 (M = 16384, K = N = 4096, G = 128, p = 0.10) with per_token
    activations: the FP6 GEMM's y equals the FP8 GEMM's bit for bit."""
    dev = _dev()
    from smoothquant import ops
    from smoothquant.fake_quant import W4A4Linear
    M, K, N, Gs, p = 16384, 4096, 4096, 128, 0.10
    gen = torch.Generator(device=dev).manual_seed(6)
    lin = torch.nn.Linear(K, N, bias=True).to(dev, torch.float16)
    lin.weight.copy_((torch.randn(N, K, generator=gen, device=dev) * 0.02).half())
    lin.bias.copy_((torch.randn(N, generator=gen, device=dev) * 0.01).half())
    x = torch.randn(M, K, generator=gen, device=dev)
    x[:, torch.randperm(K, generator=gen, device=dev)[:41]] *= 30
    x = x.half()
    imp = x[:2048].float().abs().mean(0).cpu()
    q = W4A4Linear.from_float(lin, weight_quant="per_group", act_quant="per_token",
                              importance=imp, salient_prop=p, group_size=Gs)
    pw = q.packed()
    y6 = q(x)  # kernel "auto" -> FP6
    q.kernel = "f8"
    y8 = q(x)
    assert torch.equal(y6.view(torch.int16), y8.view(torch.int16))
    a6, sa, _ = ops.quant_act_f6(x, pw, "per_token", 4)
    a8, _, _ = ops.quant_act_f8(x, pw, "per_token", 4)
    rows = torch.arange(0, M, 509, device=dev)
    assert np.array_equal(f6_unpack(a6[rows].cpu().numpy()), e4m3_to_float(a8[rows].cpu().numpy()))


def test_f6_rejects_unaligned_groups():
    """Gw % 128 != 0 (e.g. group size 64): not f6-eligible, and the C entry refuses it."""
    dev = _dev()
    from smoothquant import ops
    q, xt, _ = _layer(("fp16", "per_token", "per_group", 0.05, 64, 64, 1024, 256, False))
    pw = q.packed()
    assert not ops.f6_eligible(pw, "per_token", 4) and ops.f8_eligible(pw, "per_token", 4)
    a6, sa, xs = ops.quant_act_f6(xt, pw, "per_token", 4)
    with pytest.raises(ValueError, match="gemm_f6"):  # SQMP_EUNSUPPORTED
        ops.gemm_f6(a6, sa, xs, pw, None)
