"""GPU: the block-scaled FP8 path for per_token / per_tensor 4-bit activations.

* operands (SQMP_OUT_F8): the e4m3 act codes decode to integers c with D(c * sa) equal to
  the oracle's q_x BIT-EXACT at every non-salient column, 0 at salient and padding
  positions; the exact salient columns land in xs unchanged.
* y: relative Frobenius error vs the oracle product within the integer-path tolerance of
  test_gpu_parity (TOL_F8: the scales are factored out of the sum)."""
import zlib

import numpy as np
import pytest
import torch

from oracle import fake_quant_oracle as O
from test_gpu_parity import TOL_F8, TORCH_DT, _dev, _rand_inputs, bits_equal, make_layer, rel, to_np, to_t

pytestmark = pytest.mark.gpu


def e4m3_to_float(b):
    b = np.asarray(b, np.int64)
    s = np.where(b >> 7, -1.0, 1.0)
    e = (b >> 3) & 15
    m = b & 7
    v = np.where(e == 0, m / 8.0 * 2.0 ** -6, (1 + m / 8.0) * 2.0 ** (e - 7))
    return s * v


OPERAND_CASES = [
    # dtype, act, p, G, M, K, N
    ("fp16", "per_token", 0.05, 128, 67, 1024, 256),
    ("fp16", "per_tensor", 0.10, 64, 130, 2048, 384),
    ("bf16", "per_token", 0.10, 128, 64, 1024, 256),
    ("bf16", "per_tensor", 0.0, 256, 33, 512, 256),
    ("fp16", "per_token", 0.05, 128, 31, 1032, 256),     # K % 128 != 0: padding positions
]


@pytest.mark.parametrize("case", OPERAND_CASES, ids=[f"{c[0]}-{c[1]}-p{c[2]}-G{c[3]}-{c[4]}x{c[5]}" for c in OPERAND_CASES])
def test_f8_operands_exact(case):
    dev = _dev()
    from smoothquant import ops
    dt, aq, p, Gs, M, K, N = case
    D = O.DT(dt)
    W, x, imp, _ = _rand_inputs(zlib.crc32(repr(case).encode()), M, K, N, False)
    W, x = D.rnd(W), D.rnd(x)
    q = make_layer(W, None, dt, dev, weight_quant="per_group", act_quant=aq,
                   importance=torch.from_numpy(imp), salient_prop=p, quant_bits=4, group_size=Gs)
    pw = q.packed()
    a8, sa, xs = ops.quant_act_f8(to_t(x, dt, dev), pw, aq, 4)
    codes = e4m3_to_float(a8.cpu().numpy())
    assert np.all(codes == np.round(codes)) and np.abs(codes).max() <= 7
    sa = sa.cpu().numpy()
    sal = O.select_salient(imp, p)
    qx = D.f32(O.quantize_input(x, aq, 4, Gs, sal, D))
    amap = pw.amap.cpu().numpy()
    v = amap >= 0
    got = D.f32(D.rnd(codes[:, v] * sa[:, None]))
    assert bits_equal(got, qx[:, amap[v]])
    assert np.all(codes[:, ~v] == 0)
    if sal is not None:
        assert bits_equal(to_np(xs[:, :pw.S]), D.f32(x)[:, sal])


GEMM_CASES = [
    # dtype, act, p, G, M, K, N, bias
    ("fp16", "per_token", 0.10, 128, 1000, 4096, 640, True),
    ("fp16", "per_token", 0.05, 64, 257, 2048, 300, False),
    ("fp16", "per_tensor", 0.05, 256, 128, 1024, 512, True),
    ("fp16", "per_token", 0.0, 128, 300, 1024, 256, True),      # no salient tail
    ("fp16", "per_token", 0.10, 128, 1, 1024, 256, True),       # one row
    ("bf16", "per_token", 0.10, 128, 512, 2048, 1024, True),
    ("bf16", "per_tensor", 0.02, 64, 77, 1024, 128, False),
]


@pytest.mark.parametrize("case", GEMM_CASES, ids=[f"{c[0]}-{c[1]}-p{c[2]}-G{c[3]}-{c[4]}x{c[5]}x{c[6]}" for c in GEMM_CASES])
def test_f8_gemm_vs_oracle(case):
    dev = _dev()
    from smoothquant import ops
    dt, aq, p, Gs, M, K, N, bias = case
    D = O.DT(dt)
    W, x, imp, b = _rand_inputs(zlib.crc32(repr(case).encode()), M, K, N, bias)
    W, x = D.rnd(W), D.rnd(x)
    b = D.rnd(b) if b is not None else None
    q = make_layer(W, b, dt, dev, weight_quant="per_group", act_quant=aq,
                   importance=torch.from_numpy(imp), salient_prop=p, quant_bits=4, group_size=Gs)
    assert ops.f8_eligible(q.packed(), aq, 4)
    sal = O.select_salient(imp, p)
    w_hat = O.w4a4_from_float(W, "per_group", 4, Gs, sal, D)
    qx = O.quantize_input(x, aq, 4, Gs, sal, D)
    want = D.f32(O.linear(qx, w_hat, b, D))
    q.kernel = "f8"
    y = to_np(q(to_t(x, dt, dev)))
    assert rel(y, want) < TOL_F8[dt], rel(y, want)


@torch.no_grad()
def test_f8_full_size_config2_per_token():
    """BASELINE config 2 with per_token activations on the FP8 path (the default for this
    layer): y against an fp64 product of the faithful operands (the per_token q_x, which
    test_gpu_parity pins bit-exact, and W_hat) at M = 16384, K = N = 4096; and the e4m3
    codes of sampled rows decode to that q_x exactly."""
    dev = _dev()
    from smoothquant import ops
    from smoothquant.fake_quant import W4A4Linear
    M, K, N, Gs, p = 16384, 4096, 4096, 128, 0.10
    gen = torch.Generator(device=dev).manual_seed(5)
    lin = torch.nn.Linear(K, N, bias=True).to(dev, torch.float16)
    with torch.no_grad():
        lin.weight.copy_((torch.randn(N, K, generator=gen, device=dev) * 0.02).half())
        lin.bias.copy_((torch.randn(N, generator=gen, device=dev) * 0.01).half())
    x = torch.randn(M, K, generator=gen, device=dev)
    x[:, torch.randperm(K, generator=gen, device=dev)[:41]] *= 30
    x = x.half()
    imp = x[:2048].float().abs().mean(0).cpu()
    q = W4A4Linear.from_float(lin, weight_quant="per_group", act_quant="per_token",
                              importance=imp, salient_prop=p, group_size=Gs)
    pw = q.packed()
    assert ops.f8_eligible(pw, "per_token", 4)
    q.kernel = "f8"
    y = q(x)
    a = ops.quant_act_fp(x, pw, "per_token", 4, Gs)
    b_full = torch.cat([ops.dequant_weight_packed(pw), pw.wsal], dim=1)
    ref = torch.addmm(lin.bias.double(), a.double(), b_full.double().t())
    r = float((y.double() - ref).norm() / ref.norm())
    assert r < TOL_F8["fp16"], r
    a8, sa, _ = ops.quant_act_f8(x, pw, "per_token", 4)
    rows = torch.arange(0, M, 509, device=dev)
    codes = torch.from_numpy(e4m3_to_float(a8[rows].cpu().numpy()))
    dec = (codes * sa[rows].cpu().double()[:, None]).half()  # D(c * sa): one rounding
    assert torch.equal(dec.float()[:, :pw.Kp], a[rows, :pw.Kp].float().cpu())


def test_per_token_k_not_multiple_of_8_falls_back():
    """per_channel weights + per_token acts (the reference's from_float defaults) with
    K % 8 != 0: kernel "auto" must take the faithful path (the e4m3 quantizer needs K % 8
    == 0) and match the oracle."""
    dev = _dev()
    from smoothquant import ops
    D = O.DT("fp16")
    g = np.random.default_rng(21)
    K, N, M = 100, 64, 33
    W = D.rnd(g.standard_normal((N, K)) * 0.02)
    b = D.rnd(g.standard_normal(N) * 0.01)
    imp = np.abs(g.standard_normal(K)).astype(np.float32)
    for p in (0.0, 0.05):
        q = make_layer(W, b, "fp16", dev, weight_quant="per_channel", act_quant="per_token",
                       importance=torch.from_numpy(imp), salient_prop=p)
        assert not ops.f8_eligible(q.packed(), "per_token", 4)
        x = D.rnd(g.standard_normal((M, K)))
        sal = O.select_salient(imp, p)
        w_hat = O.w4a4_from_float(W, "per_channel", 4, 128, sal, D)
        want = D.f32(O.w4a4_forward(x, w_hat, b, "per_token", 4, 128, sal, False, D))
        y = to_np(q(to_t(x, "fp16", dev)))
        assert rel(y, want) < 2e-3


@pytest.mark.parametrize("M,K,N,p", [(2048, 4096, 4096, 0.0), (2048, 11008, 4096, 0.05),
                                     (333, 4096, 1000, 0.10), (2048, 4096, 11008, 0.0)])
def test_f8_row_tiles_bit_identical(M, K, N, p, monkeypatch):
    """The FP8 GEMM's 128-row tiles (the default where 256-row tiles leave CUs idle: the
    2048-token Llama shapes) and its 256-row tiles: the same K order per output, so y and the
    fused column maxima are bit-identical, with and without the salient tail, ragged M / N."""
    import torch
    from smoothquant import _lib, ops
    from smoothquant.fake_quant import W4A4Linear
    if not torch.cuda.is_available():
        pytest.skip("no ROCm device")
    dev = torch.device("cuda")
    gen = torch.Generator(device=dev).manual_seed(M + N)
    lin = torch.nn.Linear(K, N, bias=True).to(dev, torch.float16)
    with torch.no_grad():
        lin.weight.copy_((torch.randn(N, K, generator=gen, device=dev) * 0.02).half())
        lin.bias.copy_((torch.randn(N, generator=gen, device=dev) * 0.01).half())
    x = torch.randn(M, K, generator=gen, device=dev).half()
    q = W4A4Linear.from_float(lin, weight_quant="per_group", act_quant="per_token",
                              importance=x[:256].float().abs().mean(0).cpu(), salient_prop=p,
                              group_size=128)
    pw = q.packed()
    a8, sa, xs = ops.quant_act_f8(x, pw, "per_token", 4)
    b = lin.bias.detach()
    out = {}
    for tm in ("128", "256"):
        monkeypatch.setenv("SQMP_F8_TM", tm)
        _lib.reload_knobs()
        cm = torch.zeros(N, dtype=torch.int32, device=dev)
        y = ops.gemm_f8(a8, sa, xs, pw, b, colmax=cm)
        out[tm] = (y, cm)
    monkeypatch.delenv("SQMP_F8_TM")
    _lib.reload_knobs()
    assert torch.equal(out["128"][0], out["256"][0])
    assert torch.equal(out["128"][1], out["256"][1])
    y_auto = ops.gemm_f8(a8, sa, xs, pw, b)
    assert torch.equal(y_auto, out["256"][0])
