"""GPU: the fp32 faithful GEMM on the 16-bit MFMA -- sqmp_gemm_h2 (row-scaled two-piece fp16
splits, three products) -- the F.linear of fake_quant.py:306 for fp32 models (OPT runs in
fp32 in the reference, run_experiments.py:146-156).

* the GEMM against an fp64 product of the SAME operands (the packed A operand and the
  packed-order W_hat + salient slice): relative Frobenius error <= 2e-6 -- the rounding level
  of an fp32 GEMM (the fp32 faithful tolerance of the parity tests is 1e-5); ragged M, N
  (N % 4 != 0, N < 128), with and without bias and salient tail;
* the fused output-quant column maxima (colmax) equal max |y| per column;
* the f32-MFMA kernel (F32_GEMM = "f32") and both agree to fp32 rounding level;
* the h2 split: h + l reproduces every scaled value within 2^-22 (+ the f16 subnormal floor),
  and every row's scaled maximum lies in [2^13, 2^14).
The layer-level fp32 cases of test_gpu_parity / test_gpu_configs (oracle, reference
goldens, config 1 and 3 layers) run through the default kernel (ops.F32_GEMM)."""
import numpy as np
import pytest
import torch

from test_gpu_parity import _dev, make_layer, rel

pytestmark = pytest.mark.gpu


CASES = [
    # weight_quant, act, p, G, M, K, N, bias, quantize_output
    ("per_group", "per_group", 0.10, 128, 512, 1024, 512, True, False),
    ("per_group", "per_group", 0.05, 128, 300, 2048, 200, False, False),
    ("per_channel", "per_token", 0.0, 128, 129, 768, 77, True, False),       # N % 4 != 0
    ("per_group", "per_group", 0.05, 128, 64, 2048, 2048, True, True),      # colmax fused
    ("per_tensor", "per_tensor", 0.10, 128, 1, 1024, 256, True, False),      # one row
]


def test_split2_f16_bound():
    from smoothquant import ops
    from smoothquant._lib import load
    dev = _dev()
    g = torch.Generator().manual_seed(4)
    R, L = 29, 160
    v = torch.randn(R, L, generator=g, dtype=torch.float64)
    v *= torch.exp2(torch.randint(-30, 30, (R, 1), generator=g).double())   # per-row range
    v *= torch.exp2(torch.randint(-12, 1, (R, L), generator=g).double())    # in-row spread
    v[3] = 0.0
    v = v.float().to(dev)
    ldr = 32
    out = torch.empty((2, ldr, L), dtype=torch.float16, device=dev)
    rexp = torch.empty(ldr, dtype=torch.int32, device=dev)
    ops.check(load().sqmp_split2_f16(ops._p(v), R, L, ldr, ops._p(out), ops._p(rexp),
                                     ops._stream(v)), "split2")
    torch.cuda.synchronize()
    e = rexp[:R].double().cpu()
    vs = v.double().cpu() * torch.exp2(e)[:, None]
    mx = vs.abs().amax(1)
    nz = mx > 0
    assert bool(((mx[nz] >= 2.0 ** 13) & (mx[nz] < 2.0 ** 14)).all())
    assert int(rexp[3]) == 0 and bool((rexp[R:] == 0).all())
    rec = out[0, :R].double().cpu() + out[1, :R].double().cpu()
    err = (rec - vs).abs()
    assert bool((err <= 2.0 ** -22 * vs.abs() + 2.0 ** -25).all()), err.max()


GEMMS = ["h2"]


@pytest.mark.parametrize("gemm", GEMMS)
@pytest.mark.parametrize("case", CASES)
def test_h2_matches_fp64_product(case, gemm):
    from smoothquant import ops
    wq, act, p, G, M, K, N, has_bias, oq = case
    run = ops.gemm_h2
    dev = _dev()
    rng = np.random.default_rng(11)
    W = (rng.standard_normal((N, K)) * 0.02).astype(np.float32)
    b = (rng.standard_normal(N) * 0.1).astype(np.float32) if has_bias else None
    x = rng.standard_normal((M, K)).astype(np.float32)
    x[:, rng.choice(K, max(1, K // 100), replace=False)] *= 30.0
    q = make_layer(W, b, "fp32", dev, weight_quant=wq, act_quant=act, quantize_output=oq,
                   importance=torch.from_numpy(np.abs(x).mean(0)), salient_prop=p, group_size=G)
    pw = q.packed()
    xt = torch.from_numpy(x).to(dev)
    a = ops.quant_act_fp(xt.clone(), pw, act, 4, G)
    bias = None if q.bias is None else q.bias.detach().reshape(-1)
    y = run(a, pw, bias)
    ref = a.double() @ ops._w_full(pw).double().t()
    if bias is not None:
        ref += bias.double()
    e = rel(y.double().cpu().numpy(), ref.cpu().numpy())
    assert e <= 2e-6, e
    # the f32-MFMA kernel on the same operands
    old = ops.F32_GEMM
    try:
        ops.F32_GEMM = "f32"
        y32 = ops.gemm_fq(a, pw, bias)
    finally:
        ops.F32_GEMM = old
    assert rel(y.double().cpu().numpy(), y32.double().cpu().numpy()) <= 2e-6
    # fused column maxima
    colmax = torch.zeros(N + 5, dtype=torch.int32, device=dev)
    y2 = run(a, pw, bias, colmax=colmax)
    assert torch.equal(y2, y)
    cm = colmax[:N].view(torch.float32)
    assert torch.equal(cm, y.abs().amax(0))
    assert bool((colmax[N:] == 0).all())


@pytest.mark.parametrize("gemm", GEMMS)
def test_h2_layer_forward_uses_h2_and_matches_f32_kernel(gemm):
    """W4A4Linear.forward on an fp32 layer takes the selected 16-bit-MFMA GEMM and agrees with
    the f32-MFMA kernel to fp32 rounding level, output quantization included."""
    from smoothquant import ops
    dev = _dev()
    rng = np.random.default_rng(5)
    K, N, M = 2048, 2048, 256
    W = (rng.standard_normal((N, K)) * 0.02).astype(np.float32)
    x = torch.from_numpy(rng.standard_normal((2, M // 2, K)).astype(np.float32)).to(dev)
    q = make_layer(W, np.zeros(N, np.float32), "fp32", dev, weight_quant="per_group",
                   act_quant="per_group", quantize_output=True,
                   importance=x.abs().mean((0, 1)).cpu(), salient_prop=0.05, group_size=128)
    old = ops.F32_GEMM
    try:
        ops.F32_GEMM = gemm
        y = q(x.clone())
        assert getattr(q.packed(), gemm) is not None
        ops.F32_GEMM = "f32"
        y32 = q(x.clone())
    finally:
        ops.F32_GEMM = old
    # the group scales of the output quantizer follow last-bit differences of max |y| (every
    # value of a group moves by a few ulps), and a 4-bit code flips where y sits on a
    # rounding boundary: count the flips (differences far above fp32 rounding)
    flips = ((y - y32).abs() > 1e-4 * y32.abs().max()).float().mean().item()
    assert flips < 0.01, flips


def test_h2_full_size_config2_fp32():
    """BASELINE config 2 in fp32 (M = 16384, K = N = 4096, G = 128, 10 % salient): the
    layer forward (quantizer + sqmp_gemm_h2) against the fp64 product of the same operands
    (the packed A operand and the packed-order W_hat + salient slice)."""
    from smoothquant import ops
    dev = _dev()
    M, K, N = 16384, 4096, 4096
    g = torch.Generator(device=dev).manual_seed(9)
    W = (torch.randn(N, K, generator=g, device=dev) * 0.02).cpu().numpy()
    x = torch.randn(M, K, generator=g, device=dev)
    x[:, torch.randperm(K, generator=g, device=dev)[:41]] *= 30.0
    q = make_layer(W, np.zeros(N, np.float32), "fp32", dev, weight_quant="per_group",
                   act_quant="per_group", importance=x[:2048].abs().mean(0).cpu(),
                   salient_prop=0.10, group_size=128)
    pw = q.packed()
    with torch.no_grad():
        y = q(x)
        a = ops.quant_act_fp(x, pw, "per_group", 4, 128)
        ref = a.double() @ ops._w_full(pw).double().t() + q.bias.detach().reshape(-1).double()
    e = rel(y.double().cpu().numpy(), ref.cpu().numpy())
    assert e <= 2e-6, e


@pytest.mark.parametrize("M,N", [(4096, 4096), (300, 520)])
def test_h2_raster_groups_bit_identical(M, N):
    """SQMP_H2_GROUP_M only reorders the tiles: y bit-identical for every group size."""
    import os
    from smoothquant import ops
    dev = _dev()
    rng = np.random.default_rng(5)
    K = 1024
    W = (rng.standard_normal((N, K)) * 0.02).astype(np.float32)
    x = rng.standard_normal((M, K)).astype(np.float32)
    q = make_layer(W, None, "fp32", dev, weight_quant="per_group", act_quant="per_group",
                   importance=torch.from_numpy(np.abs(x).mean(0)), salient_prop=0.05, group_size=128)
    pw = q.packed()
    a = ops.quant_act_fp(torch.from_numpy(x).to(dev), pw, "per_group", 4, 128)
    old = os.environ.get("SQMP_H2_GROUP_M")
    ys = []
    try:
        for g in ("4", "1", "8", "32"):
            os.environ["SQMP_H2_GROUP_M"] = g
            __import__("smoothquant._lib", fromlist=["_lib"]).reload_knobs()  # (knobs are read once at load)
            ys.append(ops.gemm_h2(a, pw, None))
    finally:
        if old is None:
            os.environ.pop("SQMP_H2_GROUP_M", None)
            __import__("smoothquant._lib", fromlist=["_lib"]).reload_knobs()  # (knobs are read once at load)
        else:
            os.environ["SQMP_H2_GROUP_M"] = old
            __import__("smoothquant._lib", fromlist=["_lib"]).reload_knobs()  # (knobs are read once at load)
    for y in ys[1:]:
        assert torch.equal(y.view(torch.int32), ys[0].view(torch.int32))


@pytest.mark.parametrize("M,K,N,p,has_bias", [
    (512, 1024, 512, 0.10, True),       # whole tiles
    (300, 2048, 200, 0.05, False),      # ragged M and N (N < one 256-row weight tile)
    (1, 1024, 260, 0.10, True),         # one row; N % 256 != 0
    (2048, 2048, 8192, 0.05, True),     # OPT-1.3B fc1
    (2048, 8192, 2048, 0.05, False),    # OPT-1.3B fc2
])
def test_h2d_bit_identical_to_h2(M, K, N, p, has_bias):
    """sqmp_gemm_h2d (pre-split activation planes by LDS-DMA, weight planes in registers)
    computes exactly sqmp_gemm_h2's sums in the same order: y and the fused column maxima
    bit-identical."""
    from smoothquant import ops
    dev = _dev()
    rng = np.random.default_rng(21)
    W = (rng.standard_normal((N, K)) * 0.02).astype(np.float32)
    b = (rng.standard_normal(N) * 0.1).astype(np.float32) if has_bias else None
    x = rng.standard_normal((M, K)).astype(np.float32)
    x[:, rng.choice(K, max(1, K // 100), replace=False)] *= 30.0
    q = make_layer(W, b, "fp32", dev, weight_quant="per_group", act_quant="per_group",
                   importance=torch.from_numpy(np.abs(x).mean(0)), salient_prop=p, group_size=128)
    pw = q.packed()
    L = pw.Kp + pw.S_pad
    assert L % 64 == 0 and N % 4 == 0
    a = ops.quant_act_fp(torch.from_numpy(x).to(dev), pw, "per_group", 4, 128)
    bias = None if q.bias is None else q.bias.detach().reshape(-1)
    old = ops.H2D
    try:
        ops.H2D = False
        c0 = torch.zeros(N, dtype=torch.int32, device=dev)
        y0 = ops.gemm_h2(a, pw, bias, colmax=c0)
        ops.H2D = True
        c1 = torch.zeros(N, dtype=torch.int32, device=dev)
        y1 = ops.gemm_h2(a, pw, bias, colmax=c1)
        y2 = ops.gemm_h2(a, pw, bias)
    finally:
        ops.H2D = old
    assert pw.h2d is not None
    assert torch.equal(y1.view(torch.int32), y0.view(torch.int32))
    assert torch.equal(y2.view(torch.int32), y0.view(torch.int32))
    assert torch.equal(c1, c0)


@pytest.mark.parametrize("act,K,M,p", [
    ("per_group", 1024, 300, 0.10),     # the register-staged wave quantizer
    ("per_token", 2048, 129, 0.05),
    ("per_group", 8192, 260, 0.05),     # rows longer than 4096: quant_f32w_kernel
    ("per_token", 8192, 64, 0.0),       # no salient channel
])
def test_quantizer_h2_planes_bit_identical(act, K, M, p):
    """SQMP_OUT_H2: the fp32 quantizer writes sqmp_gemm_h2d's planes and row exponents itself,
    bit-identical to sqmp_split2_f16 of its SQMP_OUT_FP operand; the layer forward on that
    path (quantizer -> planes -> sqmp_gemm_h2d, output quantization fused) equals the forward
    on the fp32 operand + sqmp_gemm_h2, bit for bit."""
    from smoothquant import ops
    from smoothquant._lib import load
    dev = _dev()
    rng = np.random.default_rng(31)
    N = 1024
    W = (rng.standard_normal((N, K)) * 0.02).astype(np.float32)
    x = rng.standard_normal((M, K)).astype(np.float32)
    x[:, rng.choice(K, max(1, K // 100), replace=False)] *= 30.0
    q = make_layer(W, (rng.standard_normal(N) * 0.1).astype(np.float32), "fp32", dev,
                   weight_quant="per_group", act_quant=act,
                   importance=torch.from_numpy(np.abs(x).mean(0)) if p else None,
                   salient_prop=p, group_size=128)
    pw = q.packed()
    assert ops.h2_planes_ok(pw, act, M, 128)
    xt = torch.from_numpy(x).to(dev)
    planes, aexp, m = ops.quant_act_fp(xt.clone(), pw, act, 4, 128, h2=True)
    a = ops.quant_act_fp(xt.clone(), pw, act, 4, 128)
    L = pw.Kp + pw.S_pad
    ldr = planes.shape[1]
    ref = torch.empty_like(planes)
    rexp = torch.empty(ldr, dtype=torch.int32, device=dev)
    ops.check(load().sqmp_split2_f16(ops._p(a), M, L, ldr, ops._p(ref), ops._p(rexp),
                                     ops._stream(a)), "split2")
    torch.cuda.synchronize()
    assert m == M
    assert torch.equal(aexp[:M], rexp[:M])
    assert torch.equal(planes[:, :M].view(torch.int16), ref[:, :M].view(torch.int16))
    # the layer forward, and (square weights: the reference's output quantizer needs N == K
    # with salient channels) with output quantization, its column maxima fused
    layers = [q]
    if K <= 2048:
        W2 = (rng.standard_normal((K, K)) * 0.02).astype(np.float32)
        layers.append(make_layer(W2, None, "fp32", dev, weight_quant="per_group", act_quant=act,
                                 quantize_output=True,
                                 importance=torch.from_numpy(np.abs(x).mean(0)) if p else None,
                                 salient_prop=p, group_size=128))
    old = ops.H2D
    try:
        for layer in layers:
            ops.H2D = True
            y1 = layer(xt.clone())
            ops.H2D = False
            y0 = layer(xt.clone())
            assert torch.equal(y1.view(torch.int32), y0.view(torch.int32))
    finally:
        ops.H2D = old
