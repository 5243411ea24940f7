"""GPU parity of the register-operand faithful GEMM (sqmp_gemm_fq7) against an fp32 product
of its own operands and against the LDS-staged faithful GEMM (sqmp_gemm_fq).

Both kernels compute x_hat . W_hat^T with the bit-exact operands (x_hat from the
activation quantizer, W_hat = D(code * scale) decoded in registers), fp32 accumulation and
one rounding to D; they differ only in accumulation order.  Tolerances (relative
Frobenius): vs the fp32 product of the operands fp16 2e-3, bf16 1e-2 (as TOL_FQ in
test_gpu_parity.py); fq7 vs fq 1e-3 (fp16) / 8e-3 (bf16); the fused output-quant
statistics (colmax) bit-exact against the column maxima of the stored y.
"""
import pytest
import torch

pytestmark = pytest.mark.gpu

TOL = {torch.float16: 2e-3, torch.bfloat16: 1e-2}
TOL_PAIR = {torch.float16: 1e-3, torch.bfloat16: 8e-3}


def _dev():
    if not torch.cuda.is_available():
        pytest.skip("no ROCm device")
    return torch.device("cuda")


def rel(a, b):
    a, b = a.double(), b.double()
    return float((a - b).norm() / b.norm().clamp_min(1e-30))


def _layer(dev, M, K, N, Gs, p, dt, wq="per_group", bias=True, seed=0):
    from smoothquant.fake_quant import W4A4Linear
    gen = torch.Generator(device=dev).manual_seed(seed)
    W = torch.randn(N, K, generator=gen, device=dev) * 0.02
    x = torch.randn(M, K, generator=gen, device=dev)
    out = torch.randperm(K, generator=gen, device=dev)[: max(1, K // 100)]
    x[:, out] *= 30
    imp = x[: min(M, 512)].abs().mean(0).cpu()
    lin = torch.nn.Linear(K, N, bias=bias).to(dev, dt)
    with torch.no_grad():
        lin.weight.copy_(W.to(dt))
        if bias:
            lin.bias.copy_((torch.randn(N, generator=gen, device=dev) * 0.01).to(dt))
    q = W4A4Linear.from_float(lin, weight_quant=wq, act_quant="per_group", importance=imp,
                              salient_prop=p, group_size=Gs)
    return q, lin, x.to(dt)


def _ref(a, pw, bias):
    from smoothquant import ops
    w = ops.dequant_weight_packed(pw)
    b_full = torch.cat([w, pw.wsal], dim=1) if pw.S_pad else w
    r = a.float() @ b_full.float().t()
    if bias is not None:
        r = r + bias.float()
    return r


CASES = [
    # M, K, N, G, p, dtype
    (1, 64, 8, 64, 0.0, torch.float16),
    (5, 100, 24, 32, 0.05, torch.float16),
    (64, 512, 256, 128, 0.10, torch.float16),
    (100, 1100, 520, 64, 0.10, torch.float16),
    (257, 1024, 1000, 128, 0.05, torch.float16),
    (300, 2048, 1536, 256, 0.0, torch.float16),
    (1000, 4096, 640, 128, 0.10, torch.float16),
    (2048, 4096, 4096, 64, 0.05, torch.float16),
    (333, 768, 3072, 128, 0.10, torch.bfloat16),
    (129, 1100, 264, 32, 0.10, torch.bfloat16),
    (2048, 11008, 512, 64, 0.05, torch.float16),
]


@pytest.mark.parametrize("M,K,N,Gs,p,dt", CASES)
def test_fq7_matches_operand_product_and_fq(M, K, N, Gs, p, dt):
    dev = _dev()
    from smoothquant import ops
    q, lin, x = _layer(dev, M, K, N, Gs, p, dt)
    pw = q.packed()
    assert ops.fq7_eligible(pw)
    a = ops.quant_act_fp(x, pw, "per_group", 4, Gs)
    y7 = ops.gemm_fq7(a, pw, lin.bias)
    fq7 = ops.FQ7_AUTO
    ops.FQ7_AUTO = False
    try:
        y6 = ops.gemm_fq(a, pw, lin.bias)
    finally:
        ops.FQ7_AUTO = fq7
    ref = _ref(a, pw, lin.bias)
    assert torch.isfinite(y7.float()).all()
    e_ref, e_pair = rel(y7, ref), rel(y7, y6)
    assert e_ref < TOL[dt], (e_ref, e_pair)
    assert e_pair < TOL_PAIR[dt], (e_ref, e_pair)


@pytest.mark.parametrize("wq", ["per_channel", "per_tensor"])
def test_fq7_other_weight_modes_no_bias(wq):
    dev = _dev()
    from smoothquant import ops
    q, lin, x = _layer(dev, 200, 640, 768, 128, 0.05, torch.float16, wq=wq, bias=False)
    pw = q.packed()
    if not ops.fq7_eligible(pw):
        pytest.skip(f"{wq}: Gw={pw.Gw} not an fq7 group size")
    a = ops.quant_act_fp(x, pw, "per_group", 4, 128)
    y7 = ops.gemm_fq7(a, pw, None)
    assert rel(y7, _ref(a, pw, None)) < TOL[torch.float16]


def test_fq7_colmax_is_column_max_of_y():
    dev = _dev()
    from smoothquant import ops
    q, lin, x = _layer(dev, 700, 2048, 1032, 128, 0.05, torch.float16)
    pw = q.packed()
    a = ops.quant_act_fp(x, pw, "per_group", 4, 128)
    cm = torch.zeros(pw.N + 8, dtype=torch.int32, device=dev)
    y = ops.gemm_fq7(a, pw, lin.bias, cm)
    want = y.float().abs().amax(0).view(torch.int32)
    assert torch.equal(cm[: pw.N], want)
    assert (cm[pw.N:] == 0).all()


def test_fq7_full_size_config2():
    """BASELINE config 2 (M=16384, K=N=4096, G=128, 10% salient) at full size."""
    dev = _dev()
    from smoothquant import ops
    q, lin, x = _layer(dev, 16384, 4096, 4096, 128, 0.10, torch.float16)
    pw = q.packed()
    a = ops.quant_act_fp(x, pw, "per_group", 4, 128)
    y7 = ops.gemm_fq7(a, pw, lin.bias)
    ref = _ref(a, pw, lin.bias)
    assert rel(y7, ref) < 2e-3
    fq7 = ops.FQ7_AUTO
    ops.FQ7_AUTO = False
    try:
        y6 = ops.gemm_fq(a, pw, lin.bias)
    finally:
        ops.FQ7_AUTO = fq7
    assert rel(y7, y6) < 1e-3


@pytest.mark.parametrize("env,vals", [
    ("SQMP_FQ7_OPT", ("3", "8", "0")),      # two workgroups per CU (8) vs one (3, 0)
    ("SQMP_FQ7_GROUP_M", ("4", "1", "8")),  # raster group sizes
])
@pytest.mark.parametrize("M,K,N", [(2048, 4096, 11008), (2048, 4096, 4096), (700, 2048, 1032)])
def test_fq7_variants_bit_identical(env, vals, M, K, N):
    """The launch variants only reorder work: y (and the fused column maxima) bit-identical.
    2048 x 4096 -> 11008 has 688 tiles of 128 x 256 (the two-per-CU default), -> 4096 256."""
    import os
    dev = _dev()
    from smoothquant import ops
    q, lin, x = _layer(dev, M, K, N, 64, 0.05, torch.float16)
    pw = q.packed()
    a = ops.quant_act_fp(x, pw, "per_group", 4, 64)
    old = os.environ.get(env)
    outs = []
    try:
        for v in vals:
            os.environ[env] = v
            __import__("smoothquant._lib", fromlist=["_lib"]).reload_knobs()  # (knobs are read once at load)
            cm = torch.zeros(pw.N + 8, dtype=torch.int32, device=dev)
            outs.append((ops.gemm_fq7(a, pw, lin.bias, cm), cm))
    finally:
        if old is None:
            os.environ.pop(env, None)
            __import__("smoothquant._lib", fromlist=["_lib"]).reload_knobs()  # (knobs are read once at load)
        else:
            os.environ[env] = old
            __import__("smoothquant._lib", fromlist=["_lib"]).reload_knobs()  # (knobs are read once at load)
    y0, c0 = outs[0]
    assert rel(y0, _ref(a, pw, lin.bias)) < TOL[torch.float16]
    for y, c in outs[1:]:
        assert torch.equal(y.view(torch.int16), y0.view(torch.int16))
        assert torch.equal(c, c0)


@pytest.mark.parametrize("ks", ["1", "2"])  # (1: one-tile-per-CU grids, the default; 2: all)
@pytest.mark.parametrize("M,K,N,Gs,p", [
    (2048, 4096, 4096, 64, 0.05),     # Llama o_proj: 256 tiles, one per CU
    (2048, 11008, 4096, 64, 0.05),    # down_proj: odd stage count (extra barrier in half 0)
    (700, 2048, 1032, 128, 0.05),     # ragged rows and columns
    (257, 256, 264, 64, 0.0),         # Kp = 256: the smallest split (two codes stages per half)
    (64, 192, 256, 64, 0.0),          # Kp < 256: no split, the unsplit kernel runs
])
def test_fq7_ksplit(ks, M, K, N, Gs, p, monkeypatch):
    """K split inside the workgroup (SQMP_FQ7_KS, OPT bit 4): the two halves' fp32 partial
    sums are added in another order than one pass, so y matches the unsplit kernel within the
    pair tolerance (not bit for bit), the fp32 operand product within TOL, and the fused
    column maxima are those of the stored y."""
    dev = _dev()
    from smoothquant import ops
    q, lin, x = _layer(dev, M, K, N, Gs, p, torch.float16)
    pw = q.packed()
    a = ops.quant_act_fp(x, pw, "per_group", 4, Gs)
    reload = __import__("smoothquant._lib", fromlist=["_lib"]).reload_knobs
    monkeypatch.setenv("SQMP_FQ7_KS", "0")  # the unsplit kernel
    reload()
    y0 = ops.gemm_fq7(a, pw, lin.bias)
    monkeypatch.setenv("SQMP_FQ7_KS", ks)
    reload()
    cm = torch.zeros(pw.N + 8, dtype=torch.int32, device=dev)
    y1 = ops.gemm_fq7(a, pw, lin.bias, cm)
    assert rel(y1, y0) < TOL_PAIR[torch.float16]
    assert rel(y1, _ref(a, pw, lin.bias)) < TOL[torch.float16]
    assert torch.equal(cm[: pw.N], y1.float().abs().amax(0).view(torch.int32))


@pytest.mark.parametrize("ks", ["2", "3"])
@pytest.mark.parametrize("Ns", [(4096, 4096, 4096), (11008, 11008)])
def test_fq7_ksplit_grouped(ks, Ns, monkeypatch):
    """The grouped sibling launch with the K split (A/B settings: 2 on every 128-row grid --
    q/k/v; 3 also 128-row tiles for gate/up): every member within the pair tolerance of the
    unsplit grouped launch."""
    dev = _dev()
    from smoothquant import ops
    from smoothquant.fake_quant import link_siblings
    layers = [_layer(dev, 2048, 4096, n, 64, 0.05, torch.float16, seed=3)[0] for n in Ns]
    _, _, x = _layer(dev, 2048, 4096, Ns[0], 64, 0.05, torch.float16, seed=3)
    link_siblings(*layers)
    reload = __import__("smoothquant._lib", fromlist=["_lib"]).reload_knobs
    outs = {}
    for v in ("0", ks):
        monkeypatch.setenv("SQMP_FQ7_KS", v)
        reload()
        xi = x.clone()  # (a new input object: the group runs again)
        outs[v] = [m(xi).clone() for m in layers]
    for y1, y0 in zip(outs[ks], outs["0"]):
        assert rel(y1, y0) < TOL_PAIR[torch.float16]
