"""GPU parity of the activation-order faithful path (SQMP_OUT_C4 quantizer,
sqmp_perm_weight_c4, sqmp_gemm_fqt) against the packed-order path (quant_act_fp +
gemm_fq), whose operands are pinned bit-exactly to the reference (test_gpu_parity.py).

  * the activation operand: per row, the multiset of x_hat values over the non-salient
    columns (decoded from the int4 codes and group scales) is BIT-EXACT that of the
    packed-order operand, and the exact salient columns are identical;
  * the permuted weight: per row, the multiset of W_hat over the non-salient columns is
    bit-exact that of the dequantized packed weight, zeros past K - S, wsal after;
  * y: the same products summed in another order, relative Frobenius vs gemm_fq 1e-3
    (fp16) / 8e-3 (bf16), and vs the fp32 product of the path's own operands 2e-3 / 1e-2.

Both operand layouts: row-major (sqmp_gemm_fqt on fq6's structure) and tile-major
(SQMP_QA_TILED + sqmp_gemm_fqt7, untiled here before the same checks).
"""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _dev():
    if not torch.cuda.is_available():
        pytest.skip("no ROCm device")
    return torch.device("cuda")


def rel(a, b):
    a, b = a.detach().double(), b.detach().double()
    return float((a - b).norm() / b.norm().clamp_min(1e-30))


def _layer(dev, M, K, N, Gs, p, dt, wq="per_group", aq="per_group", seed=0):
    from smoothquant.fake_quant import W4A4Linear
    gen = torch.Generator(device=dev).manual_seed(seed)
    W = torch.randn(N, K, generator=gen, device=dev) * 0.02
    x = torch.randn(M, K, generator=gen, device=dev)
    out = torch.randperm(K, generator=gen, device=dev)[: max(1, K // 100)]
    x[:, out] *= 30
    imp = x[: min(M, 512)].abs().mean(0).cpu()
    lin = torch.nn.Linear(K, N, bias=True).to(dev, dt)
    with torch.no_grad():
        lin.weight.copy_(W.to(dt))
        lin.bias.copy_((torch.randn(N, generator=gen, device=dev) * 0.01).to(dt))
    q = W4A4Linear.from_float(lin, weight_quant=wq, act_quant=aq, importance=imp,
                              salient_prop=p, group_size=Gs)
    return q, lin, x.to(dt)


def decode_c4(codes, scales, Kq, G, dt):
    """int4 bpack codes [M, Kq/2] + D scales [Kq/G, Mp] -> x_hat [M, Kq] in act order."""
    M = codes.shape[0]
    w = codes.contiguous().view(torch.int32).view(M, Kq // 64, 8)  # dwords of each block
    pos = torch.arange(64, device=codes.device)
    kin = pos
    d = ((kin >> 3) & 1) * 4 + (kin >> 4)                    # bpack dword of position
    e = kin & 7
    sh = torch.where(e % 2 == 1, 16 + 4 * (e >> 1), 4 * (e >> 1))
    nib = (w[:, :, d] >> sh) & 0xF                          # [M, Kq/64, 64]
    code = (nib - 8).reshape(M, Kq).float()
    g = torch.arange(Kq, device=codes.device) // G
    s = scales[g.clamp_max(scales.shape[0] - 1)][:, :M].t().float()
    return (code * s).to(dt)                                 # D(code * s): exact in fp32


def untile_c4(codes_t, scales_t, xs_t, M, Kq, S_pad):
    """The tile-major operands (sqmp_pack_fq7 layouts, J = 2) -> row-major codes [M, Kq/2],
    scales [ngq, R], xs [M, S_pad]."""
    R = codes_t.shape[0]
    KB = Kq // 64
    w = codes_t.contiguous().view(torch.int32).reshape(R // 32, KB, 4, 16, 2, 2)  # nb kb q r j s
    codes = w.permute(0, 4, 3, 1, 2, 5).reshape(R, KB * 8).contiguous().view(torch.uint8)[:M]
    ngq = scales_t.shape[1]
    scales = scales_t.reshape(R // 32, ngq, 16, 2).permute(1, 0, 3, 2).reshape(ngq, R)
    xs = None
    if S_pad:
        W = xs_t.stride(0)
        flat = torch.as_strided(xs_t, (R * W,), (1,))[: R * S_pad]
        t = flat.reshape(R // 32, S_pad // 64, 4, 16, 2, 2, 8)         # nb kd q r j s e
        xs = torch.empty((R, S_pad), dtype=xs_t.dtype, device=xs_t.device)
        v = xs.view(R // 32, 2, 16, S_pad // 64, 8, 8)                 # nb j r kd c e
        for q in range(4):
            for sl in range(2):
                c = 4 * (q & 1) + 2 * sl + (q >> 1)
                v[:, :, :, :, c, :] = t[:, :, q, :, :, sl, :].permute(0, 3, 2, 1, 4)
        xs = xs[:M]
    return codes, scales, xs


CASES = [
    # M, K, N, G, p, dtype, act mode
    (64, 512, 256, 128, 0.10, torch.float16, "per_group"),
    (100, 1096, 520, 64, 0.10, torch.float16, "per_group"),
    (257, 1024, 1000, 128, 0.05, torch.float16, "per_group"),
    (300, 2048, 1536, 256, 0.0, torch.float16, "per_group"),
    (1000, 4096, 640, 128, 0.10, torch.float16, "per_group_mean3std"),
    (2048, 4096, 4096, 64, 0.05, torch.float16, "per_group"),
    (333, 768, 3072, 128, 0.10, torch.bfloat16, "per_group"),
    (513, 2048, 264, 64, 0.05, torch.float16, "per_group_unsorted"),
    (777, 1024, 1032, 128, 0.05, torch.bfloat16, "per_group"),
]


@pytest.mark.parametrize("tiled", [False, True], ids=["rowmajor", "tiled"])
@pytest.mark.parametrize("M,K,N,Gs,p,dt,aq", CASES)
def test_fqt_operands_exact_and_y(M, K, N, Gs, p, dt, aq, tiled):
    dev = _dev()
    from smoothquant import ops
    q, lin, x = _layer(dev, M, K, N, Gs, p, dt, aq=aq)
    pw = q.packed()
    assert ops.fqt_eligible(pw, aq, 4, Gs, M, force=True)
    Kq = (pw.K - pw.S + 63) // 64 * 64
    if tiled and Kq % 128:
        pytest.skip("tile-major operands need Kq % 128 == 0")
    fqt7 = ops.FQT7
    ops.FQT7 = tiled
    try:
        codes, scales, xs, wp = ops.quant_act_c4(x, pw, aq, 4, Gs)
    finally:
        ops.FQT7 = fqt7
    assert (scales.dim() == 3) == tiled
    y = ops.gemm_fqt(codes, scales, xs, wp, pw, lin.bias, Gs)
    if tiled:
        codes, scales, xs = untile_c4(codes, scales, xs, M, Kq, pw.S_pad)
    a = ops.quant_act_fp(x, pw, aq, 4, Gs)
    fq7 = ops.FQ7_AUTO
    ops.FQ7_AUTO = False
    try:
        y_fq = ops.gemm_fq(a, pw, lin.bias)
    finally:
        ops.FQ7_AUTO = fq7
    Kn = pw.K - pw.S
    # activation operand: multisets per row over the non-salient columns, bit-exact
    xa = decode_c4(codes, scales, Kq, Gs, dt)
    assert (xa[:, Kn:] == 0).all()
    nonsal_pos = (pw.amap[: pw.Kp] >= 0).nonzero().flatten()
    want = a[:, nonsal_pos].float().sort(dim=1).values
    got = xa[:, :Kn].float().sort(dim=1).values
    assert torch.equal(got, want)
    if pw.S_pad:
        assert torch.equal(xs[:, : pw.S], a[:, pw.Kp: pw.Kp + pw.S])
    # permuted weight: multisets per row, zeros past Kn, wsal tail
    w_hat = ops.dequant_weight_packed(pw)
    wgot = wp[: pw.N, :Kn].float().sort(dim=1).values
    wwant = w_hat[:, nonsal_pos].float().sort(dim=1).values
    assert torch.equal(wgot, wwant)
    assert (wp[: pw.N, Kn:Kq] == 0).all()
    if pw.S_pad:
        assert torch.equal(wp[: pw.N, Kq:], pw.wsal)
    # y
    ref = xa.float() @ wp[: pw.N, :Kq].float().t() + lin.bias.float()
    if pw.S_pad:
        ref = ref + xs[:, : pw.S_pad].float() @ pw.wsal.float().t()
    tol = 2e-3 if dt == torch.float16 else 1e-2
    assert rel(y, ref) < tol
    assert rel(y, y_fq) < (1e-3 if dt == torch.float16 else 8e-3)


def test_fqt_forward_dispatch_and_full_size_config2():
    """BASELINE config 2 through W4A4Linear.forward (kernel "fqt" via the auto row threshold)
    against the packed-order forward."""
    dev = _dev()
    from smoothquant import ops
    q, lin, x = _layer(dev, 16384, 4096, 4096, 128, 0.10, torch.float16)
    pw = q.packed()
    assert ops.fqt_eligible(pw, "per_group", 4, 128, 16384)
    y_t = q(x)
    q.kernel = "fq"
    y_f = q(x)
    assert rel(y_t, y_f) < 1e-3


def test_standalone_perm_matches_fused():
    """sqmp_perm_weight_c4 (standalone, after the quantizer) == the permutation the fused
    sqmp_quant_act_c4 launch built, bit for bit."""
    dev = _dev()
    import ctypes
    from smoothquant import ops
    from smoothquant._lib import load
    q, lin, x = _layer(dev, 300, 2048, 776, 128, 0.05, torch.float16)
    pw = q.packed()
    codes, scales, xs, wp = ops.quant_act_c4(x, pw, "per_group", 4, 128)
    stream = torch.cuda.current_stream(dev).cuda_stream
    e = ops._act_ws(x.device, stream, pw.K, pw.Kp, ops._ws_bytes(300, pw.K, pw.Kp))
    wp2 = torch.full_like(wp, float("nan"))
    st = load().sqmp_perm_weight_c4(ops._p(e["buf"]), pw.K, pw.Kp, pw.S, pw.S_pad,
                                    ops._p(pw.codes), ops._p(pw.wscale), ops._p(pw.wsal),
                                    ops._dtype_code(pw.dtype), pw.N, pw.Gw, pw.ngw, ops._p(wp2),
                                    ctypes.c_void_p(stream))
    assert st == 0
    assert torch.equal(wp.view(torch.int16), wp2.view(torch.int16))
