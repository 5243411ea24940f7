"""GPU parity of the activation-order faithful path (SQMP_OUT_C4 quantizer + per-forward
weight permutation, sqmp_gemm_fqt / sqmp_gemm_fqt7) against the ORACLE
(oracle/fake_quant_oracle.py, pinned bit-exact to the reference goldens):

  * the activation operand, COLUMN FOR COLUMN: act-order position j, decoded from the int4
    codes and group scales, is bit-exact the oracle's q_x column nonsal[order[j]] (order =
    the stable sort of the batch's column key, computed independently here); the exact
    salient columns are x[:, S];
  * the permuted weight, the same positions: the oracle's W_hat columns, zeros past K - S,
    then W[:, S] exactly;
  * y: relative Frobenius vs the fp64 product of the oracle's q_x and W_hat 2e-3 (fp16) /
    1e-2 (bf16), and vs the packed-order gemm_fq 1e-3 / 8e-3;
  * the BENCHMARKED kernel at full config-2 size (W4A4Linear.forward on the auto path =
    fqt7): sampled rows of y against the fp64 product of the PyTorch-CPU restatement's q_x
    (oracle/torch_cpu.py, batch-wide sort over all 16384 rows) and W_hat.

Every operand layout: row-major (sqmp_gemm_fqt on fq6's structure) and tile-major with 32-
or 64-row blocks (SQMP_QA_TILED / SQMP_QA_TILED4 + sqmp_gemm_fqt7j with J = 2 / 4, untiled
here before the same checks).
"""
import numpy as np
import pytest
import torch

from oracle import fake_quant_oracle as O

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
    """The tile-major operands (sqmp_pack_fq7 layouts, J = 2 or 4 row tiles per 16 J-row
    block) -> row-major codes [M, Kq/2], scales [ngq, R], xs [M, S_pad]."""
    R = codes_t.shape[0]
    KB = Kq // 64
    J = scales_t.shape[2] // 16
    B = 16 * J
    w = codes_t.contiguous().view(torch.int32).reshape(R // B, KB, 4, 16, J, 2)  # nb kb q r j s
    codes = w.permute(0, 4, 3, 1, 2, 5).reshape(R, KB * 8).contiguous().view(torch.uint8)[:M]
    ngq = scales_t.shape[1]
    scales = scales_t.reshape(R // B, ngq, 16, J).permute(1, 0, 3, 2).reshape(ngq, R)
    xs = None
    if S_pad:
        W = xs_t.stride(0)
        flat = torch.as_strided(xs_t, (R * W,), (1,))[: R * S_pad]
        t = flat.reshape(R // B, S_pad // 64, 4, 16, J, 2, 8)          # nb kd q r j s e
        xs = torch.empty((R, S_pad), dtype=xs_t.dtype, device=xs_t.device)
        v = xs.view(R // B, J, 16, S_pad // 64, 8, 8)                  # nb j r kd c e
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


def act_order_columns(x_np, sal, aq, D):
    """The oracle's activation order: position j of the act-order operand holds original
    column nonsal[order[j]] -- nonsal = the non-salient columns ascending (x[:, mask],
    fake_quant.py:298), order = the stable ascending sort of their batch key (column
    absmax :113; mean3std_key for the config-5 extension; identity when unsorted)."""
    K = x_np.shape[1]
    keep = np.ones(K, bool)
    if sal is not None:
        keep[sal] = False
    nonsal = np.nonzero(keep)[0]
    A = x_np[:, nonsal]
    if aq == "per_group":
        order = O.stable_argsort(D.f32(np.abs(A).max(axis=0)))
    elif aq == "per_group_mean3std":
        order = O.stable_argsort(O.mean3std_key(A, D))
    else:
        order = np.arange(len(nonsal))
    return nonsal[order]


def same_values(a, b):
    """Equal value for value (-0.0 == +0.0: code 0 dequantizes to +0.0, the reference's
    fake quantizer may give -0.0)."""
    a = np.asarray(a, np.float32)
    b = np.asarray(b, np.float32)
    ok = a == b
    if not ok.all():
        idx = np.argwhere(~ok)[:5]
        print(f"{(~ok).sum()} of {ok.size} differ; first {idx.tolist()}: "
              f"{a[tuple(idx.T)]} vs {b[tuple(idx.T)]}")
    return bool(ok.all())


@pytest.mark.parametrize("tiled", [0, 2, 4], ids=["rowmajor", "tiled", "tiled4"])
@pytest.mark.parametrize("M,K,N,Gs,p,dt,aq", CASES)
def test_fqt_operands_exact_and_y(M, K, N, Gs, p, dt, aq, tiled):
    """Column for column against the ORACLE (oracle/fake_quant_oracle.py, pinned to the
    reference goldens): act-order position j of the decoded act operand is the oracle's
    q_x column nonsal[order[j]] and of the permuted weight the oracle's W_hat column, both
    bit-exact; the salient tails are x[:, S] and W[:, S] exactly; y is within the
    accumulation-order tolerance of the fp64 product of the oracle's q_x and W_hat."""
    dev = _dev()
    from smoothquant import ops
    q, lin, x = _layer(dev, M, K, N, Gs, p, dt, aq=aq)
    pw = q.packed()
    assert ops.fqt_eligible(pw, aq, 4, Gs, M, force=True)
    Kq = (pw.K - pw.S + 63) // 64 * 64
    if tiled and Kq % 128:
        pytest.skip("tile-major operands need Kq % 128 == 0 (the dispatcher then takes "
                    "the row-major layout, covered by the rowmajor case)")
    fqt7, fqt7_j = ops.FQT7, ops.FQT7_J
    ops.FQT7, ops.FQT7_J = tiled > 0, max(tiled, 2)
    try:
        codes, scales, xs, wp = ops.quant_act_c4(x, pw, aq, 4, Gs)
    finally:
        ops.FQT7, ops.FQT7_J = fqt7, fqt7_j
    assert (scales.dim() == 3) == (tiled > 0)
    if tiled > 0:
        assert scales.shape[2] == 16 * tiled
    y = ops.gemm_fqt(codes, scales, xs, wp, pw, lin.bias, Gs)
    if tiled > 0:
        codes, scales, xs = untile_c4(codes, scales, xs, M, Kq, pw.S_pad)
    # ---- the oracle's operands (CPU, numpy)
    Dn = {torch.float16: "fp16", torch.bfloat16: "bf16"}[dt]
    D = O.DT(Dn)
    x_np = x.float().cpu().numpy()
    W_np = lin.weight.detach().float().cpu().numpy()
    sal = None if q.salient_indices is None else q.salient_indices.numpy().astype(np.int64)
    wq = "per_group"  # _layer packs the weight per_group (sorted) for every act mode
    w_hat = D.f32(O.w4a4_from_float(W_np, wq, 4, Gs, sal, D))
    qx = D.f32(O.quantize_input(D.rnd(x_np), aq, 4, Gs, sal, D))
    cols = act_order_columns(x_np, sal, aq, D)
    Kn = pw.K - pw.S
    assert len(cols) == Kn
    # act operand, position j <-> original column cols[j]
    xa = decode_c4(codes, scales, Kq, Gs, dt).float().cpu().numpy()
    assert same_values(xa[:, :Kn], qx[:, cols])
    assert (xa[:, Kn:] == 0).all()
    if pw.S:
        assert same_values(xs[:, : pw.S].float().cpu().numpy(), x_np[:, pw.salient.cpu().numpy()])
    # permuted weight, the same positions
    wpn = wp[: pw.N].float().cpu().numpy()
    assert same_values(wpn[:, :Kn], w_hat[:, cols])
    assert (wpn[:, Kn:Kq] == 0).all()
    if pw.S:
        assert same_values(wpn[:, Kq: Kq + pw.S], W_np[:, pw.salient.cpu().numpy()])
    # y against the fp64 product of the oracle's operands
    bias = lin.bias.detach().double()
    ref = torch.from_numpy(qx).to(dev).double() @ torch.from_numpy(w_hat).to(dev).double().t() + bias
    tol = 2e-3 if dt == torch.float16 else 1e-2
    assert rel(y, ref) < tol
    # and against the packed-order GEMM (the same operands in another order)
    a = ops.quant_act_fp(x, pw, aq, 4, Gs)
    fq7 = ops.FQ7_AUTO
    ops.FQ7_AUTO = False
    try:
        y_fq = ops.gemm_fq(a, pw, lin.bias)
    finally:
        ops.FQ7_AUTO = fq7
    assert rel(y, y_fq) < (1e-3 if dt == torch.float16 else 8e-3)


def test_fqt_forward_dispatch_and_full_size_config2():
    """BASELINE config 2 (M=16384, K=N=4096, G=128, 10 % salient) through
    W4A4Linear.forward on the auto path -- the kernel bench.py times (fqt7 on tile-major
    operands) -- against the oracle directly: sampled rows of y vs the fp64 product of the
    PyTorch-CPU restatement's q_x (oracle/torch_cpu.py: the batch-wide column sort over all
    16384 rows, fp16 rounding points of fake_quant.py:104-154) and its W_hat
    (:156-207 + :347-365), tolerance 2e-3; and vs the packed-order forward 1e-3."""
    dev = _dev()
    from oracle import torch_cpu as T
    from smoothquant import ops
    q, lin, x = _layer(dev, 16384, 4096, 4096, 128, 0.10, torch.float16)
    pw = q.packed()
    assert ops.fqt_eligible(pw, "per_group", 4, 128, 16384)
    seen = []
    real = ops.gemm_fqt

    def spy(codes, scales, *a, **k):
        seen.append(scales.dim())
        return real(codes, scales, *a, **k)

    ops.gemm_fqt = spy
    try:
        y_t = q(x)
    finally:
        ops.gemm_fqt = real
    assert seen == [3], "the auto path must run the tile-major fqt7 GEMM"
    # the oracle on CPU: q_x over the whole batch, W_hat
    xc = x.cpu()
    sal = q.salient_indices.cpu()
    keep = torch.ones(4096, dtype=torch.bool)
    keep[sal] = False
    qx = xc.clone()
    qx[:, keep] = T.act_quant(xc[:, keep], "per_group", 4, 128)
    w_hat = T.quantize_weight(lin.weight.detach().cpu(), "per_group", 4, 128, sal)
    assert torch.equal(q.weight.cpu(), w_hat)
    rows = torch.arange(0, 16384, 61)
    ref = qx[rows].double() @ w_hat.double().t() + lin.bias.detach().cpu().double()
    assert rel(y_t[rows.to(dev)].cpu(), ref) < 2e-3
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

