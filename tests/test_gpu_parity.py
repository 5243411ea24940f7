"""GPU parity of the HIP path against the reference goldens and the CPU oracle.

Tolerances (stated once, used everywhere):
  * W_hat (the `weight` buffer) and the dequantized activations q_x: BIT-EXACT.
  * y: relative Frobenius error vs the oracle's fp64-accumulated product, which differs
    from any fp32-accumulating GEMM only by accumulation order:
        fp32 1e-5, fp16 2e-3, bf16 1e-2            (faithful "fq" kernel)
    The "f8" kernel (e4m3 codes) factors the scales out of the sum, so each product
    differs by the D rounding of x_hat and W_hat (<= 2^-11 rel for fp16, 2^-8 for bf16):
        fp16 3e-3, bf16 2e-2.
"""
import zlib

import numpy as np
import pytest
import torch

from oracle import fake_quant_oracle as O
from golden_io import Golden

pytestmark = pytest.mark.gpu

TORCH_DT = {"fp32": torch.float32, "fp16": torch.float16, "bf16": torch.bfloat16}
TOL_FQ = {"fp32": 1e-5, "fp16": 2e-3, "bf16": 1e-2}
TOL_F8 = {"fp16": 3e-3, "bf16": 2e-2}

G = Golden()


def _dev():
    if not torch.cuda.is_available():
        pytest.skip("no ROCm device")
    return torch.device("cuda")


def to_t(a, dt, dev):
    return torch.from_numpy(np.ascontiguousarray(np.asarray(a, dtype=np.float32))).to(dev, TORCH_DT[dt])


def to_np(t):
    return t.detach().float().cpu().numpy()


def bits_equal(a, b):
    """Exact equality of every value.  The only representational difference allowed is the
    sign of zero: the reference's fake quantizer yields -0.0 where a negative input rounds
    to code 0 (fake_quant.py:193), an integer code 0 dequantizes to +0.0; -0.0 == +0.0 in
    every later operation."""
    a = np.asarray(a, np.float32)
    b = np.asarray(b, np.float32)
    if a.shape != b.shape:
        print("shape mismatch", a.shape, b.shape)
        return False
    ok = (a == b) | (np.isnan(a) & np.isnan(b))
    if not ok.all():
        idx = np.argwhere(~ok)
        print(f"{(~ok).sum()} of {ok.size} values differ; first {idx[:5].tolist()}: "
              f"got {a[tuple(idx[:5].T)]} want {b[tuple(idx[:5].T)]}")
    return bool(ok.all())


def rel(a, b):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    return np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-30)


def make_layer(W, b, dt, dev, **kw):
    from smoothquant.fake_quant import W4A4Linear
    K = W.shape[1]
    N = W.shape[0]
    lin = torch.nn.Linear(K, N, bias=b is not None)
    lin = lin.to(dev, TORCH_DT[dt])
    with torch.no_grad():
        lin.weight.copy_(to_t(W, dt, dev))
        if b is not None:
            lin.bias.copy_(to_t(b, dt, dev))
    return W4A4Linear.from_float(lin, **kw)


def a_operand_to_original(q, a, K):
    """Map the packed A operand [M, Kp+S_pad] back to original column order."""
    pw = q.packed()
    amap = pw.amap.cpu().numpy()
    a_np = to_np(a)
    out = np.zeros((a_np.shape[0], K), np.float32)
    valid = amap >= 0
    out[:, amap[valid]] = a_np[:, :pw.Kp][:, valid]
    if pw.S:
        sal = pw.salient.cpu().numpy()
        out[:, sal] = a_np[:, pw.Kp:pw.Kp + pw.S]
    return out


# ------------------------------------------------------------------ reference goldens
LAYERS = G.meta["layers"]


@pytest.mark.parametrize("m", LAYERS, ids=[l["key"] for l in LAYERS])
def test_golden_layer(m):
    dev = _dev()
    from smoothquant import ops
    dt, key = m["dtype"], m["key"]
    W = G.arr(key + "_W", dt)
    x = G.arr(key + "_x", dt)
    b = G.arr(key + "_b", dt) if m["bias"] else None
    imp = torch.from_numpy(G.z[key + "_imp"])
    q = make_layer(W, b, dt, dev, weight_quant=m["weight_quant"], act_quant=m["act_quant"],
                   quantize_output=m["quantize_output"], importance=imp,
                   salient_prop=m["salient_prop"], quant_bits=m["n_bits"],
                   group_size=m["group_size"])
    if m["has_salient"]:
        assert np.array_equal(q.salient_indices.numpy(), G.z[key + "_sal"])
    else:
        assert q.salient_indices is None
    # W_hat bit-exact (fake_quant.py:324-371)
    assert bits_equal(to_np(q.weight), G.arr(key + "_What", dt))
    K = m["K"]
    xt = to_t(x, dt, dev)
    # q_x bit-exact (fake_quant.py:291-304) through the packed A operand
    a = ops.quant_act_fp(xt.reshape(-1, K).contiguous(), q.packed(), m["act_quant"],
                         m["n_bits"], m["group_size"])
    assert bits_equal(a_operand_to_original(q, a, K), G.arr(key + "_qx", dt))
    # forward
    kernels = ["fq"]
    if ops.f8_eligible(q.packed(), m["act_quant"], m["n_bits"]):
        kernels.append("f8")
    want = G.arr(key + "_y", dt)
    for kern in kernels:
        q.kernel = kern
        y = q(xt.clone())
        assert tuple(y.shape) == tuple(want.shape)
        tol = TOL_FQ[dt] if kern == "fq" else TOL_F8[dt]
        if m["quantize_output"]:
            tol = tol * 10 + 1e-6
        assert rel(to_np(y), want) < tol, (kern, rel(to_np(y), want))


# ------------------------------------------------------------------ oracle, random sizes
CASES = [
    # dtype, wq, aq, p, bits, G, M, K, N, bias
    ("fp16", "per_group", "per_group", 0.10, 4, 128, 300, 1024, 384, True),
    ("fp16", "per_group", "per_token", 0.10, 4, 128, 257, 1024, 520, True),
    ("fp16", "per_group", "per_tensor", 0.05, 4, 64, 129, 512, 256, False),
    ("fp16", "per_channel", "per_token", 0.0, 4, 128, 64, 768, 3072, True),
    ("fp16", "per_group", "per_group", 0.05, 4, 64, 200, 1100, 300, True),
    ("fp16", "per_group", "per_group", 0.10, 4, 4, 64, 256, 128, True),       # G=4 dense fallback
    ("fp16", "per_group", "per_group", 0.0, 4, 1024, 64, 2200, 128, True),    # padded last group
    ("fp16", "per_group", "per_group", 0.10, 8, 128, 100, 512, 256, True),    # 8-bit
    ("bf16", "per_group", "per_group", 0.10, 4, 128, 300, 1024, 384, True),
    ("bf16", "per_group", "per_token", 0.10, 4, 64, 96, 512, 256, True),
    ("fp32", "per_group", "per_group", 0.10, 4, 128, 130, 512, 200, True),
    ("fp32", "per_tensor", "per_token", 0.0, 4, 128, 33, 256, 64, False),
]


def _rand_inputs(seed, M, K, N, bias):
    g = np.random.default_rng(seed)
    W = (g.standard_normal((N, K)) * 0.02).astype(np.float32)
    x = g.standard_normal((M, K)).astype(np.float32)
    out = g.permutation(K)[: max(1, K // 100)]
    x[:, out] *= 30.0
    cal = np.abs(g.standard_normal((256, K)).astype(np.float32))
    cal[:, out] *= 30.0
    imp = cal.mean(0)
    b = (g.standard_normal(N) * 0.01).astype(np.float32) if bias else None
    return W, x, imp, b


@pytest.mark.parametrize("case", CASES, ids=[f"{c[0]}-{c[1]}-{c[2]}-p{c[3]}-b{c[4]}-G{c[5]}-{c[6]}x{c[7]}x{c[8]}" for c in CASES])
def test_oracle_parity(case):
    dev = _dev()
    from smoothquant import ops
    dt, wq, aq, p, bits, Gs, M, K, N, bias = case
    D = O.DT(dt)
    W, x, imp, b = _rand_inputs(zlib.crc32(repr(case).encode()), M, K, N, bias)
    W, x = D.rnd(W), D.rnd(x)
    b = D.rnd(b) if b is not None else None
    q = make_layer(W, b, dt, dev, weight_quant=wq, act_quant=aq, importance=torch.from_numpy(imp),
                   salient_prop=p, quant_bits=bits, group_size=Gs)
    sal = O.select_salient(imp, p)
    if sal is None:
        assert q.salient_indices is None
    else:
        assert np.array_equal(q.salient_indices.numpy(), sal)
    w_hat = O.w4a4_from_float(W, wq, bits, Gs, sal, D)
    assert bits_equal(to_np(q.weight), D.f32(w_hat))
    xt = to_t(x, dt, dev)
    qx = O.quantize_input(x, aq, bits, Gs, sal, D)
    a = ops.quant_act_fp(xt, q.packed(), aq, bits, Gs)
    assert bits_equal(a_operand_to_original(q, a, K), D.f32(qx))
    want = O.linear(qx, w_hat, b, D)
    kernels = ["fq"] + (["f8"] if ops.f8_eligible(q.packed(), aq, bits) else [])
    for kern in kernels:
        q.kernel = kern
        y = q(xt.clone())
        tol = TOL_FQ[dt] if kern == "fq" else TOL_F8[dt]
        assert rel(to_np(y), D.f32(want)) < tol, (kern, rel(to_np(y), D.f32(want)))


# ------------------------------------------------------------------ edge cases
def test_edge_shapes_and_errors():
    dev = _dev()
    from smoothquant.fake_quant import W4A4Linear
    D = O.DT("fp16")
    g = np.random.default_rng(7)
    # K not a multiple of 8 (unvectorised row path), 3-D input, no bias, M=1
    K, N = 100, 72
    W = D.rnd(g.standard_normal((N, K)) * 0.02)
    imp = np.abs(g.standard_normal(K)).astype(np.float32)
    q = make_layer(W, None, "fp16", dev, weight_quant="per_group", act_quant="per_group",
                   importance=torch.from_numpy(imp), salient_prop=0.1, group_size=16)
    for shape in [(1, K), (2, 3, K), (5, K)]:
        x = D.rnd(g.standard_normal(shape))
        y = q(to_t(x, "fp16", dev))
        sal = O.select_salient(imp, 0.1)
        w_hat = O.w4a4_from_float(W, "per_group", 4, 16, sal, D)
        want = O.w4a4_forward(x, w_hat, None, "per_group", 4, 16, sal, False, D)
        assert tuple(y.shape) == tuple(want.shape)
        assert rel(to_np(y), D.f32(want)) < TOL_FQ["fp16"]
    # all-zero input: scales clamp at 1e-5 (fake_quant.py:139), output = bias
    b = D.rnd(g.standard_normal(N) * 0.01)
    q2 = make_layer(W, b, "fp16", dev, weight_quant="per_group", act_quant="per_group",
                    importance=torch.from_numpy(imp), salient_prop=0.1, group_size=16)
    y0 = q2(torch.zeros(4, K, dtype=torch.float16, device=dev))
    assert np.allclose(to_np(y0), np.broadcast_to(D.f32(b), (4, N)))
    # every channel salient: activations pass through exactly
    q3 = make_layer(W, b, "fp16", dev, weight_quant="per_group", act_quant="per_group",
                    importance=torch.from_numpy(imp), salient_prop=1.0, group_size=16)
    x = D.rnd(g.standard_normal((8, K)))
    want = O.linear(x, W, b, D)
    assert rel(to_np(q3(to_t(x, "fp16", dev))), D.f32(want)) < TOL_FQ["fp16"]
    # output quantization with salient channels needs N == K (IndexError, like the reference)
    q4 = make_layer(W, b, "fp16", dev, weight_quant="per_group", act_quant="per_group",
                    quantize_output=True, importance=torch.from_numpy(imp), salient_prop=0.1,
                    group_size=16)
    with pytest.raises(IndexError):
        q4(to_t(x, "fp16", dev))
    with pytest.raises(ValueError):
        make_layer(W, b, "fp16", dev, weight_quant="per_row")


def test_per_token_mutates_input_like_reference():
    """fake_quant.py:304 + :56-64: without salient channels the per_token quantizer runs in
    place on the caller's activation."""
    dev = _dev()
    D = O.DT("fp16")
    g = np.random.default_rng(11)
    W = D.rnd(g.standard_normal((64, 256)) * 0.02)
    q = make_layer(W, None, "fp16", dev, weight_quant="per_channel", act_quant="per_token")
    x = D.rnd(g.standard_normal((16, 256)))
    xt = to_t(x, "fp16", dev)
    q(xt)
    assert bits_equal(to_np(xt), D.f32(O.quantize_activation_per_token_absmax(x, 4, D)))


def test_primitives_match_oracle():
    dev = _dev()
    from smoothquant import fake_quant as F
    D = O.DT("fp16")
    g = np.random.default_rng(3)
    t = D.rnd(g.standard_normal((2, 50, 192)))
    for name, fn in [("quantize_activation_per_group_absmax_sort", lambda a: F.quantize_activation_per_group_absmax_sort(a, 4, 32)),
                     ("quantize_activation_per_group_absmax", lambda a: F.quantize_activation_per_group_absmax(a, 4, 32))]:
        got = fn(to_t(t, "fp16", dev))
        want = getattr(O, name)(t, 4, D, group_size=32)
        assert bits_equal(to_np(got), D.f32(want)), name
    w = D.rnd(g.standard_normal((40, 136)) * 0.02)
    got = F.quantize_weight_per_group_absmax_sort(to_t(w, "fp16", dev), 4, 64)
    assert bits_equal(to_np(got), D.f32(O.quantize_weight_per_group_absmax_sort(w, 4, D, 64)))
    wt = to_t(w, "fp16", dev)
    F.quantize_weight_per_channel_absmax(wt, 4)
    assert bits_equal(to_np(wt), D.f32(O.quantize_weight_per_channel_absmax(w, 4, D)))


# ------------------------------------------------------------------ full-size properties
def test_full_size_config2_properties():
    """BASELINE config 2 (M=16384, K=N=4096, G=128, 10% salient): the GEMM output equals
    an independent fp32 product of the kernel's own operands (checks the GEMM at full
    size), the per_group activation operand matches the oracle on sampled rows (checks
    the batch-wide sort), and W_hat matches the oracle on sampled rows."""
    dev = _dev()
    from smoothquant import ops
    D = O.DT("fp16")
    M, K, N, Gs, p = 16384, 4096, 4096, 128, 0.10
    gen = torch.Generator(device=dev).manual_seed(0)
    W = (torch.randn(N, K, generator=gen, device=dev) * 0.02).half()
    x = torch.randn(M, K, generator=gen, device=dev)
    out = torch.randperm(K, generator=gen, device=dev)[:41]
    x[:, out] *= 30
    x = x.half()
    imp = x[:2048].float().abs().mean(0).cpu()
    lin = torch.nn.Linear(K, N, bias=True).to(dev, torch.float16)
    with torch.no_grad():
        lin.weight.copy_(W)
        lin.bias.copy_(torch.randn(N, generator=gen, device=dev).half() * 0.01)
    from smoothquant.fake_quant import W4A4Linear
    q = W4A4Linear.from_float(lin, weight_quant="per_group", act_quant="per_group",
                              importance=imp, salient_prop=p, group_size=Gs)
    pw = q.packed()
    a = ops.quant_act_fp(x, pw, "per_group", 4, Gs)
    y = ops.gemm_fq(a, pw, lin.bias)
    b_full = torch.cat([ops.dequant_weight_packed(pw) if pw.dense is None else pw.dense,
                        pw.wsal], dim=1) if pw.S_pad else ops.dequant_weight_packed(pw)
    ref = (a.float() @ b_full.float().t() + lin.bias.float()).half()
    assert rel(to_np(y), to_np(ref)) < 2e-3
    # sampled rows of q_x against the oracle (the sort is batch-wide: oracle on all rows)
    x_np = to_np(x).astype(np.float16)
    sal = q.salient_indices.numpy()
    mask = np.ones(K, bool)
    mask[sal] = False
    A = x_np[:, mask]
    col_max = np.abs(A).max(axis=0)
    perm = O.stable_argsort(D.f32(col_max))
    rows = np.arange(0, M, 997)
    deq, _, _ = O._group_quant_rows(A[rows][:, perm], 4, Gs, D)
    inv = np.argsort(perm, kind="stable")
    want_rows = x_np[rows].astype(np.float32)
    want_rows[:, mask] = deq[:, inv].astype(np.float32)
    got_rows = a_operand_to_original(q, a[torch.from_numpy(rows).to(dev)], K)
    assert bits_equal(got_rows, want_rows)
    # W_hat rows
    w_rows = np.arange(0, N, 511)
    W_np = to_np(W).astype(np.float16)
    w_hat = O.w4a4_from_float(W_np, "per_group", 4, Gs, sal, D)
    assert bits_equal(to_np(q.weight)[w_rows], D.f32(w_hat)[w_rows])


# ------------------------------------------------------------------ rounding stress
@pytest.mark.parametrize("dt", ["fp16", "bf16"])
@pytest.mark.parametrize("act", ["per_token", "per_tensor", "per_group"])
def test_act_quant_rounding_stress(dt, act):
    """The activation operand x_hat = D(rne(D(x / s)) * s) is bit-exact on ~1M elements.
    The kernel divides by multiplying with RN(1/s) and falls back to the exact division
    only within a few fp32 ulps of a D rounding midpoint (sqmp_actquant.hip fast_code);
    random data hits that window ~1e-3 of the time, and rows whose scale is a power of two
    put quotients exactly on half-integers (round-half-even of the code)."""
    dev = _dev()
    from smoothquant import ops
    D = O.DT(dt)
    M, K, N, Gs = 512, 2048, 256, 128
    g = np.random.default_rng(zlib.crc32(f"stress-{dt}-{act}".encode()))
    x = g.standard_normal((M, K)).astype(np.float32)
    x[:, g.permutation(K)[:20]] *= 25.0
    # rows 0..63: absmax 7 * 2^e -> s = 2^e exactly, the rest multiples of s/2 (ties)
    for r in range(64):
        e = int(g.integers(-6, 3))
        x[r] = np.round(x[r] * 2.0) / 2.0 * 2.0 ** e
        x[r] = np.clip(x[r], -7 * 2.0 ** e, 7 * 2.0 ** e)
        x[r, 0] = 7 * 2.0 ** e
    x = D.rnd(x)
    W = D.rnd(g.standard_normal((N, K)).astype(np.float32) * 0.02)
    imp = torch.from_numpy(np.abs(g.standard_normal(K)).astype(np.float32))
    q = make_layer(W, None, dt, dev, weight_quant="per_channel", act_quant=act,
                   importance=imp, salient_prop=0.05, quant_bits=4, group_size=Gs)
    pw = q.packed()
    xt = to_t(x, dt, dev)
    a = ops.quant_act_fp(xt, pw, act, 4, Gs)
    got = a_operand_to_original(q, a, K)
    sal = q.salient_indices.cpu().numpy()
    want = O.quantize_input(x, act, 4, Gs, sal, D)
    assert bits_equal(got, D.f32(want))


# ------------------------------------------------------------------ packed checkpoints
def test_packed_checkpoint_roundtrip(tmp_path):
    """A quantized layer saved with its packed state reloads into a fresh module (safe
    loader) and computes the identical output, with no re-quantization."""
    dev = _dev()
    import os
    from smoothquant.checkpoint import load_quantized, save_quantized
    from smoothquant.fake_quant import W4A4Linear
    g = np.random.default_rng(11)
    K, N = 512, 512
    W = g.standard_normal((N, K)).astype(np.float32) * 0.02
    b = g.standard_normal(N).astype(np.float32) * 0.01
    imp = torch.from_numpy(np.abs(g.standard_normal(K)).astype(np.float32))
    model = torch.nn.Sequential(torch.nn.Linear(K, N), torch.nn.Linear(N, N)).to(dev).half()
    model[0] = make_layer(W, b, "fp16", dev, weight_quant="per_group", act_quant="per_group",
                          importance=imp, salient_prop=0.05, quant_bits=4, group_size=64)
    model[1] = make_layer(W, b, "fp16", dev, weight_quant="per_channel", act_quant="per_token",
                          quantize_output=True, importance=imp, salient_prop=0.05)
    x = to_t(g.standard_normal((64, K)), "fp16", dev)
    y0 = model(x.clone())
    p = os.path.join(tmp_path, "q.pt")
    save_quantized(model, p)
    fresh = torch.nn.Sequential(torch.nn.Linear(K, N), torch.nn.Linear(N, N)).to(dev).half()
    load_quantized(fresh, p)
    assert all(isinstance(m, W4A4Linear) for m in fresh)
    y1 = fresh(x.clone())
    assert bits_equal(to_np(y1), to_np(y0))
    assert bits_equal(to_np(fresh[0].weight), to_np(model[0].weight))


# ------------------------------------------------------------------ casts (.to / _apply)
def test_dtype_cast_keeps_packing_when_exact():
    """model.float() on an fp16 W4A4Linear turns the reference's W_hat buffer into
    cast(W_hat) = fp32(fp16(code * s)).  When that equals code * fp32(s) for every weight
    (here: power-of-two group scales) the layer stays int4-packed with fp32 scales; when it
    does not (random weights: fp16 rounded the products) it keeps the reference's values as
    a dense operand and warns.  Either way the values are the reference's."""
    dev = _dev()
    import warnings
    D16, D32 = O.DT("fp16"), O.DT("fp32")
    g = np.random.default_rng(17)
    K, N, M = 512, 256, 64
    imp = np.abs(g.standard_normal(K)).astype(np.float32)
    sal = O.select_salient(imp, 0.05)
    x = D32.rnd(g.standard_normal((M, K)))
    codes = g.integers(-7, 8, (N, K)).astype(np.float32)
    codes[g.integers(0, N, K), np.arange(K)] = 7  # every column absmax 7 -> s = 2^-6
    cases = [(codes * 2.0 ** -6, False), (D16.rnd(g.standard_normal((N, K)) * 0.02), True)]
    for W, expect_warn in cases:
        b = D16.rnd(g.standard_normal(N) * 0.01)
        q = make_layer(W, b, "fp16", dev, weight_quant="per_group", act_quant="per_group",
                       importance=torch.from_numpy(imp), salient_prop=0.05, group_size=64)
        w_cast = to_np(q.weight.float())
        with warnings.catch_warnings(record=True) as rec:
            warnings.simplefilter("always")
            q.float()
        warned = any(issubclass(w.category, RuntimeWarning) for w in rec)
        assert warned == expect_warn
        pw = q.packed()
        assert pw.dtype == torch.float32 and pw.n_bits == (0 if expect_warn else 4)
        assert bits_equal(to_np(q.weight), w_cast)
        want = D32.f32(O.w4a4_forward(x, w_cast, D32.rnd(b), "per_group", 4, 64, sal, False, D32))
        assert rel(to_np(q(to_t(x, "fp32", dev))), want) < TOL_FQ["fp32"]


def test_packed_checkpoint_loads_into_from_float_module(tmp_path):
    """A checkpoint loads into a model whose layers are already W4A4Linear.from_float
    modules (their bias is the aliased nn.Parameter of the source Linear,
    fake_quant.py:369-370) and reproduces the saved model's output exactly."""
    dev = _dev()
    import os
    from smoothquant.checkpoint import load_quantized, save_quantized
    g = np.random.default_rng(23)
    K, N = 256, 256
    imp = torch.from_numpy(np.abs(g.standard_normal(K)).astype(np.float32))

    def model_from(seed):
        gg = np.random.default_rng(seed)
        W = gg.standard_normal((N, K)).astype(np.float32) * 0.02
        b = gg.standard_normal(N).astype(np.float32) * 0.01
        return torch.nn.Sequential(
            make_layer(W, b, "fp16", dev, weight_quant="per_group", act_quant="per_group",
                       importance=imp, salient_prop=0.05, group_size=64))

    src, dst = model_from(1), model_from(2)
    assert isinstance(dst[0].bias, torch.nn.Parameter)
    x = to_t(g.standard_normal((32, K)), "fp16", dev)
    y0 = src(x.clone())
    p = os.path.join(tmp_path, "q.pt")
    save_quantized(src, p)
    load_quantized(dst, p)
    assert bits_equal(to_np(dst(x.clone())), to_np(y0))


def test_device_round_trip_keeps_packing_and_output():
    """model.to("cpu") then .to("cuda") (nn.Module device moves, fake_quant.py:272-277 keeps
    W_hat as a buffer): the packed buffers travel with the module, stay int4-packed, the
    forward on the GPU afterwards is bit-identical, and a forward on the CPU raises (the
    operator has no CPU path) instead of silently falling back."""
    dev = _dev()
    g = np.random.default_rng(29)
    K, N, M = 512, 384, 48
    W = g.standard_normal((N, K)).astype(np.float32) * 0.02
    b = g.standard_normal(N).astype(np.float32) * 0.01
    imp = torch.from_numpy(np.abs(g.standard_normal(K)).astype(np.float32))
    for dtn in ("fp16", "fp32"):
        q = make_layer(W, b, dtn, dev, weight_quant="per_group", act_quant="per_group",
                       importance=imp, salient_prop=0.05, group_size=64)
        x = to_t(g.standard_normal((M, K)), dtn, dev)
        y0 = q(x.clone())
        q.to("cpu")
        assert q.w_codes.device.type == "cpu" and q.packed().n_bits == 4
        with pytest.raises(RuntimeError):
            q(x.cpu())
        q.to(dev)
        assert q.w_codes.device == x.device and q.packed().n_bits == 4
        assert bits_equal(to_np(q(x.clone())), to_np(y0))
