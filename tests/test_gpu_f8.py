"""GPU: the block-scaled FP8 path for per_token / per_tensor 4-bit activations.

* operands (SQMP_OUT_F8): the e4m3 act codes decode to integers c with D(c * sa) equal to
  the oracle's q_x BIT-EXACT at every non-salient column, 0 at salient and padding
  positions; the exact salient columns land in xs unchanged.
* y: relative Frobenius error vs the oracle product within the integer-path tolerance of
  test_gpu_parity (TOL_I8: the scales are factored out of the sum)."""
import zlib

import numpy as np
import pytest
import torch

from oracle import fake_quant_oracle as O
from test_gpu_parity import TOL_I8, TORCH_DT, _dev, _rand_inputs, bits_equal, make_layer, rel, to_np, to_t

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
    assert rel(y, want) < TOL_I8[dt], rel(y, want)
