"""Pin the CPU oracle against fixtures produced by the reference itself (CPU, no GPU).

Every quantizer primitive and every W4A4Linear golden must match BIT-EXACTLY for the
dequantized tensors (W_hat, q_x).  The layer output y comes from the reference's CPU
F.linear (MKL/oneDNN accumulation order); the oracle accumulates in fp64 and rounds
once, so y is compared with an accumulation-order tolerance stated below.
"""
import numpy as np
import pytest

from oracle import fake_quant_oracle as O
from golden_io import Golden

G = Golden()
PRIMS = G.meta["prims"]
LAYERS = G.meta["layers"]


def _bits(a, dt):
    a = np.asarray(a)
    if dt == "fp16":
        return a.astype(np.float16).view(np.uint16)
    return a.astype(np.float32).view(np.uint32)


@pytest.mark.parametrize("m", PRIMS, ids=[p["name"] for p in PRIMS])
def test_primitive_bit_exact(m):
    dt = O.DT(m["dtype"])
    x = G.arr(m["key"] + "_in", m["dtype"])
    want = G.arr(m["key"] + "_out", m["dtype"])
    fn = getattr(O, m["fn"])
    kw = {}
    if m["group_size"] is not None:
        kw["group_size"] = m["group_size"]
    got = fn(x.copy(), m["n_bits"], dt, **kw)
    got = np.asarray(got).reshape(want.shape)
    assert np.array_equal(_bits(got, m["dtype"]), _bits(want, m["dtype"])), m["name"]


@pytest.mark.parametrize("m", LAYERS, ids=[l["key"] for l in LAYERS])
def test_layer_weight_and_input_bit_exact(m):
    dtn = m["dtype"]
    dt = O.DT(dtn)
    W = G.arr(m["key"] + "_W", dtn)
    x = G.arr(m["key"] + "_x", dtn)
    sal = G.z[m["key"] + "_sal"]
    sal = sal if m["has_salient"] else None
    imp = G.z[m["key"] + "_imp"]
    # salient selection restated (fake_quant.py:265-270)
    want_sal = O.select_salient(imp, m["salient_prop"])
    if sal is None:
        assert want_sal is None
    else:
        assert np.array_equal(want_sal, sal)
    w_hat = O.w4a4_from_float(W, m["weight_quant"], m["n_bits"], m["group_size"], sal, dt)
    assert np.array_equal(_bits(w_hat, dtn), _bits(G.arr(m["key"] + "_What", dtn), dtn))
    K = m["K"]
    qx = O.quantize_input(x.reshape(-1, K), m["act_quant"], m["n_bits"], m["group_size"],
                          sal, dt)
    assert np.array_equal(_bits(qx, dtn), _bits(G.arr(m["key"] + "_qx", dtn), dtn))


# accumulation-order tolerance for y vs the reference's CPU F.linear (relative Frobenius)
Y_TOL = {"fp32": 1e-6, "fp16": 2e-3, "bf16": 1e-2}


@pytest.mark.parametrize("m", LAYERS, ids=[l["key"] for l in LAYERS])
def test_layer_forward_close(m):
    dtn = m["dtype"]
    dt = O.DT(dtn)
    key = m["key"]
    W = G.arr(key + "_W", dtn)
    x = G.arr(key + "_x", dtn)
    b = G.arr(key + "_b", dtn) if m["bias"] else None
    sal = G.z[key + "_sal"] if m["has_salient"] else None
    w_hat = O.w4a4_from_float(W, m["weight_quant"], m["n_bits"], m["group_size"], sal, dt)
    y = O.w4a4_forward(x, w_hat, b, m["act_quant"], m["n_bits"], m["group_size"], sal,
                       m["quantize_output"], dt)
    want = G.arr(key + "_y", dtn).astype(np.float64)
    got = np.asarray(y, dtype=np.float64)
    assert got.shape == want.shape
    rel = np.linalg.norm(got - want) / np.linalg.norm(want)
    if m["quantize_output"]:
        # output quantization re-derives scales from the GEMM output, so fp32 ulps of
        # the accumulation move every scale by an ulp (values then differ ~1e-7); a
        # flipped rounding would show up as a ~1/7 relative jump in one element.
        assert rel < Y_TOL[dtn] * 10 + 1e-6, rel
    else:
        assert rel < Y_TOL[dtn], rel


def test_error_conventions():
    dt = O.DT("fp32")
    with pytest.raises(ValueError):
        O.act_quant_fn("per_row", 4, 128, dt)
    with pytest.raises(ValueError):
        O.weight_quant_fn("per_row", 4, 128, dt)
    with pytest.raises(ValueError):
        O.w4a4_forward(np.zeros((1, 2, 3, 4), np.float32), np.zeros((4, 4), np.float32),
                       None, "per_token", 4, 128, None, False, dt)
