"""Config 5 (W4A8 + sort sweep): pin the oracle against reference-generated fixtures.

tests/golden/sweep_golden.npz holds the reference's own outputs for the compositions a
user of the reference writes for W4A8 (act_quant rebound to n_bits=8) and sort=none
(the unwired unsorted quantizers, fake_quant.py:29-53 / :77-101).  W_hat and q_x must
match bit-exactly; y within the CPU accumulation-order tolerance of test_oracle_golden.
The mean+3sigma key has no reference implementation (README.md:36 only): its tests
check the oracle's own definition (parity unpinned).
"""
import json
import os

import numpy as np
import pytest

import sweep_inputs as SI
from oracle import fake_quant_oracle as O

PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "sweep_golden.npz")
Z = np.load(PATH, allow_pickle=False)
META = json.loads(bytes(Z["meta_json"]).decode())
CASES = META["cases"]
Y_TOL = {"fp32": 1e-6, "fp16": 2e-3, "bf16": 1e-2}


def arr(key, dt):
    a = Z[key]
    return (a.astype(np.uint32) << 16).view(np.float32) if dt == "bf16" else a


def bits(a, dt):
    a = np.asarray(a)
    return a.astype(np.float16).view(np.uint16) if dt == "fp16" else a.astype(np.float32).view(np.uint32)


def modes(m):
    return ("per_group", "per_group") if m["sort"] == "max" else ("per_group_unsorted",) * 2


def case_arrays(m):
    """(W, x, b, importance) of a sweep case as float32 numpy: stored arrays, or for the
    digest cases re-drawn from the generator's seed (tests/sweep_inputs.py)."""
    key, dtn = m["key"], m["dtype"]
    if "index" in m:
        w, b, x, imp = SI.case_inputs(m["index"], m["case"])
        f = lambda t: None if t is None else t.float().numpy()  # noqa: E731
        return f(w), f(x), f(b), imp.numpy().astype(np.float32)
    W, x = arr(key + "_W", dtn), arr(key + "_x", dtn)
    b = arr(key + "_b", dtn) if m["bias"] else None
    return W, x, b, Z[key + "_imp"]


@pytest.mark.parametrize("m", CASES, ids=[f"{c['key']}-{c['dtype']}-{c['sort']}-a{c['act_bits']}-G{c['group_size']}-K{c['K']}" for c in CASES])
def test_sweep_case(m):
    dtn, key = m["dtype"], m["key"]
    dt = O.DT(dtn)
    wq, aq = modes(m)
    W, x, b, imp = case_arrays(m)
    sal = Z[key + "_sal"] if m["has_salient"] else None
    assert (O.select_salient(imp, m["salient_prop"]) is None) == (sal is None)
    if sal is not None:
        assert np.array_equal(O.select_salient(imp, m["salient_prop"]), sal)
    w_hat = O.w4a4_from_float(W, wq, m["w_bits"], m["group_size"], sal, dt)
    K = m["K"]
    qx = O.quantize_input(x.reshape(-1, K), aq, m["act_bits"], m["group_size"], sal, dt)
    if "index" in m:
        assert SI.digest(dt.f32(w_hat)) == m["what_sha256"]
        assert SI.digest(dt.f32(qx)) == m["qx_sha256"]
    else:
        assert np.array_equal(bits(w_hat, dtn), bits(arr(key + "_What", dtn), dtn))
        assert np.array_equal(bits(qx, dtn), bits(arr(key + "_qx", dtn), dtn))
    y = O.w4a4_forward(x, w_hat, b, aq, m["w_bits"], m["group_size"], sal, False, dt,
                       act_bits=m["act_bits"])
    want = arr(key + "_y", dtn).astype(np.float64)
    rel = np.linalg.norm(np.asarray(y, np.float64) - want) / np.linalg.norm(want)
    assert rel < Y_TOL[dtn], rel


def test_mean3std_key_definition():
    g = np.random.default_rng(0)
    dt = O.DT("fp16")
    t = dt.rnd(g.standard_normal((300, 40)) * np.linspace(0.1, 3, 40))
    k = O.mean3std_key(t, dt)
    a = np.abs(t.astype(np.float64))
    want = (a.mean(0) + 3 * a.std(0)).astype(np.float32)
    np.testing.assert_allclose(k, want, rtol=1e-6)
    # a column with a lower max but a heavier bulk sorts after one with a single spike
    t2 = np.zeros((100, 2), np.float32)
    t2[:, 0] = 1.0
    t2[0, 1] = 5.0
    k2 = O.mean3std_key(t2, O.DT("fp32"))
    assert np.abs(t2).max(0)[1] > np.abs(t2).max(0)[0] and k2[1] > k2[0]
    # ties (identical columns) keep the stable order
    t3 = np.repeat(t[:, :1], 3, axis=1)
    assert list(O.stable_argsort(O.mean3std_key(t3, dt))) == [0, 1, 2]


def test_mean3std_sorted_groups_partition():
    """Every group of the mean3std quantizer is G consecutive columns of the key order."""
    g = np.random.default_rng(1)
    dt = O.DT("fp32")
    t = g.standard_normal((64, 96)).astype(np.float32)
    G = 32
    deq, code, s, perm = O._sorted_group_quant(t, 4, G, dt, "mean3std")
    assert list(perm) == list(O.stable_argsort(O.mean3std_key(t, dt)))
    for grp in range(3):
        cols = perm[grp * G:(grp + 1) * G]
        sc = O._scales(np.abs(t[:, cols]).max(axis=1), 7, dt)
        np.testing.assert_array_equal(s[:, grp], sc)
