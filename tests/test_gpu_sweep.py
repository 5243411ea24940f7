"""GPU parity for BASELINE config 5: W4A8 (act_quant rebound to 8 bits), the unsorted
groups (sort=none) and the mean+3sigma sort -- through the drop-in module API.

W4A8 and sort=none are pinned to reference-generated fixtures (tests/golden/
sweep_golden.npz, gen_golden_sweep.py); mean+3sigma has no reference implementation and
is checked against the oracle's definition only (parity unpinned).  Tolerances as in
test_gpu_parity.py: W_hat and q_x bit-exact, y relative Frobenius fp32 1e-5 / fp16 2e-3
/ bf16 1e-2 against the oracle's fp64-accumulated product.
"""
import json
import os
from functools import partial

import numpy as np
import pytest
import torch

import sweep_inputs as SI
from oracle import fake_quant_oracle as O
from test_gpu_parity import TOL_FQ, _dev, bits_equal, make_layer, rel, to_np, to_t

pytestmark = pytest.mark.gpu

PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "sweep_golden.npz")
Z = np.load(PATH, allow_pickle=False)
CASES = json.loads(bytes(Z["meta_json"]).decode())["cases"]


def arr(key, dt):
    a = Z[key]
    return (a.astype(np.uint32) << 16).view(np.float32) if dt == "bf16" else a


def case_arrays(m):
    """(W, x, b, importance) as float32 numpy: stored, or re-drawn for digest cases."""
    key, dtn = m["key"], m["dtype"]
    if "index" in m:
        w, b, x, imp = SI.case_inputs(m["index"], m["case"])
        f = lambda t: None if t is None else t.float().numpy()  # noqa: E731
        return f(w), f(x), f(b), imp.numpy().astype(np.float32)
    W, x = arr(key + "_W", dtn), arr(key + "_x", dtn)
    b = arr(key + "_b", dtn) if m["bias"] else None
    return W, x, b, Z[key + "_imp"]


@pytest.mark.parametrize("m", CASES, ids=[f"{c['key']}-{c['dtype']}-{c['sort']}-a{c['act_bits']}-G{c['group_size']}-K{c['K']}" for c in CASES])
def test_sweep_golden(m):
    dev = _dev()
    from smoothquant import fake_quant as FQ
    dtn, key, G = m["dtype"], m["key"], m["group_size"]
    W, x, b, imp = case_arrays(m)
    imp = torch.from_numpy(imp)
    digest = "index" in m
    wq = "per_group" if m["sort"] == "max" else "per_group_unsorted"
    q = make_layer(W, b, dtn, dev, weight_quant=wq, act_quant="per_group", importance=imp,
                   salient_prop=m["salient_prop"], quant_bits=4, group_size=G)
    # the reference user's composition: rebind the bound act quantizer
    fn = (FQ.quantize_activation_per_group_absmax_sort if m["sort"] == "max"
          else FQ.quantize_activation_per_group_absmax)
    q.act_quant = partial(fn, n_bits=m["act_bits"], group_size=G)
    sal = Z[key + "_sal"] if m["has_salient"] else None
    aq = "per_group" if m["sort"] == "max" else "per_group_unsorted"
    if digest:
        assert SI.digest(q.weight) == m["what_sha256"]
        w_hat = O.DT(dtn).f32(O.w4a4_from_float(W, wq, 4, G, sal, O.DT(dtn)))
    else:
        assert bits_equal(to_np(q.weight), arr(key + "_What", dtn))
        w_hat = arr(key + "_What", dtn)
    xt = to_t(x, dtn, dev)
    y = to_np(q(xt.clone()))
    want = O.w4a4_forward(x, w_hat, b, aq, 4, G, sal, False, O.DT(dtn), act_bits=m["act_bits"])
    assert rel(y, want) < TOL_FQ[dtn]
    assert rel(y, arr(key + "_y", dtn)) < TOL_FQ[dtn] * 2
    # q_x through the bound quantizer itself, bit-exact with the reference's q_x
    K = m["K"]
    x2 = xt.reshape(-1, K)
    if sal is not None:
        mask = torch.ones(K, dtype=torch.bool, device=dev)
        mask[torch.from_numpy(sal).to(dev)] = False
        qx = x2.clone()
        qx[:, mask] = q.act_quant(x2[:, mask].contiguous())
    else:
        qx = q.act_quant(x2.clone())
    if digest:
        assert SI.digest(qx) == m["qx_sha256"]
    else:
        assert bits_equal(to_np(qx), arr(key + "_qx", dtn))


@pytest.mark.parametrize("dtn", ["fp16", "bf16", "fp32"])
@pytest.mark.parametrize("G", [32, 64, 128])
def test_mean3std_sort_vs_oracle(dtn, G):
    dev = _dev()
    from smoothquant import fake_quant as FQ
    dt = O.DT(dtn)
    g = np.random.default_rng(G)
    N, K, M = 160, 320, 96
    W = dt.rnd(g.standard_normal((N, K)) * 0.02 * np.exp(g.standard_normal(K) * 0.5))
    b = dt.rnd(g.standard_normal(N) * 0.01)
    x = g.standard_normal((M, K)).astype(np.float32)
    x[:, g.permutation(K)[:5]] *= 30
    x = dt.rnd(x)
    imp = np.abs(x).mean(0).astype(np.float32)
    q = make_layer(W, b, dtn, dev, weight_quant="per_group_mean3std",
                   act_quant="per_group_mean3std", importance=torch.from_numpy(imp),
                   salient_prop=0.05, quant_bits=4, group_size=G)
    sal = O.select_salient(imp, 0.05)
    w_hat = O.w4a4_from_float(W, "per_group_mean3std", 4, G, sal, dt)
    assert bits_equal(to_np(q.weight), w_hat)
    y = to_np(q(to_t(x, dtn, dev)))
    want = O.w4a4_forward(x, w_hat, b, "per_group_mean3std", 4, G, sal, False, dt)
    assert rel(y, want) < TOL_FQ[dtn]
    # the primitive on its own (no salient split), W4A8 rounding
    xa = to_t(x, dtn, dev)
    got = to_np(FQ.quantize_activation_per_group_mean3std_sort(xa, n_bits=8, group_size=G))
    assert bits_equal(got, O.quantize_activation_per_group_mean3std_sort(x, 8, dt, G))
    gw = to_np(FQ.quantize_weight_per_group_mean3std_sort(to_t(W, dtn, dev), n_bits=4,
                                                          group_size=G))
    assert bits_equal(gw, O.quantize_weight_per_group_mean3std_sort(W, 4, dt, G))


def test_w4a8_per_token_both_kernels():
    """W4A8 with per-token activations: the rebinding reaches the faithful kernel (forced
    and auto; 8-bit codes are not exact in e4m3, so auto never takes the FP8 path)."""
    dev = _dev()
    from smoothquant import fake_quant as FQ
    dt = O.DT("fp16")
    g = np.random.default_rng(7)
    N, K, M, G = 256, 512, 64, 128
    W = dt.rnd(g.standard_normal((N, K)) * 0.02)
    x = dt.rnd(g.standard_normal((M, K)))
    imp = np.abs(x).mean(0).astype(np.float32)
    q = make_layer(W, None, "fp16", dev, weight_quant="per_group", act_quant="per_token",
                   importance=torch.from_numpy(imp), salient_prop=0.1, quant_bits=4,
                   group_size=G)
    q.act_quant = partial(FQ.quantize_activation_per_token_absmax, n_bits=8)
    sal = O.select_salient(imp, 0.1)
    w_hat = O.w4a4_from_float(W, "per_group", 4, G, sal, dt)
    want = O.w4a4_forward(x, w_hat, None, "per_token", 4, G, sal, False, dt, act_bits=8)
    for kern, tol in (("fq", 2e-3), ("auto", 2e-3)):
        q.kernel = kern
        y = to_np(q(to_t(x, "fp16", dev)))
        assert rel(y, want) < tol, kern


def test_unsupported_quantizer_raises():
    dev = _dev()
    q = make_layer(np.zeros((64, 128), np.float32), None, "fp16", dev, weight_quant="per_group",
                   act_quant="per_group", group_size=64)
    q.act_quant = lambda t: t
    with pytest.raises(NotImplementedError):
        q(torch.zeros(4, 128, dtype=torch.float16, device=dev))
