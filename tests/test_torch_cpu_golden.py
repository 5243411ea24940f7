"""Pin oracle/torch_cpu.py (bench.py's CPU baseline: the reference's fake-quant layer on
PyTorch-CPU) against the reference-generated goldens: W_hat and q_x BIT-EXACT in fp32,
fp16 and bf16, and y equal to the reference's own CPU F.linear output (same torch op on
the same operands; compared with the CPU accumulation-order tolerance of
test_oracle_golden.py in case the BLAS picks another kernel)."""
import numpy as np
import pytest
import torch

from golden_io import Golden
from oracle import torch_cpu as T

G = Golden()
LAYERS = G.meta["layers"]
TDT = {"fp32": torch.float32, "fp16": torch.float16, "bf16": torch.bfloat16}
Y_TOL = {"fp32": 1e-6, "fp16": 2e-3, "bf16": 1e-2}


def _t(key, dt):
    a = G.z[key]
    if dt == "bf16":
        return torch.from_numpy(a.astype(np.int16)).view(torch.bfloat16)
    return torch.from_numpy(np.ascontiguousarray(a)).to(TDT[dt])


def _same_bits(a: torch.Tensor, b: torch.Tensor) -> bool:
    # -0.0 and +0.0 compare equal (the integer codes of the packed path give +0.0)
    return a.shape == b.shape and bool(torch.equal(a.float(), b.float()))


@pytest.mark.parametrize("m", LAYERS, ids=[l["key"] for l in LAYERS])
def test_torch_cpu_layer_matches_reference(m):
    dt, key = m["dtype"], m["key"]
    if m["act_quant"] not in ("per_token", "per_tensor", "per_group"):
        pytest.skip("composition case")
    W, x = _t(key + "_W", dt), _t(key + "_x", dt)
    b = _t(key + "_b", dt) if m["bias"] else None
    imp = torch.from_numpy(G.z[key + "_imp"])
    layer = T.CPUFakeQuantLinear(W, b, m["weight_quant"], m["act_quant"], m["n_bits"],
                                 m["group_size"], imp, m["salient_prop"], m["quantize_output"])
    if m["has_salient"]:
        assert np.array_equal(layer.salient.numpy(), G.z[key + "_sal"])
    assert _same_bits(layer.w_hat, _t(key + "_What", dt))
    K = m["K"]
    qx = layer.quantize_input(x.reshape(-1, K))
    assert _same_bits(qx, _t(key + "_qx", dt).reshape(-1, K))
    y = layer(x.clone()).double().numpy()
    want = _t(key + "_y", dt).double().numpy()
    rel = np.linalg.norm(y - want) / np.linalg.norm(want)
    tol = Y_TOL[dt] * (10 if m["quantize_output"] else 1) + (1e-6 if m["quantize_output"] else 0)
    assert rel < tol, rel
