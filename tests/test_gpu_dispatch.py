"""GPU tests of the forward dispatcher's eligibility rules and of from_float on a
CPU-resident source Linear.

  * ops.fqt_eligible mirrors the C4 quantizer's limits (quant_lc_supported: power-of-two
    groups of 64 .. 1024 ranks): at the auto row threshold a per_group layer with G = 2048
    (the reference's sweeps go to 1024, run_experiments.py:262; 2048 is a legal
    group_size of fake_quant.py:104-154) or G = 192 runs on the packed-order path and
    matches the oracle instead of raising;
  * from_float on a Linear still on the CPU (the usual state of a model before .cuda())
    packs on the GPU and, for per_channel / per_tensor, writes W_hat back into the
    source weight in place as the reference does (fake_quant.py:349-355, :363-365).
"""
import numpy as np
import pytest
import torch

from oracle import torch_cpu as T

pytestmark = pytest.mark.gpu


def _dev():
    if not torch.cuda.is_available():
        pytest.skip("no ROCm device")
    return torch.device("cuda")


def _rel(a, b):
    a, b = a.detach().double().cpu(), b.detach().double().cpu()
    return float((a - b).norm() / b.norm().clamp_min(1e-30))


@pytest.mark.parametrize("G", [2048, 192])
def test_auto_path_group_sizes_outside_fqt(G):
    dev = _dev()
    from smoothquant import ops
    from smoothquant.fake_quant import W4A4Linear
    M, K, N = ops.FQT_MIN_ROWS, 4096, 256
    gen = torch.Generator(device=dev).manual_seed(G)
    x = torch.randn(M, K, generator=gen, device=dev).half()
    lin = torch.nn.Linear(K, N).to(dev, torch.float16)
    with torch.no_grad():
        lin.weight.copy_((torch.randn(N, K, generator=gen, device=dev) * 0.02).half())
    imp = x[:512].float().abs().mean(0).cpu()
    q = W4A4Linear.from_float(lin, weight_quant="per_group", act_quant="per_group",
                              importance=imp, salient_prop=0.05, group_size=G)
    assert not ops.fqt_eligible(q.packed(), "per_group", 4, G, M)
    y = q(x)
    # oracle on sampled rows (batch-wide sort over every row)
    xc = x.cpu()
    sal = q.salient_indices.cpu()
    keep = torch.ones(K, dtype=torch.bool)
    keep[sal] = False
    qx = xc.clone()
    qx[:, keep] = T.act_quant(xc[:, keep], "per_group", 4, G)
    w_hat = T.quantize_weight(lin.weight.detach().cpu(), "per_group", 4, G, sal)
    rows = torch.arange(0, M, 97)
    ref = qx[rows].double() @ w_hat.double().t() + lin.bias.detach().cpu().double()
    assert _rel(y[rows.to(dev)], ref) < 2e-3


@pytest.mark.parametrize("wq", ["per_channel", "per_tensor", "per_group"])
def test_from_float_cpu_source_linear(wq):
    dev = _dev()
    from smoothquant.fake_quant import W4A4Linear
    torch.manual_seed(3)
    K, N = 512, 192
    lin = torch.nn.Linear(K, N).half()                      # stays on the CPU
    w0 = lin.weight.detach().clone()
    b0 = lin.bias.detach().clone()   # from_float aliases the bias Parameter (:369-370)
    imp = torch.rand(K)
    q = W4A4Linear.from_float(lin, weight_quant=wq, act_quant="per_token", importance=imp,
                              salient_prop=0.05, group_size=128)
    assert q.w_codes.device.type == "cpu"                  # moved back to the source device
    sal = q.salient_indices
    w_hat = T.quantize_weight(w0, wq, 4, 128, sal)
    if wq in ("per_channel", "per_tensor"):
        assert torch.equal(lin.weight.detach(), w_hat)      # in place, like the reference
    else:
        assert torch.equal(lin.weight.detach(), w0)         # per_group returns a new tensor
    q = q.to(dev)
    assert torch.equal(q.weight.cpu(), w_hat)
    x = torch.randn(64, K).half()
    y = q(x.to(dev))
    keep = torch.ones(K, dtype=torch.bool)
    keep[sal] = False
    qx = x.clone()
    qx[:, keep] = T.act_quant(x[:, keep], "per_token", 4, 128)
    ref = qx.double() @ w_hat.double().t() + b0.double()
    assert _rel(y, ref) < 3e-3
