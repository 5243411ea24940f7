"""Output quantization with its statistics fused into the GEMM epilogue (fake_quant.py:
308-316; OPT q/k/v quantize their outputs because quantize_opt defaults to
quantize_bmm_input=True, :377-461) on every GEMM that supports it: the activation-order
fqt7 GEMM (per_group, the auto path from 16384 rows) and the FP8 GEMM (per_tensor /
per_token activations, Gw % 128 == 0).

For each: the forward with the fused statistics is BIT-IDENTICAL to the forward with the
separate statistics pass (fake_quant._OQ_FUSE = False), and that output is the reference's
output quantizer (the PyTorch-CPU restatement, oracle/torch_cpu.py) applied to the same
GEMM's own pre-quantization output, bit for bit.
"""
import pytest
import torch

from oracle import torch_cpu as T

pytestmark = pytest.mark.gpu


def _dev():
    if not torch.cuda.is_available():
        pytest.skip("no ROCm device")
    return torch.device("cuda")


CASES = [
    # kernel, act, M, K(=N), G, salient_prop
    ("fqt", "per_group", 300, 1024, 128, 0.05),
    ("fqt", "per_group", 1000, 2048, 64, 0.0),
    ("fqt", "per_group", 16384, 2048, 128, 0.02),     # the auto path (ops.FQT_MIN_ROWS)
    ("f8", "per_tensor", 512, 1024, 128, 0.0),
    ("f8", "per_tensor", 333, 2048, 256, 0.05),
    ("f8", "per_token", 257, 1024, 128, 0.05),        # per_token output: not fused (no stats)
]


@pytest.mark.parametrize("kern,act,M,K,G,p", CASES)
def test_fused_output_quant_bit_exact(kern, act, M, K, G, p):
    dev = _dev()
    from smoothquant import fake_quant as FQ
    from smoothquant import ops
    from smoothquant.fake_quant import W4A4Linear
    gen = torch.Generator(device=dev).manual_seed(M + K)
    lin = torch.nn.Linear(K, K).to(dev, torch.float16)
    with torch.no_grad():
        lin.weight.copy_((torch.randn(K, K, generator=gen, device=dev) * 0.02).half())
    x = torch.randn(M, K, generator=gen, device=dev)
    x[:, torch.randperm(K, generator=gen, device=dev)[: K // 100]] *= 30.0
    x = x.half()
    q = W4A4Linear.from_float(lin, weight_quant="per_group", act_quant=act, quantize_output=True,
                              importance=x[:256].float().abs().mean(0).cpu(), salient_prop=p,
                              group_size=G)
    q.kernel = "auto" if (kern == "fqt" and M >= ops.FQT_MIN_ROWS) or kern == "f8" else kern
    pw = q.packed()
    if kern == "f8":
        assert ops.f8_auto(pw, act, 4)
    seen = []
    real_fqt, real_f8 = ops.gemm_fqt, ops.gemm_f8

    def spy_fqt(*a, **k):
        seen.append(("fqt", k.get("colmax") is not None))
        return real_fqt(*a, **k)

    def spy_f8(*a, **k):
        seen.append(("f8", k.get("colmax") is not None))
        return real_f8(*a, **k)

    ops.gemm_fqt, ops.gemm_f8 = spy_fqt, spy_f8
    try:
        y_fused = q(x.clone())
        FQ._OQ_FUSE = False
        try:
            y_sep = q(x.clone())
        finally:
            FQ._OQ_FUSE = True
    finally:
        ops.gemm_fqt, ops.gemm_f8 = real_fqt, real_f8
    fused_expected = act in ("per_group", "per_tensor")
    assert seen == [(kern, fused_expected), (kern, False)], seen
    assert torch.equal(y_fused.view(torch.int16), y_sep.view(torch.int16))
    # the separate path against the CPU restatement of the reference's output quantizer,
    # applied to this GEMM's own pre-quantization output
    xin = x.clone()
    if kern == "fqt":
        c4 = ops.quant_act_c4(xin, pw, act, 4, G)
        y_pre = ops.gemm_fqt(*c4, pw, q.bias.reshape(-1), G)
    else:
        a8, sa, xs = ops.quant_act_f8(xin, pw, act, 4)
        y_pre = ops.gemm_f8(a8, sa, xs, pw, q.bias.reshape(-1))
    want = y_pre.cpu().clone()
    keep = torch.ones(K, dtype=torch.bool)
    if q.salient_indices is not None:
        keep[q.salient_indices.cpu()] = False
    want[:, keep] = T.act_quant(want[:, keep], act, 4, G)
    assert torch.equal(y_sep.cpu().view(torch.int16), want.view(torch.int16))
