"""GPU: sibling operand reuse (sqmp_permute_act, ops.quant_act_fp).  Layers that quantize the
same input with the same salient set and act mode (q/k/v, gate/up) get the first layer's
operand with its positions moved into their own packed order; that operand must be the one
their own quantizer pass writes, bit for bit (fake_quant.py:291-304: x_hat depends only on x,
the salient set and the act mode; each weight has its own packed order, :157-207)."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _dev():
    if not torch.cuda.is_available():
        pytest.skip("no ROCm device")
    return torch.device("cuda")


def _siblings(dev, M, K, Ns, G, p, dt, seed=0):
    from smoothquant.fake_quant import W4A4Linear
    gen = torch.Generator(device=dev).manual_seed(seed)
    x = torch.randn(M, K, generator=gen, device=dev)
    x[:, torch.randperm(K, generator=gen, device=dev)[: max(1, K // 100)]] *= 30
    imp = x[: min(M, 256)].abs().mean(0).cpu()  # one importance vector: one salient set
    layers = []
    for N in Ns:
        lin = torch.nn.Linear(K, N, bias=True).to(dev, dt)
        with torch.no_grad():
            lin.weight.copy_((torch.randn(N, K, generator=gen, device=dev) * 0.02).to(dt))
            lin.bias.copy_((torch.randn(N, generator=gen, device=dev) * 0.01).to(dt))
        layers.append(W4A4Linear.from_float(lin, weight_quant="per_group", act_quant="per_group",
                                            importance=imp, salient_prop=p, group_size=G))
    return layers, x.to(dt)


@pytest.mark.parametrize("M,K,Ns,G,p,dt", [
    (256, 1024, (512, 256, 256), 64, 0.05, torch.float16),
    (2048, 4096, (4096, 4096, 4096), 64, 0.05, torch.float16),   # Llama q/k/v
    (2048, 4096, (11008, 11008), 64, 0.05, torch.float16),       # Llama gate/up
    (300, 768, (768, 768, 768), 128, 0.10, torch.bfloat16),
    (77, 1024, (256, 512), 128, 0.0, torch.float16),
])
def test_sibling_operand_equals_own_quantization(M, K, Ns, G, p, dt):
    dev = _dev()
    from smoothquant import ops
    layers, x = _siblings(dev, M, K, Ns, G, p, dt)
    pws = [q.packed() for q in layers]
    assert all(ops._sibling_ok(pws[0], pw) for pw in pws[1:])
    old = ops.SIB_REUSE
    try:
        ops.SIB_REUSE = True
        reused = [ops.quant_act_fp(x, pw, "per_group", 4, G) for pw in pws]
        ops.SIB_REUSE = False
        own = [ops.quant_act_fp(x.clone(), pw, "per_group", 4, G) for pw in pws]
    finally:
        ops.SIB_REUSE = old
    for a, b in zip(reused, own):
        assert torch.equal(a.view(torch.int16), b.view(torch.int16))


def test_sibling_forward_bit_identical_and_no_reuse_after_change():
    """Module level: q/k/v forwards with reuse on equal those with reuse off; an input modified
    in place between siblings (a new version) is quantized again, not reused."""
    dev = _dev()
    from smoothquant import ops
    layers, x = _siblings(dev, 512, 2048, (2048, 1024, 1024), 64, 0.05, torch.float16, seed=3)
    old = ops.SIB_REUSE
    try:
        ops.SIB_REUSE = True
        y_on = [q(x) for q in layers]
        ops.SIB_REUSE = False
        y_off = [q(x) for q in layers]
        ops.SIB_REUSE = True
        y0 = layers[0](x)
        x.mul_(1.5)  # in place: a new version of the same tensor
        y1 = layers[1](x)
        ops.SIB_REUSE = False
        y1_ref = layers[1](x)
    finally:
        ops.SIB_REUSE = old
    for a, b in zip(y_on, y_off):
        assert torch.equal(a.view(torch.int16), b.view(torch.int16))
    assert torch.equal(y0.view(torch.int16), y_on[0].view(torch.int16))
    assert torch.equal(y1.view(torch.int16), y1_ref.view(torch.int16))
