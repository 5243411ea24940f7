"""GPU: the activation quantizer's A operand (ops.quant_act_fp) against the CPU oracle,
BIT-EXACT including the sign of zero (the reference's fake quantizer yields -0.0 for small
negative values, fake_quant.py:142), over the shapes that select each kernel variant:
rank ranges of one or many waves (K up to 11008), group sizes below / at / above the
per-thread rank count, odd M (a half row pair), 4- and 8-bit codes, every act mode."""
import numpy as np
import pytest
import torch

from oracle import fake_quant_oracle as O
from test_gpu_parity import TORCH_DT, _dev

pytestmark = pytest.mark.gpu

CASES = [
    # M, K, G, act, dtype, salient_prop, bits
    (256, 4096, 64, "per_group", "fp16", 0.05, 4),
    (129, 4096, 128, "per_group", "bf16", 0.10, 4),
    (129, 11008, 64, "per_group", "fp16", 0.05, 4),
    (64, 11008, 64, "per_group", "bf16", 0.05, 4),
    (64, 1024, 8, "per_group", "fp16", 0.10, 4),
    (64, 1024, 16, "per_group_unsorted", "bf16", 0.0, 4),
    (64, 2048, 1024, "per_group", "fp16", 0.05, 4),
    (63, 4096, 64, "per_token", "fp16", 0.05, 4),
    (64, 4096, 64, "per_token", "bf16", 0.0, 4),
    (64, 4096, 64, "per_tensor", "bf16", 0.10, 4),
    (64, 2048, 64, "per_group", "fp16", 0.05, 8),
    (64, 4096, 64, "per_group_mean3std", "fp16", 0.05, 4),
    (96, 8192, 128, "per_group", "fp16", 0.05, 4),
    (2, 4096, 32, "per_group", "fp16", 0.05, 4),
    # fp32 (OPT): register-staged wave kernel (K <= 4096) and the LDS wave kernel (longer)
    (64, 2048, 128, "per_group", "fp32", 0.05, 4),
    (65, 8192, 128, "per_group", "fp32", 0.05, 4),
    (64, 8192, 64, "per_token", "fp32", 0.05, 4),
    (33, 6144, 128, "per_tensor", "fp32", 0.10, 4),
    (64, 4096, 128, "per_group_mean3std", "fp32", 0.05, 4),
]


def _bits(a, dtn):
    a = np.asarray(a, np.float32)
    if dtn == "fp32":
        return a.view(np.uint32)
    if dtn == "fp16":
        return a.astype(np.float16).view(np.uint16)
    return (a.view(np.uint32) >> 16).astype(np.uint16)


@pytest.mark.parametrize("case", CASES, ids=[f"{c[0]}x{c[1]}-G{c[2]}-{c[3]}-{c[4]}-p{c[5]}-b{c[6]}" for c in CASES])
def test_quant_act_operand_bit_exact(case):
    dev = _dev()
    from smoothquant import ops
    from smoothquant.fake_quant import W4A4Linear
    M, K, G, act, dtn, p, bits = case
    dt = O.DT(dtn)
    g = np.random.default_rng(K + M + G)
    x = g.standard_normal((M, K)).astype(np.float32)
    x[:, g.permutation(K)[: max(1, K // 100)]] *= 30
    x[:, 5] = 0.0                       # a zero column
    x[0, :] *= 1e-3                     # a row of small values (many -0.0 codes)
    x = dt.rnd(x)
    imp = np.abs(x).mean(0).astype(np.float32)
    lin = torch.nn.Linear(K, 256, bias=False).to(dev, TORCH_DT[dtn])
    with torch.no_grad():
        lin.weight.copy_(torch.from_numpy(g.standard_normal((256, K)).astype(np.float32) * 0.02))
    q = W4A4Linear.from_float(lin, weight_quant="per_group", act_quant="per_group",
                              importance=torch.from_numpy(imp), salient_prop=p,
                              quant_bits=4, group_size=64 if G > 4096 else G)
    pw = q.packed()
    xt = torch.from_numpy(x).to(dev, TORCH_DT[dtn])
    a = ops.quant_act_fp(xt, pw, act, bits, G).float().cpu().numpy()
    sal = O.select_salient(imp, p)
    qx = O.quantize_input(x, act, bits, G, sal, dt)
    amap = pw.amap.cpu().numpy()
    want = np.zeros_like(a)
    v = amap >= 0
    want[:, :pw.Kp][:, v] = qx[:, amap[v]]
    if sal is not None:
        want[:, pw.Kp:pw.Kp + pw.S] = qx[:, sal]
    got_b, want_b = _bits(a, dtn), _bits(want, dtn)
    bad = np.argwhere(got_b != want_b)
    assert len(bad) == 0, (f"{len(bad)} of {a.size} differ; first "
                           f"{[(int(m), int(c), float(a[m, c]), float(want[m, c])) for m, c in bad[:5]]}")


@pytest.mark.parametrize("act,dtn,oq", [("per_group", "fp16", False),
                                         ("per_group_mean3std", "fp16", False),
                                         ("per_group", "fp32", False),
                                         ("per_group", "fp32", True),
                                         ("per_group", "fp16", True)])
def test_sibling_layers_share_statistics(act, dtn, oq):
    """q/k/v-style siblings (same input object, same salient set) reuse the first layer's
    column statistics and rank: outputs are bit-identical to independent computation (also
    with the OPT pattern of each sibling quantizing its output in between, on workspaces of
    its own), and an in-place change of the input between calls invalidates the reuse."""
    dev = _dev()
    from smoothquant.fake_quant import W4A4Linear
    dt = TORCH_DT[dtn]
    g = torch.Generator(device=dev).manual_seed(3)
    K, M = 1024, 96
    N = K if oq else 320
    x = torch.randn(M, K, generator=g, device=dev).to(dt)
    imp = x.float().abs().mean(0).cpu()
    layers = []
    for i in range(3):
        lin = torch.nn.Linear(K, N, bias=True).to(dev, dt)
        with torch.no_grad():
            lin.weight.copy_(torch.randn(N, K, generator=g, device=dev) * 0.02)
        layers.append(W4A4Linear.from_float(lin, weight_quant="per_group", act_quant=act,
                                            quantize_output=oq, importance=imp,
                                            salient_prop=0.05, group_size=64))
    shared = [q(x) for q in layers]
    alone = [q(x.clone()) for q in layers]
    for a, b in zip(shared, alone):
        assert torch.equal(a, b)
    # in-place update of the shared input: the next sibling must not reuse stale statistics
    layers[0](x)
    x.mul_(-0.5).add_(0.25)
    y1 = layers[1](x)
    assert torch.equal(y1, layers[1](x.clone()))


TIE_CASES = [
    # M, K, dtype, salient_prop  (list lengths select every sort-table block shape)
    (4, 1024, "fp16", 0.0), (3, 2048, "bf16", 0.05), (4, 4096, "fp16", 0.05),
    (2, 8192, "bf16", 0.05), (5, 11008, "fp16", 0.05), (2, 16384, "fp16", 0.02),
    (2, 18432, "fp16", 0.02),  # list > RT_MAX: rank_count + lc_table
]


@pytest.mark.parametrize("case", TIE_CASES, ids=[f"{c[0]}x{c[1]}-{c[2]}-p{c[3]}" for c in TIE_CASES])
def test_sorted_groups_tie_order(case):
    """Small-integer activations over few rows: most column maxima tie, so the group
    assignment depends on the stable tie rule of the reference's argsort (fake_quant.py:113,
    equal keys keep column order).  Bit-exact A operand against the oracle."""
    dev = _dev()
    from smoothquant import ops
    from smoothquant.fake_quant import W4A4Linear
    M, K, dtn, p = case
    dt = O.DT(dtn)
    g = np.random.default_rng(K + M)
    x = dt.rnd(np.round(g.standard_normal((M, K)) * 2.0).astype(np.float32))
    x[:, g.permutation(K)[:8]] = 0.0
    imp = (np.abs(x).mean(0) + g.random(K) * 1e-3).astype(np.float32)
    lin = torch.nn.Linear(K, 128, bias=False).to(dev, TORCH_DT[dtn])
    q = W4A4Linear.from_float(lin, weight_quant="per_group", act_quant="per_group",
                              importance=torch.from_numpy(imp), salient_prop=p, group_size=64)
    pw = q.packed()
    a = ops.quant_act_fp(torch.from_numpy(x).to(dev, TORCH_DT[dtn]), pw, "per_group", 4, 64)
    a = a.float().cpu().numpy()
    sal = O.select_salient(imp, p)
    qx = O.quantize_input(x, "per_group", 4, 64, sal, dt)
    amap = pw.amap.cpu().numpy()
    want = np.zeros_like(a)
    v = amap >= 0
    want[:, :pw.Kp][:, v] = qx[:, amap[v]]
    if sal is not None:
        want[:, pw.Kp:pw.Kp + pw.S] = qx[:, sal]
    bad = np.argwhere(_bits(a, dtn) != _bits(want, dtn))
    assert len(bad) == 0, f"{len(bad)} of {a.size} differ; first {bad[:5].tolist()}"


INPLACE_CASES = [
    # M, K, G, act, dtype, salient_prop -- the in-place output quantizer (fake_quant.py:308-316)
    (64, 2048, 128, "per_group", "fp32", 0.05),
    (33, 8192, 128, "per_group", "fp32", 0.05),
    (64, 2048, 128, "per_token", "fp32", 0.0),
    (64, 2048, 64, "per_tensor", "fp32", 0.10),
    (64, 2048, 128, "per_group", "fp16", 0.05),
]


@pytest.mark.parametrize("case", INPLACE_CASES,
                         ids=[f"{c[0]}x{c[1]}-G{c[2]}-{c[3]}-{c[4]}-p{c[5]}" for c in INPLACE_CASES])
def test_inplace_output_quant_bit_exact(case):
    """y quantized in place over its non-salient columns, salient columns passing through
    (the oracle's quantize_input on y), bit-exact."""
    dev = _dev()
    from smoothquant import ops
    from smoothquant.fake_quant import W4A4Linear
    M, K, G, act, dtn, p = case
    dt = O.DT(dtn)
    g = np.random.default_rng(K + M + 7)
    y = g.standard_normal((M, K)).astype(np.float32)
    y[:, g.permutation(K)[: max(1, K // 100)]] *= 30
    y = dt.rnd(y)
    imp = np.abs(y).mean(0).astype(np.float32)
    lin = torch.nn.Linear(K, K, bias=False).to(dev, TORCH_DT[dtn])
    q = W4A4Linear.from_float(lin, weight_quant="per_group", act_quant=act,
                              importance=torch.from_numpy(imp), salient_prop=p,
                              quant_bits=4, group_size=G)
    pw = q.packed()
    yt = torch.from_numpy(y).to(dev, TORCH_DT[dtn])
    ops.fake_quant_inplace(yt, act, 4, G, pw.amap_fq, pw.nonsal, pw.S)
    got = yt.float().cpu().numpy()
    want = O.quantize_input(y, act, 4, G, O.select_salient(imp, p), dt)
    bad = np.argwhere(_bits(got, dtn) != _bits(want, dtn))
    assert len(bad) == 0, (f"{len(bad)} of {got.size} differ; first "
                           f"{[(int(m), int(c), float(got[m, c]), float(want[m, c])) for m, c in bad[:5]]}")
