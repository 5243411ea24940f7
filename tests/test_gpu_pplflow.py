"""The reference's SmoothQuant baseline evaluation flow (smoothquant/ppl_eval.py:69-83,
examples/ppl_eval.sh): a bf16 model, quantize_model(weight_quant="per_channel",
act_quant="per_token", quantize_bmm_input=True) with no calibration features, i.e. no salient
channels.  There the reference's act quantizer rewrites the caller's x in place
(fake_quant.py:56-75 via :304) and q/k/v quantize their outputs (:308-316).

Round 6 made that flow take one quantizer pass per linear: the in-place quantization of x IS
the GEMM operand when the packed order is the column order (ops.identity_layout), and the
in-place quantizers of consecutive layers reuse the list table they leave in their workspace
(SQMP_QA_TABLE_READY).  These tests pin both against the two-pass path they replace, bit for
bit, and the table reuse against fresh workspaces across interleaved modes, dtypes, row counts
and the quantizers' fallback path.
"""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _dev():
    if not torch.cuda.is_available():
        pytest.skip("no ROCm device")
    return torch.device("cuda")


def _linear(dev, K, N, dt, seed, bias=True):
    from smoothquant.fake_quant import W4A4Linear
    gen = torch.Generator(device=dev).manual_seed(seed)
    lin = torch.nn.Linear(K, N, bias=bias).to(dev, dt)
    with torch.no_grad():
        lin.weight.copy_((torch.randn(N, K, generator=gen, device=dev) * 0.02).to(dt))
        if bias:
            lin.bias.copy_((torch.randn(N, generator=gen, device=dev) * 0.01).to(dt))
    return W4A4Linear.from_float(lin, weight_quant="per_channel", act_quant="per_token",
                                 quantize_output=False)


def _x(dev, M, K, dt, seed):
    gen = torch.Generator(device=dev).manual_seed(seed)
    x = torch.randn(M, K, generator=gen, device=dev)
    x[:, torch.randperm(K, generator=gen, device=dev)[: max(1, K // 100)]] *= 30
    return x.to(dt)


def _two_pass(q, x):
    """The path before round 6: the OUT_FP operand from an untouched copy, then the in-place
    quantization of x, then the GEMM on the operand (fresh workspaces for every call)."""
    from smoothquant import ops
    from smoothquant.fake_quant import resolve_quantizer
    pw = q.packed()
    mode, bits, g = resolve_quantizer(q.act_quant)
    ops._WS.clear()
    a = ops.quant_act_fp(x.clone(), pw, mode, bits, g)
    ops._WS.clear()
    ops.fake_quant_inplace(x, mode, bits, g, pw.amap_fq, pw.nonsal, 0)
    ops._WS.clear()
    b = None if q.bias is None else q.bias.reshape(-1)
    return ops.gemm_fq(a, pw, b)


@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("M", [2048, 300])
def test_inplace_operand_matches_two_pass(dt, M):
    """forward == the two-pass path, y and the mutated x bit for bit; M = 300 takes the
    padded copy of the quantized rows (the GEMM's tiles read past M)."""
    dev = _dev()
    from smoothquant import ops
    q = _linear(dev, 4096, 1536, dt, seed=1)
    assert ops.identity_layout(q.packed())
    x0 = _x(dev, M, 4096, dt, seed=2)
    xa, xb = x0.clone(), x0.clone()
    y_new = q(xa)
    y_old = _two_pass(q, xb)
    assert torch.equal(xa, xb), "the caller's x is quantized in place as before"
    assert torch.equal(y_new, y_old)
    assert not torch.equal(xa, x0)


def test_identity_layout_only_without_salient_or_sort():
    dev = _dev()
    from smoothquant import ops
    from smoothquant.fake_quant import W4A4Linear
    lin = torch.nn.Linear(512, 256, bias=False).to(dev, torch.bfloat16)
    imp = torch.rand(512)
    q1 = W4A4Linear.from_float(lin, weight_quant="per_channel", act_quant="per_token",
                               importance=imp, salient_prop=0.05)
    q2 = W4A4Linear.from_float(lin, weight_quant="per_group", act_quant="per_token",
                               group_size=128)
    q3 = W4A4Linear.from_float(lin, weight_quant="per_channel", act_quant="per_token")
    assert not ops.identity_layout(q1.packed())       # salient columns move to the tail
    assert not ops.identity_layout(q2.packed())       # weight-sorted packed order
    assert ops.identity_layout(q3.packed())


def test_table_reuse_across_modes_matches_fresh_workspaces():
    """In-place quantizers on one workspace (C = 4096), interleaving per_token (table reused),
    sorted per_group (rank table over the same region), per_tensor (no table), unsorted
    per_group, a misaligned view (the quantizers' fallback path) and fp32 rows: every result
    equals the same call on a fresh workspace."""
    dev = _dev()
    from smoothquant import ops
    from smoothquant.fake_quant import _fq_act
    seq = [("per_token", torch.bfloat16, 2048), ("per_token", torch.bfloat16, 512),
           ("per_group", torch.bfloat16, 2048), ("per_token", torch.bfloat16, 2048),
           ("per_tensor", torch.bfloat16, 1000), ("per_token", torch.bfloat16, 2048),
           ("per_group_unsorted", torch.bfloat16, 2048), ("per_token", torch.float16, 777),
           ("misaligned", torch.bfloat16, 2048), ("per_token", torch.bfloat16, 2048),
           ("per_token", torch.float32, 640), ("per_token", torch.bfloat16, 64)]
    ops._WS.clear()
    for i, (mode, dt, M) in enumerate(seq):
        x = _x(dev, M, 4096, dt, seed=10 + i)
        m = "per_token" if mode == "misaligned" else mode
        want = x.clone()
        saved = dict(ops._WS)
        ops._WS.clear()
        _fq_act(want, m, 4, 128)                              # a fresh workspace
        ops._WS.clear()
        ops._WS.update(saved)
        if mode == "misaligned":
            # rows 2 B off a 16-B boundary: the lane-contiguous quantizer refuses them and the
            # general path quantizes (it must leave the list table behind all the same)
            flat = torch.empty(M * 4096 + 8, dtype=dt, device=dev)
            got = flat[1:1 + M * 4096].view(M, 4096)
            got.copy_(x)
        else:
            got = x.clone()
        _fq_act(got, m, 4, 128)
        assert torch.equal(got, want), (i, mode, dt, M)


def test_pplflow_layer_matches_oracle_shapes():
    """A Llama-shaped bf16 ppl_eval-flow layer (q/k/v with output quantization, o, gate, up,
    down at 2048 tokens, the reference's in-place chain: k and v quantize the x that q
    already quantized): every output equals the two-pass path, each member's y within the
    bf16 GEMM tolerance of the fp64 product of its operands."""
    dev = _dev()
    from smoothquant import ops
    from smoothquant.fake_quant import W4A4Linear
    gen = torch.Generator(device=dev).manual_seed(5)
    shapes = [("q", 4096, 4096, True), ("k", 4096, 4096, True), ("v", 4096, 4096, True),
              ("o", 4096, 4096, False), ("gate", 4096, 11008, False),
              ("up", 4096, 11008, False), ("down", 11008, 4096, False)]
    x_attn = _x(dev, 2048, 4096, torch.bfloat16, 6)
    x_mlp = _x(dev, 2048, 4096, torch.bfloat16, 7)
    ins = {"q": x_attn, "k": x_attn, "v": x_attn, "o": _x(dev, 2048, 4096, torch.bfloat16, 8),
           "gate": x_mlp, "up": x_mlp, "down": _x(dev, 2048, 11008, torch.bfloat16, 9)}
    copies = {id(v): (v.clone(), v.clone()) for v in ins.values()}
    for name, K, N, oq in shapes:
        lin = torch.nn.Linear(K, N, bias=False).to(dev, torch.bfloat16)
        with torch.no_grad():
            lin.weight.copy_((torch.randn(N, K, generator=gen, device=dev) * 0.02).bfloat16())
        q = W4A4Linear.from_float(lin, weight_quant="per_channel", act_quant="per_token",
                                  quantize_output=oq)
        xa, xb = copies[id(ins[name])]
        y = q(xa)
        y_old = _two_pass(q, xb)
        if oq:
            ops._WS.clear()
            from smoothquant.fake_quant import _fq_act
            _fq_act(y_old, "per_token", 4)
        assert torch.equal(xa, xb), name
        assert torch.equal(y, y_old), name
        # the GEMM against fp64 on the quantized operand (bf16 output rounding)
        if not oq:
            ref = xb.double() @ q.weight.double().t()
            rel = float((y.double() - ref).norm() / ref.norm())
            assert rel < 8e-3, (name, rel)


@pytest.mark.parametrize("dt", [torch.float16, torch.bfloat16])
@pytest.mark.parametrize("M,K", [(1, 8), (3, 4096), (2048, 4096), (7, 11008), (5, 16392),
                                 (4, 32768), (3, 32776), (2, 40000), (2, 24)])
def test_token_rows_inplace_matches_oracle(dt, M, K):
    """The row-pair in-place per-token quantizer (launch_token_rows, K % 8 == 0: rows cached
    in registers up to K = 32768, streamed twice beyond) against the PyTorch-CPU restatement of
    fake_quant.py:56-64 (oracle/torch_cpu.py, pinned to the reference goldens), bit for bit,
    signed zeros included; outliers x30 and an all-zero row (scale clamp at 1e-5)."""
    dev = _dev()
    from oracle import torch_cpu as T
    from smoothquant.fake_quant import _fq_act
    x = _x(dev, M, K, dt, seed=M * 7 + K)
    x[0, : min(K, 16)] = -1e-4           # small negatives -> -0.0 after the round
    if M > 2:
        x[2] = 0                         # an all-zero row
    want = T.act_quant(x.cpu(), "per_token", 4, 128)
    got = x.clone()
    _fq_act(got, "per_token", 4)
    assert torch.equal(got.cpu().view(torch.int16), want.view(torch.int16))


@pytest.mark.parametrize("M,K,N", [(2048, 4096, 4096), (301, 11008, 1024), (64, 4224, 520)])
def test_f8_write_x_matches_two_passes(M, K, N):
    """fp16 per_token without salient channels (quantize_llama_like's defaults) on the FP8
    path: one pass writes the e4m3 codes, the row scales and x_hat over x (SQMP_QA_WRITE_X);
    codes, scales, the mutated x and y equal the two-pass path (the table-driven F8 quantizer,
    then the in-place quantizer), bit for bit."""
    dev = _dev()
    from smoothquant import ops
    q = _linear(dev, K, N, torch.float16, seed=M + K)
    pw = q.packed()
    x0 = _x(dev, M, K, torch.float16, seed=K)
    assert ops.f8_auto(pw, "per_token", 4) and ops.f8_write_x_ok(x0, pw, "per_token", 4)
    xa, xb = x0.clone(), x0.clone()
    a8n, san, _ = ops.quant_act_f8(xa, pw, "per_token", 4, write_x=True)
    a8o, sao, xs = ops.quant_act_f8(xb, pw, "per_token", 4)
    ops.fake_quant_inplace(xb, "per_token", 4, 128, pw.amap_fq, pw.nonsal, 0)
    torch.cuda.synchronize()
    assert torch.equal(a8n, a8o) and torch.equal(san, sao)
    assert torch.equal(xa, xb)
    xc, xd = x0.clone(), x0.clone()
    y = q(xc)                                    # the forward takes the one-pass form
    b = q.bias.reshape(-1)
    y_old = ops.gemm_f8(a8o, sao, xs, pw, b)
    assert torch.equal(xc, xb) and torch.equal(y, y_old)
