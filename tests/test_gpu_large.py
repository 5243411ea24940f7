"""Size-independent parity at serving-scale batches (up to 131072 tokens, 1 GiB inputs).

The reference quantizes activations over the WHOLE batch (/root/reference/smoothquant/
fake_quant.py:104-154: the column order is argsort of x.abs().max(dim=0) over every row;
:56-75: per_token scales per row, per_tensor one scale for the tensor) and then runs F.linear
(:306) row by row.  A batch made of r copies of x0 therefore has the same column maxima, the
same stable order, the same per-row group scales and codes, and each output row is x0's row:

    forward(cat([x0] * r)) == cat([forward(x0)] * r)      (bit for bit)

whenever both launches take the same kernel and the same K-accumulation order (the HIP
kernels fix each output's order per kernel variant, independent of M).  Where the launch
plans differ (the packed-order GEMM's in-workgroup K split, ops.fq7_plan OPT bit 16) the
partial sums add in another order and the copies must agree within the pair tolerance
instead.  These checks reach sizes the CPU oracle cannot finish inside a test and exercise
the row offsets of every kernel on the path past 2^31 bytes: inputs of 1 GiB, outputs of
1 GiB, ragged row counts.
"""
import pytest
import torch

pytestmark = pytest.mark.gpu

PAIR_TOL = 1e-3   # fp32 partial sums in another order (tests/test_gpu_fq7.py::test_fq7_ksplit)


def _dev():
    if not torch.cuda.is_available():
        pytest.skip("no ROCm device")
    return torch.device("cuda")


def _rel(a, b):
    a, b = a.double(), b.double()
    return float((a - b).norm() / b.norm().clamp_min(1e-30))


def _layer(dev, M0, K, N, G, p, dt, aq="per_group", wq="per_group", seed=0):
    from smoothquant.fake_quant import W4A4Linear
    gen = torch.Generator(device=dev).manual_seed(seed)
    x = torch.randn(M0, K, generator=gen, device=dev)
    x[:, torch.randperm(K, generator=gen, device=dev)[: max(1, K // 100)]] *= 30
    lin = torch.nn.Linear(K, N, bias=True).to(dev, dt)
    with torch.no_grad():
        lin.weight.copy_((torch.randn(N, K, generator=gen, device=dev) * 0.02).to(dt))
        lin.bias.copy_((torch.randn(N, generator=gen, device=dev) * 0.01).to(dt))
    imp = x[: min(M0, 512)].abs().mean(0).cpu()
    q = W4A4Linear.from_float(lin, weight_quant=wq, act_quant=aq, importance=imp,
                              salient_prop=p, group_size=G)
    return q, x.to(dt)


def _check_replicated(q, x0, r, exact=True):
    y0 = q(x0)
    big = x0.repeat(r, 1)
    yb = q(big)
    torch.cuda.synchronize()
    assert yb.shape == (r * x0.shape[0], y0.shape[1])
    assert torch.isfinite(yb).all()
    yb = yb.view(r, *y0.shape)
    if exact:
        for i in range(r):
            assert torch.equal(yb[i], y0), f"copy {i} differs from the single batch"
    else:
        for i in range(r):
            assert _rel(yb[i], y0) < PAIR_TOL, i
        # the copies inside one launch still agree with each other bit for bit
        assert torch.equal(yb[0], yb[r - 1])
    del big, yb


@pytest.mark.parametrize("dt,r", [(torch.float16, 8), (torch.bfloat16, 4)])
def test_activation_order_path_replicated(dt, r):
    """Config 2's benchmarked path (sorted per_group act, activation-order fqt7 GEMM) on
    16384 x r tokens: 131072 rows in fp16 (x 1 GiB, y 1 GiB)."""
    dev = _dev()
    from smoothquant import ops
    q, x0 = _layer(dev, 16384, 4096, 4096, 128, 0.10, dt)
    assert ops.fqt_eligible(q.packed(), "per_group", 4, 128, 16384 * r)
    _check_replicated(q, x0, r)


def test_activation_order_path_ragged():
    """A row count that is no multiple of any tile (16411 = 64 * 256 + 27) on the
    activation-order path, twice over: the partial row tile of each copy lands in the middle
    of the doubled batch's tiles."""
    dev = _dev()
    q, x0 = _layer(dev, 16411, 4096, 1000, 128, 0.10, torch.float16, seed=1)
    _check_replicated(q, x0, 2)


@pytest.mark.parametrize("aq", ["per_token", "per_tensor"])
def test_fp8_path_replicated(aq):
    """per_token / per_tensor 4-bit activations on the block-scaled FP8 GEMM, 4096 x 32 =
    131072 tokens (the per-row / per-tensor scales of a replicated batch are the single
    batch's)."""
    dev = _dev()
    q, x0 = _layer(dev, 4096, 4096, 4096, 128, 0.10, torch.float16, aq=aq, seed=2)
    _check_replicated(q, x0, 32)


@pytest.mark.parametrize("K,N", [(4096, 4096), (11008, 4096), (4096, 11008)])
def test_packed_order_path_replicated(K, N):
    """Llama-2-7B shapes on the packed-order fq7 GEMM (below 16384 rows): 2048 tokens and
    4 x 2048.  The two launches may take different K-split variants; the result must then be
    within the pair tolerance, else bit for bit."""
    dev = _dev()
    from smoothquant import ops
    q, x0 = _layer(dev, 2048, K, N, 64, 0.05, torch.float16, seed=3)
    pw = q.packed()
    r = 4
    assert 2048 * r < ops.FQT_MIN_ROWS  # both launches on the packed-order path
    same = True
    if ops.fq7_eligible(pw):
        a = ops.fq7_plan([pw], 2048, group=False)
        b = ops.fq7_plan([pw], 2048 * r, group=False)
        same = not ((a[1] ^ b[1]) & 16)
    _check_replicated(q, x0, r, exact=same)


def test_fp32_path_replicated():
    """The fp32 layer (the reference's OPT dtype: h2d GEMM on the quantizer's two fp16 planes)
    at 8 x 2048 tokens."""
    dev = _dev()
    q, x0 = _layer(dev, 2048, 2048, 2048, 128, 0.05, torch.float32, seed=4)
    _check_replicated(q, x0, 8)
