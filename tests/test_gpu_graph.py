"""Graph capture: every C entry enqueues on the given stream without host synchronisation or
allocation (include/sqmp_w4a4.h, "Conventions"), so a W4A4Linear forward can be captured into
a HIP graph (torch.cuda.graph) and replayed.  Replays on new input data give the bits the
eager forward gives on that data, for the per_group packed-order path, the per_token FP8
path, the activation-order path and a linked sibling group (q/k/v)."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _dev():
    if not torch.cuda.is_available():
        pytest.skip("no ROCm device")
    return torch.device("cuda", 0)


def _layer(dev, K, N, act, G, p, seed):
    from smoothquant.fake_quant import W4A4Linear
    gen = torch.Generator(device=dev).manual_seed(seed)
    lin = torch.nn.Linear(K, N, bias=True).to(dev, torch.float16)
    with torch.no_grad():
        lin.weight.copy_((torch.randn(N, K, generator=gen, device=dev) * 0.02).half())
        lin.bias.copy_((torch.randn(N, generator=gen, device=dev) * 0.01).half())
    imp = torch.rand(K, generator=gen, device=dev).cpu() + 0.1
    return W4A4Linear.from_float(lin, weight_quant="per_group", act_quant=act, importance=imp,
                                 salient_prop=p, group_size=G)


def _inputs(dev, M, K, seed, n):
    gen = torch.Generator(device=dev).manual_seed(seed)
    xs = []
    for _ in range(n):
        x = torch.randn(M, K, generator=gen, device=dev)
        x[:, torch.randperm(K, generator=gen, device=dev)[: K // 64]] *= 25
        xs.append(x.half())
    return xs


def _check_graph(fwd, static_x, xs):
    """Capture fwd(static_x) once, then for every x: copy into static_x, replay, compare with
    the eager fwd(x)."""
    s = torch.cuda.Stream(static_x.device)
    s.wait_stream(torch.cuda.current_stream(static_x.device))
    with torch.cuda.stream(s):
        for _ in range(2):  # warm-up on the capture stream (workspaces, kernel attributes)
            fwd(static_x)
    torch.cuda.current_stream(static_x.device).wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.no_grad(), torch.cuda.graph(g, stream=s):
        static_y = fwd(static_x)
    for x in xs:
        static_x.copy_(x)
        g.replay()
        torch.cuda.synchronize()
        want = fwd(x.clone())
        got = static_y if isinstance(static_y, (list, tuple)) else [static_y]
        want = want if isinstance(want, (list, tuple)) else [want]
        for a, b in zip(got, want):
            assert torch.equal(a.view(torch.int16), b.view(torch.int16))


@pytest.mark.parametrize("act,M,K,N,G,p", [
    ("per_group", 512, 1024, 768, 64, 0.05),      # packed-order fq7
    ("per_token", 300, 2048, 512, 128, 0.10),     # FP8 GEMM on e4m3 codes
])
@torch.no_grad()
def test_forward_graph_replay(act, M, K, N, G, p):
    dev = _dev()
    q = _layer(dev, K, N, act, G, p, seed=3)
    xs = _inputs(dev, M, K, 11, 3)
    static_x = xs[0].clone()
    _check_graph(lambda x: q(x), static_x, xs)


@torch.no_grad()
def test_activation_order_graph_replay():
    """The config-2 path (sorted per_group activations from 16384 rows: C4 quantizer +
    permutation + fqt7) captured and replayed."""
    dev = _dev()
    from smoothquant import ops
    q = _layer(dev, 1024, 1024, "per_group", 128, 0.10, seed=5)
    xs = _inputs(dev, 16384, 1024, 13, 2)
    assert ops.fqt_eligible(q.packed(), "per_group", 4, 128, 16384)
    static_x = xs[0].clone()
    _check_graph(lambda x: q(x), static_x, xs)


@torch.no_grad()
def test_sibling_group_graph_replay():
    """A linked q/k/v group: one statistics pass, one quantizer pass and one grouped GEMM per
    replay; every member's output bit-identical to the eager group's."""
    dev = _dev()
    from smoothquant.fake_quant import link_siblings
    K = 1024
    imp_gen = torch.Generator().manual_seed(9)
    imp = torch.rand(K, generator=imp_gen) + 0.1
    from smoothquant.fake_quant import W4A4Linear
    layers = []
    for i, N in enumerate((1024, 512, 512)):
        gen = torch.Generator(device=dev).manual_seed(20 + i)
        lin = torch.nn.Linear(K, N, bias=False).to(dev, torch.float16)
        lin.weight.copy_((torch.randn(N, K, generator=gen, device=dev) * 0.02).half())
        layers.append(W4A4Linear.from_float(lin, weight_quant="per_group", act_quant="per_group",
                                            importance=imp, salient_prop=0.05, group_size=64))
    link_siblings(*layers)
    xs = _inputs(dev, 512, K, 17, 3)
    static_x = xs[0].clone()
    _check_graph(lambda x: [m(x) for m in layers], static_x, xs)
