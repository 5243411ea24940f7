"""Every C entry runs on its stream's device (SQMP_DEVICE_GUARD, sqmp_common.h).

The reference's only multi-GPU mechanism is accelerate's device_map="auto"
(run_experiments.py:146-148, smoothquant/ppl_eval.py:69-71, examples/ppl_eval.sh:17-18): layers
sit on several GPUs and run one after another, so a layer's tensors need not be on the current
device.  Here:
  * a forward under a torch.cuda.device context of its own index, on a side stream and on the
    default stream give the same bits (sibling group included);
  * with two or more devices, a layer on device 1 called while device 0 is current gives the
    bits it gives with device 1 current, and leaves device 0 current (skipped on one GPU).
"""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _layers(dev, seed=0, M=512, K=1024, N=768):
    from smoothquant.fake_quant import W4A4Linear, link_siblings
    gen = torch.Generator(device=dev).manual_seed(seed)
    x = torch.randn(M, K, generator=gen, device=dev).half()
    x[:, :8] *= 30.0
    imp = x.float().abs().mean(0).cpu()
    qs = []
    for _ in range(3):
        lin = torch.nn.Linear(K, N).to(dev, torch.float16)
        with torch.no_grad():
            lin.weight.copy_((torch.randn(N, K, generator=gen, device=dev) * 0.02).half())
        qs.append(W4A4Linear.from_float(lin, weight_quant="per_group", act_quant="per_group",
                                        importance=imp, salient_prop=0.05, group_size=64))
    link_siblings(*qs)
    return qs, x


def _run(qs, x):
    return [q(x) for q in qs]


@torch.no_grad()
def test_forward_under_device_context_and_side_stream():
    if not torch.cuda.is_available():
        pytest.skip("no ROCm device")
    dev = torch.device("cuda", 0)
    qs, x = _layers(dev)
    ref = [y.clone() for y in _run(qs, x)]
    with torch.cuda.device(dev):
        got = _run(qs, x.clone())
    for a, b in zip(got, ref):
        assert torch.equal(a, b)
    s = torch.cuda.Stream(dev)
    s.wait_stream(torch.cuda.current_stream(dev))
    with torch.cuda.stream(s):
        xs = x.clone()
        got = _run(qs, xs)
    s.synchronize()
    for a, b in zip(got, ref):
        assert torch.equal(a, b)


@torch.no_grad()
def test_layer_on_another_device_than_the_current():
    if not torch.cuda.is_available() or torch.cuda.device_count() < 2:
        pytest.skip("needs two ROCm devices")
    d1 = torch.device("cuda", 1)
    with torch.cuda.device(d1):
        qs, x = _layers(d1, seed=3)
        ref = [y.clone() for y in _run(qs, x)]
    torch.cuda.set_device(0)
    got = _run(qs, x.clone())
    assert torch.cuda.current_device() == 0
    torch.cuda.synchronize(d1)
    for a, b in zip(got, ref):
        assert a.device == d1 and torch.equal(a, b)
