"""Falcon golden mismatch diagnosis: per W4A4Linear, the GPU W_hat vs the PyTorch-CPU
restatement's W_hat on the same smoothed weight (count of differing elements, samples)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "smoothquant-mixedprecision_amd"), os.path.join(ROOT, "tests")]
import torch  # noqa: E402

from model_cases import FALCON_GOLDEN, ModelGolden, build_falcon  # noqa: E402
from oracle import torch_cpu as T  # noqa: E402
from smoothquant.fake_quant import W4A4Linear, quantize_falcon  # noqa: E402
from smoothquant.smooth import smooth_lm  # noqa: E402

FG = ModelGolden(FALCON_GOLDEN)
for case in FG.cases()[:3]:
    key = case["key"]
    kw = dict(weight_quant="per_channel", act_quant="per_token", salient_prop=0, quant_bits=4,
              group_size=128)
    kw.update(case["kwargs"])
    model = build_falcon(case, FG.meta["archs"])
    if case["alpha"] is not None:
        smooth_lm(model, FG.scales(key), case["alpha"])
    w0 = {n: m.weight.detach().clone() for n, m in model.named_modules()
          if isinstance(m, torch.nn.Linear) and n.startswith("transformer")}
    q = quantize_falcon(model.to("cuda"), input_feat=FG.feat(key), **case["kwargs"])
    for n, m in q.named_modules():
        if not isinstance(m, W4A4Linear):
            continue
        sal = None if m.salient_indices is None else m.salient_indices.cpu()
        ref = T.quantize_weight(w0[n].clone(), kw["weight_quant"], kw["quant_bits"],
                                kw["group_size"], sal)
        got = m.weight.detach().float().cpu()
        d = (got != ref)
        same_in = torch.equal(w0[n], w0[n])
        print(key, n, tuple(got.shape), got.dtype, "ndiff", int(d.sum()), flush=True)
        if d.any():
            idx = d.nonzero()[:4]
            for r, c in idx.tolist():
                print("   ", r, c, "w", float(w0[n][r, c]), "got", float(got[r, c]), "ref",
                      float(ref[r, c]), "rowmax", float(w0[n][r].abs().max()))
