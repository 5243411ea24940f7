"""Model-level parity on the GPU: seeded tiny OPT / Llama models quantized by THIS repo
(quantize_opt / quantize_llama_like, smooth_lm) against the reference-generated logits
and Evaluator perplexity (tests/golden/gen_model_golden.py; reference run on CPU fp32).

Every W4A4 layer's operands are bit-exact with the reference's given the same input
(test_gpu_parity.py); across a model the non-quantized ops (attention, norms, softmax)
run on the GPU here vs the CPU there, so hidden states differ by fp32 rounding and an
activation code can flip at a rounding boundary in a later layer.  Tolerances:
logits relative Frobenius error <= 2e-2, perplexity relative error <= 1e-2.
"""
import copy

import numpy as np
import pytest
import torch

from model_cases import ModelGolden, build_model

pytestmark = pytest.mark.gpu
MG = ModelGolden()
TOL_LOGITS, TOL_PPL = 2e-2, 1e-2


@pytest.mark.parametrize("case", MG.cases(), ids=[c["key"] for c in MG.cases()])
def test_tiny_model_matches_reference(case):
    if not torch.cuda.is_available():
        pytest.skip("no ROCm device")
    from smoothquant.fake_quant import W4A4Linear, quantize_llama_like, quantize_opt
    from smoothquant.ppl import Evaluator
    from smoothquant.smooth import smooth_lm
    key = case["key"]
    model = build_model(case)
    if case["alpha"] is not None:
        smooth_lm(model, MG.scales(key), case["alpha"])
    model = model.to("cuda")
    feat = MG.feat(key)
    fn = quantize_opt if case["quantizer"] == "quantize_opt" else quantize_llama_like
    q = fn(model, input_feat=feat, **case["kwargs"])
    n_w4 = sum(isinstance(m, W4A4Linear) for m in q.modules())
    assert n_w4 == (12 if case["model"] == "opt" else 14)
    x = torch.from_numpy(MG.arr(key, "x").copy()).cuda()
    with torch.no_grad():
        logits = q(x).logits.float().cpu().numpy()
    want = MG.arr(key, "logits")
    rel = np.linalg.norm(logits - want) / np.linalg.norm(want)
    ev = torch.from_numpy(MG.arr(key, "ev").copy())
    B = case["eval_window"]  # the golden evaluates every full window (gen_model_golden.py)
    ppl = float(Evaluator(None, None, "cuda", n_samples=ev.size(1) // B, batch_size=B,
                          input_ids=ev).evaluate(q))
    print(f"{key}: logits rel {rel:.3e}, ppl {ppl:.4f} vs {case['ppl']:.4f}")
    assert rel <= TOL_LOGITS
    assert abs(ppl - case["ppl"]) <= TOL_PPL * case["ppl"]
