"""CPU side of the Falcon goldens (tests/golden/falcon_golden.npz, from the reference's
quantize_falcon + smooth_lm; gen_falcon_golden.py): this repo's smooth_lm (plain torch)
followed by the PyTorch-CPU restatement of W4A4Linear.from_float (oracle/torch_cpu.py)
reproduces every reference W_hat and salient set bit-exactly, and the features sit under the
"model." + name keys quantize_falcon looks up (fake_quant.py:671-731 walks
model.named_modules())."""
import hashlib

import pytest
import torch

from model_cases import FALCON_GOLDEN, ModelGolden, build_falcon
from oracle import torch_cpu as T

FG = ModelGolden(FALCON_GOLDEN)
PROJ = ("self_attention.query_key_value", "self_attention.dense", "mlp.dense_h_to_4h",
        "mlp.dense_4h_to_h")


@pytest.mark.parametrize("case", FG.cases(), ids=[c["key"] for c in FG.cases()])
def test_falcon_what_matches_reference(case):
    from smoothquant.smooth import smooth_lm
    key = case["key"]
    kw = dict(weight_quant="per_channel", act_quant="per_token", salient_prop=0, quant_bits=4,
              group_size=128)
    kw.update(case["kwargs"])
    model = build_falcon(case, FG.meta["archs"])
    if case["alpha"] is not None:
        smooth_lm(model, FG.scales(key), case["alpha"])
        # within 1e-6 of the reference's smoothed tensors (bit-exact on the AVX2 host that made
        # the goldens; smooth_lm's fp32 pow rounds per host ISA), then exactly those
        sd = model.state_dict()
        ref_sm = FG.smoothed(key)
        assert ref_sm
        with torch.no_grad():
            for n, t in ref_sm.items():
                torch.testing.assert_close(sd[n], t, rtol=1e-6, atol=0)
                sd[n].copy_(t)
    feat = FG.feat(key)
    mods = dict(model.named_modules())
    n_checked = 0
    for layer in range(2):
        for proj in PROJ:
            name = f"transformer.h.{layer}.{proj}"
            imp = None
            if feat is not None:
                imp = sum(feat["model." + name]).float()   # the key quantize_falcon uses
            sal = T.select_salient(imp, kw["salient_prop"])
            with torch.no_grad():
                w_hat = T.quantize_weight(mods[name].weight.detach().clone(), kw["weight_quant"],
                                          kw["quant_bits"], kw["group_size"], sal)
            digest = hashlib.sha256((w_hat.float().contiguous() + 0.0).numpy().tobytes()).hexdigest()
            assert digest == case["w_hat"][name], name
            want_sal = case["w_hat"][name + "#salient"]
            got_sal = None if sal is None else hashlib.sha256(
                sal.to(torch.int64).numpy().tobytes()).hexdigest()
            assert got_sal == want_sal, name
            n_checked += 1
    assert n_checked == len([k for k in case["w_hat"] if "#" not in k]) == 8
