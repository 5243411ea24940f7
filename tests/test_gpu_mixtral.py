"""quantize_mixtral (/root/reference/smoothquant/fake_quant.py:564-668) on a tiny random
Mixtral in the installed transformers' layout (5.x: the attention projections are nn.Linear;
the router is a MixtralTopKRouter and the experts are fused 3-D parameters, so there is no
nn.Linear to swap there).  The reference's quantize_mixtral cannot run on this transformers
(it imports MixtralBLockSparseTop2MLP, which 5.x no longer defines), so parity is pinned against
the oracle layer instead (oracle/torch_cpu.py, itself pinned to the reference's layer goldens):
every swapped layer's W_hat and salient set equal the oracle's bit for bit, q/k/v run as one
sibling group, and the logits equal those of the same model with the oracle layers swapped in
(CPU, fp32) within the model-test tolerance."""
import copy
import hashlib

import pytest
import torch
from torch import nn

pytestmark = pytest.mark.gpu
PROJ = ("q_proj", "k_proj", "v_proj", "o_proj")


def _model(seed):
    from transformers import MixtralConfig, MixtralForCausalLM
    cfg = MixtralConfig(vocab_size=512, hidden_size=64, intermediate_size=96, num_hidden_layers=2,
                        num_attention_heads=4, num_key_value_heads=2, num_local_experts=4,
                        num_experts_per_tok=2, max_position_embeddings=256,
                        attn_implementation="eager")
    torch.manual_seed(seed)
    return MixtralForCausalLM(cfg).eval()


def _tokens(seed, n):
    g = torch.Generator().manual_seed(seed)
    return torch.randint(0, 512, (1, n), generator=g)


@torch.no_grad()
def _feat(model, blocks):
    feat = {}
    hs = [m.register_forward_hook(
        lambda m, x, y, n=n: feat.setdefault("model." + n, []).append(
            x[0].reshape(-1, x[0].shape[-1]).abs().mean(0).cpu()))
        for n, m in model.model.named_modules() if isinstance(m, nn.Linear)]
    for b in blocks:
        model(b)
    for h in hs:
        h.remove()
    return feat


class _OracleLinear(nn.Module):
    def __init__(self, layer):
        super().__init__()
        self.layer = layer

    def forward(self, x):
        return self.layer(x)


@pytest.mark.parametrize("case", [
    dict(weight_quant="per_group", act_quant="per_group", salient_prop=0.1, group_size=32,
         quantize_bmm_input=False),
    dict(weight_quant="per_channel", act_quant="per_token", salient_prop=0.05, group_size=128,
         quantize_bmm_input=False),
    dict(weight_quant="per_group", act_quant="per_group", salient_prop=0, group_size=16,
         quantize_bmm_input=True),
], ids=["group_salient", "channel_token", "group_bmm"])
def test_quantize_mixtral_matches_oracle(case):
    if not torch.cuda.is_available():
        pytest.skip("no ROCm device")
    from oracle import torch_cpu as T
    from smoothquant.fake_quant import W4A4Linear, quantize_mixtral
    base = _model(11)
    feat = _feat(base, [_tokens(100 + b, 32) for b in range(2)])
    x = _tokens(7, 40)
    # the oracle model: the same modules swapped for the CPU restatement of the reference layer
    ref = copy.deepcopy(base)
    w_ref = {}
    for name, m in ref.model.named_modules():
        if type(m).__name__ == "MixtralAttention":
            for p in PROJ:
                lin = getattr(m, p)
                imp = sum(feat["model." + name + "." + p]).float()
                layer = T.CPUFakeQuantLinear(
                    lin.weight.detach().clone(), None if lin.bias is None else lin.bias.detach(),
                    case["weight_quant"], case["act_quant"], 4, case["group_size"], imp,
                    case["salient_prop"], quantize_output=case["quantize_bmm_input"] and p != "o_proj")
                w_ref[name + "." + p] = (layer.w_hat, layer.salient)
                setattr(m, p, _OracleLinear(layer))
    with torch.no_grad():
        logits_ref = ref(x).logits.float()
    q = quantize_mixtral(copy.deepcopy(base).to("cuda"), input_feat=feat, quant_bits=4, **case)
    n_swapped = 0
    for name, m in q.model.named_modules():
        if type(m).__name__ == "MixtralAttention":
            for p in PROJ:
                layer = getattr(m, p)
                assert isinstance(layer, W4A4Linear)
                w_hat, sal = w_ref[name + "." + p]
                got = (layer.weight.detach().float().cpu() + 0.0).numpy().tobytes()
                want = (w_hat.float() + 0.0).numpy().tobytes()
                assert hashlib.sha256(got).digest() == hashlib.sha256(want).digest(), name + p
                if sal is None:
                    assert layer.salient_indices is None
                else:
                    assert torch.equal(layer.salient_indices.cpu().long(), sal.long())
                n_swapped += 1
            grp = m.q_proj.__dict__.get("_sqmp_group")
            assert grp is not None and m.k_proj.__dict__.get("_sqmp_group") is grp
    assert n_swapped == 8
    with torch.no_grad():
        logits = q(x.to("cuda")).logits.float().cpu()
    rel = float((logits - logits_ref).norm() / logits_ref.norm())
    assert rel < 2e-2, rel
