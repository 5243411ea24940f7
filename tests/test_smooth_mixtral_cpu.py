"""smooth_lm's Mixtral branch (/root/reference/smoothquant/smooth.py:142-156) on the installed
transformers' layout (5.x: mlp.gate is a MixtralTopKRouter, the experts one fused
gate_up_proj [E, 2I, H]): the act scales are collected for the router too (calibration's
hooks), the post-attention norm is divided by s and the router and every expert's w1 / w3
rows multiplied by it, so the smoothed model computes the same function (fp32)."""
import torch

from smoothquant.calibration import LinearInputStats, _fold_channel_absmax
from smoothquant.smooth import smooth_lm


def _model():
    from transformers import MixtralConfig, MixtralForCausalLM
    cfg = MixtralConfig(vocab_size=512, hidden_size=64, intermediate_size=96, num_hidden_layers=2,
                        num_attention_heads=4, num_key_value_heads=2, num_local_experts=4,
                        num_experts_per_tok=2, max_position_embeddings=256,
                        attn_implementation="eager")
    torch.manual_seed(3)
    return MixtralForCausalLM(cfg).eval()


@torch.no_grad()
def test_smooth_lm_mixtral_is_a_reparametrization():
    m = _model()
    g = torch.Generator().manual_seed(1)
    x = torch.randint(0, 512, (1, 48), generator=g)
    with LinearInputStats(m, _fold_channel_absmax) as col:
        m(x)
    scales = col.stats
    assert "model.layers.0.mlp.gate" in scales and "model.layers.0.self_attn.q_proj" in scales
    before = m(x).logits.clone()
    ln0 = m.model.layers[0].post_attention_layernorm.weight.clone()
    gu0 = m.model.layers[0].mlp.experts.gate_up_proj.clone()
    r0 = m.model.layers[0].mlp.gate.weight.clone()
    smooth_lm(m, scales, 0.5)
    layer = m.model.layers[0]
    assert not torch.equal(layer.post_attention_layernorm.weight, ln0)
    s = ln0 / layer.post_attention_layernorm.weight          # the smoothing factors
    torch.testing.assert_close(layer.mlp.gate.weight, r0 * s.view(1, -1))
    torch.testing.assert_close(layer.mlp.experts.gate_up_proj, gu0 * s.view(1, 1, -1))
    after = m(x).logits
    assert float((after - before).norm() / before.norm()) < 1e-5
