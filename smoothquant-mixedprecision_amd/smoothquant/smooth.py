"""SmoothQuant folding (the reference's smoothquant/smooth.py:18-160).

s_j = max|X_j|^alpha / max_i|W_ij|^(1-alpha) per input channel j (clamped at 1e-5, cast to
the weight dtype); the norm's weight (and bias) are divided by s and every following
Linear's columns multiplied by s.  Offline, zero runtime cost: the packed W4A4 weights
are produced from the already-smoothed Linear weights.
"""
import torch
import torch.nn as nn


def _smoothing_scales(fcs, act_scales, alpha):
    device, dtype = fcs[0].weight.device, fcs[0].weight.dtype
    act_scales = act_scales.to(device=device, dtype=dtype)
    w_scales = torch.stack([fc.weight.abs().max(dim=0)[0] for fc in fcs]).max(dim=0)[0]
    w_scales = w_scales.clamp(min=1e-5)
    return (act_scales.pow(alpha) / w_scales.pow(1 - alpha)).clamp(min=1e-5).to(device).to(dtype)


def _check(ln, fcs, act_scales):
    for fc in fcs:
        # nn.Linear as in the reference; also a transformers-5 MoE router (MixtralTopKRouter:
        # a [E, H] weight applied by F.linear) and the fused experts' rows (_FusedRows)
        assert isinstance(fc, nn.Linear) or fc.weight.dim() == 2
        assert ln.weight.numel() == fc.weight.shape[-1] == act_scales.numel()


class _FusedRows:
    """The w1 / w3 rows of every expert of a transformers-5 fused MixtralExperts
    (gate_up_proj [E, 2I, H]) as one [E * 2I, H] weight view: their column maxima and the
    in-place column scaling are exactly those of the reference's per-expert w1 / w3 Linears
    (smooth.py:142-156)."""

    def __init__(self, gate_up_proj):
        self.weight = gate_up_proj.data.view(-1, gate_up_proj.shape[-1])


@torch.no_grad()
def smooth_ln_fcs(ln, fcs, act_scales, alpha=0.5):
    """smooth.py:18-45 (LayerNorm with bias)."""
    fcs = fcs if isinstance(fcs, list) else [fcs]
    assert isinstance(ln, nn.LayerNorm)
    _check(ln, fcs, act_scales)
    s = _smoothing_scales(fcs, act_scales, alpha)
    ln.weight.div_(s)
    ln.bias.div_(s)
    for fc in fcs:
        fc.weight.mul_(s.view(1, -1))


@torch.no_grad()
def smooth_ln_fcs_llama_like(ln, fcs, act_scales, alpha=0.5):
    """smooth.py:48-71 (RMSNorm, no bias)."""
    from transformers.models.llama.modeling_llama import LlamaRMSNorm
    from transformers.models.mistral.modeling_mistral import MistralRMSNorm
    from transformers.models.mixtral.modeling_mixtral import MixtralRMSNorm
    fcs = fcs if isinstance(fcs, list) else [fcs]
    assert isinstance(ln, (LlamaRMSNorm, MistralRMSNorm, MixtralRMSNorm))
    _check(ln, fcs, act_scales)
    s = _smoothing_scales(fcs, act_scales, alpha)
    ln.weight.div_(s)
    for fc in fcs:
        fc.weight.mul_(s.view(1, -1))


@torch.no_grad()
def smooth_lm(model, scales, alpha=0.5):
    """smooth.py:74-160: fold per-channel smoothing into every decoder block's norms."""
    from transformers.models.bloom.modeling_bloom import BloomBlock
    from transformers.models.falcon.modeling_falcon import FalconDecoderLayer
    from transformers.models.llama.modeling_llama import LlamaDecoderLayer
    from transformers.models.mistral.modeling_mistral import MistralDecoderLayer
    from transformers.models.mixtral.modeling_mixtral import MixtralDecoderLayer
    from transformers.models.opt.modeling_opt import OPTDecoderLayer
    for name, module in model.named_modules():
        if isinstance(module, OPTDecoderLayer):
            attn = module.self_attn
            smooth_ln_fcs(module.self_attn_layer_norm, [attn.q_proj, attn.k_proj, attn.v_proj],
                          scales[name + ".self_attn.q_proj"], alpha)
            smooth_ln_fcs(module.final_layer_norm, module.fc1, scales[name + ".fc1"], alpha)
        elif isinstance(module, BloomBlock):
            smooth_ln_fcs(module.input_layernorm, module.self_attention.query_key_value,
                          scales[name + ".self_attention.query_key_value"], alpha)
            smooth_ln_fcs(module.post_attention_layernorm, module.mlp.dense_h_to_4h,
                          scales[name + ".mlp.dense_h_to_4h"], alpha)
        elif isinstance(module, FalconDecoderLayer):
            qkv = module.self_attention.query_key_value
            fc1 = module.mlp.dense_h_to_4h
            qkv_s = scales[name + ".self_attention.query_key_value"]
            fc1_s = scales[name + ".mlp.dense_h_to_4h"]
            cfg = module.config
            if not cfg.new_decoder_architecture and cfg.parallel_attn:
                smooth_ln_fcs(module.input_layernorm, [qkv, fc1], qkv_s, alpha)
            else:
                attn_ln = module.ln_attn if cfg.new_decoder_architecture else module.input_layernorm
                ffn_ln = module.ln_mlp if cfg.new_decoder_architecture else module.post_attention_layernorm
                smooth_ln_fcs(attn_ln, qkv, qkv_s, alpha)
                smooth_ln_fcs(ffn_ln, fc1, fc1_s, alpha)
        elif isinstance(module, (LlamaDecoderLayer, MistralDecoderLayer)):
            attn = module.self_attn
            smooth_ln_fcs_llama_like(module.input_layernorm, [attn.q_proj, attn.k_proj, attn.v_proj],
                                     scales[name + ".self_attn.q_proj"], alpha)
            smooth_ln_fcs_llama_like(module.post_attention_layernorm,
                                     [module.mlp.gate_proj, module.mlp.up_proj],
                                     scales[name + ".mlp.gate_proj"], alpha)
        elif isinstance(module, MixtralDecoderLayer):
            attn = module.self_attn
            smooth_ln_fcs_llama_like(module.input_layernorm, [attn.q_proj, attn.k_proj, attn.v_proj],
                                     scales[name + ".self_attn.q_proj"], alpha)
            # transformers 4.x: block_sparse_moe.gate (nn.Linear) + experts with w1 / w3
            # Linears (the reference's layout); 5.x: mlp.gate (MixtralTopKRouter) + fused experts
            moe = getattr(module, "block_sparse_moe", None)
            key = name + ".block_sparse_moe.gate"
            if moe is None:
                moe, key = module.mlp, name + ".mlp.gate"
            fcs = [moe.gate]
            experts = getattr(moe, "experts", [])
            if isinstance(experts, nn.ModuleList):
                for expert in experts:
                    fcs += [expert.w1, expert.w3]
            elif hasattr(experts, "gate_up_proj"):
                fcs.append(_FusedRows(experts.gate_up_proj))
            smooth_ln_fcs_llama_like(module.post_attention_layernorm, fcs, scales[key], alpha)
