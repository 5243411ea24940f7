"""BASELINE configs 1, 3 and 4 at their real layer dimensions (random-init weights; no
checkpoint can be fetched): the seeded models, calibration/eval tokens and quantizer
settings shared by the golden generator (tests/golden/gen_config_golden.py, run in the
survey container against the reference) and the GPU tests (tests/test_gpu_configs.py).

  opt125m      config 1: OPT-125M (768 / 3072, 12 layers, vocab 50272), fp32 (the
               reference's OPT dtype, run_experiments.py:152-154), quantize_opt DEFAULTS
               (weight per_tensor, act per_tensor, bmm-input quant on; fake_quant.py:377-386)
               with G=128, 10 % salient
  opt1.3b_l    config 3: one OPT-1.3B decoder layer (2048 / 8192, 32 heads), G=128, 5 %
               salient, per_group / per_group + bmm-input quant, seq 2048, fp32 and fp16
  llama7b_l    config 4: one Llama-2-7B decoder layer (4096 / 11008, 32 heads), G=64, 5 %
               salient, per_group / per_group (max-sorted), seq 2048, fp16

Model weights come from transformers' own init under torch.manual_seed (CPU RNG; the
tiny-model goldens rely on the same reproducibility), token ids from torch.Generator.
"""
from __future__ import annotations

import json
import os

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
GOLDEN = os.path.join(HERE, "golden", "config_golden.npz")

CASES = [
    dict(key="opt125m", config=1, arch="opt", dims=dict(vocab=50272, hidden=768, ffn=3072,
                                                        layers=12, heads=12),
         dtype="fp32", seed=501, quantizer="quantize_opt",
         kwargs=dict(weight_quant="per_tensor", act_quant="per_tensor", quantize_bmm_input=True,
                     salient_prop=0.1, quant_bits=4, group_size=128),
         cal_blocks=2, cal_len=128, eval_len=256),
    dict(key="opt1.3b_l_fp32", config=3, arch="opt", dims=dict(vocab=512, hidden=2048, ffn=8192,
                                                               layers=1, heads=32),
         dtype="fp32", seed=503, quantizer="quantize_opt",
         kwargs=dict(weight_quant="per_group", act_quant="per_group", quantize_bmm_input=True,
                     salient_prop=0.05, quant_bits=4, group_size=128),
         cal_blocks=2, cal_len=256, eval_len=2048),
    dict(key="opt1.3b_l_fp16", config=3, arch="opt", dims=dict(vocab=512, hidden=2048, ffn=8192,
                                                               layers=1, heads=32),
         dtype="fp16", seed=504, quantizer="quantize_opt",
         kwargs=dict(weight_quant="per_group", act_quant="per_group", quantize_bmm_input=True,
                     salient_prop=0.05, quant_bits=4, group_size=128),
         cal_blocks=2, cal_len=256, eval_len=2048),
    dict(key="llama7b_l", config=4, arch="llama", dims=dict(vocab=512, hidden=4096, ffn=11008,
                                                            layers=1, heads=32),
         dtype="fp16", seed=505, quantizer="quantize_llama_like",
         kwargs=dict(weight_quant="per_group", act_quant="per_group", salient_prop=0.05,
                     quant_bits=4, group_size=64),
         cal_blocks=2, cal_len=256, eval_len=2048),
    # ---- round 3: config 5 at Llama-2-7B layer shapes (4096 -> 4096 / 11008, 11008 ->
    # 4096) and the ppl_eval.py flow in bf16.  post: how a user of the reference composes
    # the variant after quantize_llama_like: "w4a8" rebinds every layer's
    # act_quant to partial(quantize_activation_per_group_absmax_sort, n_bits=8, G);
    # "unsorted" replaces W_hat by the unsorted per-group quantizer (fake_quant.py:29-53,
    # salient columns restored as :347/:363-365) and rebinds act_quant to :77-101.  This
    # repo expresses "unsorted" with weight_quant / act_quant "per_group_unsorted"
    # (test_kwargs) and "w4a8" with the same rebinding.
    dict(key="llama7b_l_w4a8_g128", config=5, arch="llama",
         dims=dict(vocab=512, hidden=4096, ffn=11008, layers=1, heads=32),
         dtype="fp16", seed=506, quantizer="quantize_llama_like",
         kwargs=dict(weight_quant="per_group", act_quant="per_group", salient_prop=0.05,
                     quant_bits=4, group_size=128),
         post="w4a8", cal_blocks=2, cal_len=256, eval_len=2048),
    dict(key="llama7b_l_none_g1024", config=5, arch="llama",
         dims=dict(vocab=512, hidden=4096, ffn=11008, layers=1, heads=32),
         dtype="fp16", seed=507, quantizer="quantize_llama_like",
         kwargs=dict(weight_quant="per_group", act_quant="per_group", salient_prop=0.05,
                     quant_bits=4, group_size=1024),
         test_kwargs=dict(weight_quant="per_group_unsorted", act_quant="per_group_unsorted"),
         post="unsorted", cal_blocks=2, cal_len=256, eval_len=2048),
    # smoothquant/ppl_eval.py:69-83: bf16 model, smooth_lm(act_scales, alpha=0.5), then
    # quantize_model(weight per_channel, act per_token, quantize_bmm_input=True) with no
    # input_feat (no salient channels); act scales = per-channel max|x| over the
    # calibration blocks (calibration.py:13-51's statistic), stored in the fixture
    dict(key="llama7b_l_bf16_pplflow", config=4, arch="llama",
         dims=dict(vocab=512, hidden=4096, ffn=11008, layers=1, heads=32),
         dtype="bf16", seed=508, quantizer="quantize_model",
         kwargs=dict(weight_quant="per_channel", act_quant="per_token", quantize_bmm_input=True),
         smooth=0.5, input_feat=False, cal_blocks=2, cal_len=256, eval_len=2048),
]
TDT = {"fp32": torch.float32, "fp16": torch.float16, "bf16": torch.bfloat16}
# logits positions stored per case (first, middle, last few)
N_POS = 8
VOCAB_SLICE = 2048


def build(case):
    """The seeded random-init model of `case` (CPU, eval, eager attention, case dtype)."""
    d = case["dims"]
    torch.manual_seed(case["seed"])
    if case["arch"] == "opt":
        from transformers import OPTConfig, OPTForCausalLM
        cfg = OPTConfig(vocab_size=d["vocab"], hidden_size=d["hidden"], ffn_dim=d["ffn"],
                        num_hidden_layers=d["layers"], num_attention_heads=d["heads"],
                        max_position_embeddings=2048, word_embed_proj_dim=d["hidden"],
                        do_layer_norm_before=True, dropout=0.0, attention_dropout=0.0,
                        activation_dropout=0.0, attn_implementation="eager")
        model = OPTForCausalLM(cfg)
    else:
        from transformers import LlamaConfig, LlamaForCausalLM
        cfg = LlamaConfig(vocab_size=d["vocab"], hidden_size=d["hidden"],
                          intermediate_size=d["ffn"], num_hidden_layers=d["layers"],
                          num_attention_heads=d["heads"], num_key_value_heads=d["heads"],
                          max_position_embeddings=4096, attn_implementation="eager")
        model = LlamaForCausalLM(cfg)
    return model.to(TDT[case["dtype"]]).eval()


def tokens(case, what):
    """Calibration blocks (list of [1, cal_len]) or the eval sequence [1, eval_len]."""
    vocab = case["dims"]["vocab"]
    if what == "cal":
        out = []
        for b in range(case["cal_blocks"]):
            g = torch.Generator().manual_seed(case["seed"] * 100 + b)
            out.append(torch.randint(0, vocab, (1, case["cal_len"]), generator=g))
        return out
    g = torch.Generator().manual_seed(case["seed"] * 100 + 99)
    return torch.randint(0, vocab, (1, case["eval_len"]), generator=g)


def positions(case):
    L = case["eval_len"]
    return np.array(sorted({0, 1, L // 2, L // 2 + 1, L - 4, L - 3, L - 2, L - 1}), np.int64)


def what_digest(w: torch.Tensor) -> str:
    """sha256 of W_hat's bytes in its dtype, -0.0 folded to +0.0 (the packed path stores
    integer codes, whose zero dequantizes to +0.0); bf16 as its 16-bit patterns."""
    import hashlib
    a = (w.detach().cpu().contiguous() + 0.0)
    if a.dtype == torch.bfloat16:
        a = a.view(torch.int16)
    return hashlib.sha256(a.numpy().tobytes()).hexdigest()


def post_quantize(model, case, fq, w_orig=None):
    """Apply the case's `post` composition to every W4A4Linear of `model`, using the
    quantizer functions of module `fq` (the reference's fake_quant in the generator, this
    repo's in the tests).  "unsorted" needs the pre-quantization weights (w_orig: {name:
    W}) -- only the generator uses it; the tests quantize with test_kwargs instead."""
    from functools import partial
    post = case.get("post")
    if not post:
        return
    G = case["kwargs"]["group_size"]
    for n, m in model.named_modules():
        if type(m).__name__ != "W4A4Linear":
            continue
        if post == "w4a8":
            m.act_quant = partial(fq.quantize_activation_per_group_absmax_sort, n_bits=8,
                                  group_size=G)
        elif post == "unsorted" and w_orig is not None:
            w = w_orig[n].clone()
            sal = m.salient_indices
            keep = w[:, sal].clone() if sal is not None else None
            w_hat = fq.quantize_weight_per_group_absmax(w, n_bits=4, group_size=G)
            if sal is not None:
                w_hat[:, sal] = keep
            m.weight = w_hat
            m.act_quant = partial(fq.quantize_activation_per_group_absmax, n_bits=4,
                                  group_size=G)


class ConfigGolden:
    def __init__(self, path=GOLDEN):
        self.z = np.load(path, allow_pickle=False)
        self.meta = json.loads(bytes(self.z["meta_json"]).decode())

    def case_meta(self, key):
        return self.meta["cases"][key]

    def act_scales(self, key):
        pre = f"{key}__act__"
        return {k[len(pre):]: torch.from_numpy(self.z[k].copy())
                for k in self.z.files if k.startswith(pre)}

    def importance(self, key):
        pre = f"{key}__imp__"
        return {k[len(pre):]: torch.from_numpy(self.z[k].copy())
                for k in self.z.files if k.startswith(pre)}

    def arr(self, key, name):
        return self.z[f"{key}__{name}"]
