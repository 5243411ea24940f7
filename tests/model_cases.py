"""Shared helpers for the tiny-model goldens (tests/golden/model_golden.npz)."""
import json
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
GOLDEN = os.path.join(HERE, "golden", "model_golden.npz")


class ModelGolden:
    def __init__(self, path=GOLDEN):
        self.z = np.load(path, allow_pickle=False)
        self.meta = json.loads(bytes(self.z["meta_json"]).decode())

    def cases(self):
        return self.meta["cases"]

    def feat(self, key):
        pre = f"{key}__feat__"
        out = {}
        for k in self.z.files:
            if k.startswith(pre):
                arr = self.z[k]
                out[k[len(pre):]] = [torch.from_numpy(a.copy()) for a in arr]
        return out or None

    def scales(self, key):
        pre = f"{key}__scale__"
        return {k[len(pre):]: torch.from_numpy(self.z[k].copy()) for k in self.z.files if k.startswith(pre)}

    def smoothed(self, key):
        """The reference's smoothed tensors (state_dict names) of a case, when stored."""
        pre = f"{key}__smoothed__"
        return {k[len(pre):]: torch.from_numpy(self.z[k].copy()) for k in self.z.files if k.startswith(pre)}

    def arr(self, key, name):
        return self.z[f"{key}__{name}"]


def build_model(case):
    """The same seeded random-init model the generator built (CPU, fp32, eager)."""
    sys.path.insert(0, os.path.join(HERE, "golden"))
    from transformers import LlamaConfig, LlamaForCausalLM, OPTConfig, OPTForCausalLM
    if case["model"] == "opt":
        cfg = OPTConfig(vocab_size=512, hidden_size=64, num_hidden_layers=2, ffn_dim=256,
                        num_attention_heads=4, max_position_embeddings=256, word_embed_proj_dim=64,
                        do_layer_norm_before=True, dropout=0.0, attention_dropout=0.0,
                        activation_dropout=0.0, attn_implementation="eager")
        torch.manual_seed(case["seed"])
        return OPTForCausalLM(cfg).eval()
    cfg = LlamaConfig(vocab_size=512, hidden_size=64, intermediate_size=192, num_hidden_layers=2,
                      num_attention_heads=4, num_key_value_heads=4, max_position_embeddings=256,
                      attn_implementation="eager")
    torch.manual_seed(case["seed"])
    return LlamaForCausalLM(cfg).eval()


def cal_blocks(case):
    out = []
    for s in case["cal_seeds"]:
        g = torch.Generator().manual_seed(s)
        out.append(torch.randint(0, 512, (1, case["cal_len"]), generator=g))
    return out


FALCON_GOLDEN = os.path.join(HERE, "golden", "falcon_golden.npz")


def build_falcon(case, archs):
    """The seeded random-init tiny Falcon of tests/golden/gen_falcon_golden.py (CPU, fp32)."""
    from transformers import FalconConfig, FalconForCausalLM
    cfg = FalconConfig(vocab_size=512, hidden_size=64, num_hidden_layers=2, num_attention_heads=4,
                       bias=False, alibi=False, attention_dropout=0.0, hidden_dropout=0.0,
                       max_position_embeddings=256, attn_implementation="eager",
                       **archs[case["arch"]])
    torch.manual_seed(case["seed"])
    return FalconForCausalLM(cfg).eval()
