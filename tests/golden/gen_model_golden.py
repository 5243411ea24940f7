"""Tiny-model golden fixtures from the REFERENCE (golden family 3).

Builds seeded random-init OPT and Llama models (transformers, CPU, fp32, eager
attention), computes calibration statistics with the reference's formulas
(run_experiments.py:55-84 mean|x| features; calibration.py:13-51 channel absmax),
quantizes with the reference's own `quantize_opt` / `quantize_llama_like` (and
`smooth_lm`), and stores: the calibration statistics the quantizers consumed, the input
tokens, the quantized model's logits and the Evaluator perplexity
(run_experiments.py:86-123) over two windows.  The tests rebuild the same models from
the same seeds and run them through this repo's GPU operator.

Loaded from /root/reference by file path (no bytecode written, nothing copied); argsort
pinned stable as in gen_golden.py.  Output: tests/golden/model_golden.npz (arrays + a
JSON metadata string; no pickles).

Usage:  python tests/golden/gen_model_golden.py     (needs /root/reference)
"""
from __future__ import annotations

import copy
import importlib.util
import json
import os
import sys

import numpy as np
import torch
import torch.nn as nn

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from gen_golden import _StableTorch, load_reference  # noqa: E402

REF_SMOOTH = "/root/reference/smoothquant/smooth.py"
OUT = os.path.join(HERE, "model_golden.npz")

VOCAB, SEQ, CAL_BLOCKS, EVAL_WINDOW = 512, 48, 2, 64


def tiny_opt(seed):
    from transformers import OPTConfig, OPTForCausalLM
    cfg = OPTConfig(vocab_size=VOCAB, hidden_size=64, num_hidden_layers=2, ffn_dim=256,
                    num_attention_heads=4, max_position_embeddings=256, word_embed_proj_dim=64,
                    do_layer_norm_before=True, dropout=0.0, attention_dropout=0.0,
                    activation_dropout=0.0, attn_implementation="eager")
    torch.manual_seed(seed)
    return OPTForCausalLM(cfg).eval()


def tiny_llama(seed):
    from transformers import LlamaConfig, LlamaForCausalLM
    cfg = LlamaConfig(vocab_size=VOCAB, hidden_size=64, intermediate_size=192,
                      num_hidden_layers=2, num_attention_heads=4, num_key_value_heads=4,
                      max_position_embeddings=256, attn_implementation="eager")
    torch.manual_seed(seed)
    return LlamaForCausalLM(cfg).eval()


MODELS = {"opt": tiny_opt, "llama": tiny_llama}


def tokens(seed, n):
    g = torch.Generator().manual_seed(seed)
    return torch.randint(0, VOCAB, (1, n), generator=g)


@torch.no_grad()
def calib_feat(model, blocks):
    """run_experiments.py:55-84: per-Linear list of mean_m |x| (one per block)."""
    feat = {}

    def hook(m, x, y, name):
        x = x[0] if isinstance(x, tuple) else x
        feat.setdefault(name, []).append(x.view(-1, x.shape[-1]).abs().mean(dim=0).cpu().detach())

    hs = [m.register_forward_hook(lambda m, x, y, n=n: hook(m, x, y, n))
          for n, m in model.named_modules() if isinstance(m, nn.Linear)]
    for b in blocks:
        model(b)
    for h in hs:
        h.remove()
    return feat


@torch.no_grad()
def act_scales(model, blocks):
    """calibration.py:13-51: per-Linear per-channel absmax (fp32)."""
    sc = {}

    def hook(m, x, y, name):
        x = x[0] if isinstance(x, tuple) else x
        cm = x.view(-1, x.shape[-1]).abs().detach().max(dim=0)[0].float().cpu()
        sc[name] = torch.max(sc[name], cm) if name in sc else cm

    hs = [m.register_forward_hook(lambda m, x, y, n=n: hook(m, x, y, n))
          for n, m in model.named_modules() if isinstance(m, nn.Linear)]
    for b in blocks:
        model(b)
    for h in hs:
        h.remove()
    return sc


@torch.no_grad()
def evaluator_ppl(model, ids, B):
    """run_experiments.py:86-123 with n_samples = all full windows."""
    n = ids.size(1) // B
    nlls = []
    for i in range(n):
        batch = ids[:, i * B:(i + 1) * B]
        logits = model(batch).logits
        sl = logits[:, :-1, :].contiguous().float()
        lab = batch[:, 1:]
        loss = nn.CrossEntropyLoss()(sl.view(-1, sl.size(-1)), lab.reshape(-1))
        nlls.append(loss.float() * B)
    return float(torch.exp(torch.stack(nlls).sum() / (n * B)))


CASES = [
    # key, model, quantizer, kwargs, smooth alpha (None = no smoothing)
    ("opt_defaults", "opt", "quantize_opt",
     dict(weight_quant="per_tensor", act_quant="per_tensor", quantize_bmm_input=True,
          salient_prop=0.1, quant_bits=4, group_size=32), None),
    ("opt_group", "opt", "quantize_opt",
     dict(weight_quant="per_group", act_quant="per_group", quantize_bmm_input=True,
          salient_prop=0.05, quant_bits=4, group_size=32), None),
    ("llama_group", "llama", "quantize_llama_like",
     dict(weight_quant="per_group", act_quant="per_group", salient_prop=0.05, quant_bits=4,
          group_size=32), None),
    ("llama_smooth_token", "llama", "quantize_llama_like",
     dict(weight_quant="per_channel", act_quant="per_token", salient_prop=0.0, quant_bits=4,
          group_size=128), 0.5),
]


def main():
    ref = load_reference()
    sys.dont_write_bytecode = True
    spec = importlib.util.spec_from_file_location("_ref_smooth", REF_SMOOTH)
    smooth = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(smooth)
    arrays, meta = {}, []
    for i, (key, mname, qname, kw, alpha) in enumerate(CASES):
        seed = 100 + i
        model = MODELS[mname](seed)
        cal = [tokens(1000 + seed * 10 + b, 32) for b in range(CAL_BLOCKS)]
        x = tokens(2000 + seed, SEQ)
        ev = tokens(3000 + seed, 2 * EVAL_WINDOW)
        m = copy.deepcopy(model)
        if alpha is not None:
            sc = act_scales(m, cal)
            for n, v in sc.items():
                arrays[f"{key}__scale__{n}"] = v.numpy()
            smooth.smooth_lm(m, sc, alpha)
        feat = calib_feat(m, cal) if kw.get("salient_prop", 0) > 0 or qname == "quantize_opt" else None
        if feat is not None:
            for n, lst in feat.items():
                arrays[f"{key}__feat__{n}"] = torch.stack(lst).numpy()
        q = getattr(ref, qname)(m, input_feat=feat, **kw)
        with torch.no_grad():
            logits = q(x).logits.float()
        arrays[f"{key}__x"] = x.numpy()
        arrays[f"{key}__ev"] = ev.numpy()
        arrays[f"{key}__logits"] = logits.numpy()
        ppl = evaluator_ppl(q, ev, EVAL_WINDOW)
        meta.append(dict(key=key, model=mname, seed=seed, quantizer=qname, kwargs=kw, alpha=alpha,
                         cal_seeds=[1000 + seed * 10 + b for b in range(CAL_BLOCKS)],
                         cal_len=32, ppl=ppl, eval_window=EVAL_WINDOW))
        print(key, "ppl", ppl, "logits", tuple(logits.shape))
    info = dict(source="adithyab100/smoothquant-mixedprecision (reference fake_quant.py + smooth.py, "
                       "CPU fp32, argsort pinned stable)",
                torch=torch.__version__, vocab=VOCAB, seq=SEQ, cases=meta)
    arrays["meta_json"] = np.frombuffer(json.dumps(info).encode(), dtype=np.uint8)
    np.savez_compressed(OUT, **arrays)
    print("wrote", OUT)


if __name__ == "__main__":
    main()
