"""Tiny-Falcon golden fixtures from the REFERENCE (quantize_falcon and smooth_lm's Falcon
branch).

Seeded random-init Falcon models (transformers, CPU, fp32, eager attention) in three
architectures -- parallel attention + multi-query (the Falcon-7B layout), the new decoder
architecture (ln_attn / ln_mlp, grouped KV heads: Falcon-40B/180B) and the sequential
layout -- smoothed with the reference's smooth_lm (/root/reference/smoothquant/smooth.py:
74-160, Falcon branch) where a case says so, then quantized with the reference's own
quantize_falcon (/root/reference/smoothquant/fake_quant.py:671-731).  Stored per case: the
statistics the reference consumed (act scales; mean|x| features under the "model." + name
keys quantize_falcon looks up), the input tokens, the logits, the Evaluator perplexity
(run_experiments.py:86-123 over two windows) and the sha256 of every W4A4Linear's W_hat
buffer and salient_indices.  The fused query_key_value with quantize_bmm_input=True and
salient channels is the reference's IndexError edge (fake_quant.py:311-314: a K-long mask
indexing the N-wide output, N != K): that case stores the exception type and message.

Loaded from /root/reference by file path (no bytecode written, nothing copied); argsort
pinned stable as in gen_golden.py.  Output: tests/golden/falcon_golden.npz.

Usage:  python tests/golden/gen_falcon_golden.py     (needs /root/reference)
"""
from __future__ import annotations

import copy
import hashlib
import importlib.util
import json
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from gen_golden import load_reference  # noqa: E402
from gen_model_golden import act_scales, calib_feat, evaluator_ppl, tokens  # noqa: E402

REF_SMOOTH = "/root/reference/smoothquant/smooth.py"
OUT = os.path.join(HERE, "falcon_golden.npz")
VOCAB, SEQ, CAL_BLOCKS, EVAL_WINDOW = 512, 48, 2, 64

ARCHS = {
    "parallel_mq": dict(new_decoder_architecture=False, parallel_attn=True, multi_query=True),
    "new_arch": dict(new_decoder_architecture=True, num_kv_heads=2),
    "sequential": dict(new_decoder_architecture=False, parallel_attn=False, multi_query=False),
}


def falcon_config(arch):
    from transformers import FalconConfig
    return FalconConfig(vocab_size=VOCAB, hidden_size=64, num_hidden_layers=2,
                        num_attention_heads=4, bias=False, alibi=False, attention_dropout=0.0,
                        hidden_dropout=0.0, max_position_embeddings=256,
                        attn_implementation="eager", **ARCHS[arch])


def tiny_falcon(arch, seed):
    from transformers import FalconForCausalLM
    torch.manual_seed(seed)
    return FalconForCausalLM(falcon_config(arch)).eval()


CASES = [
    # key, arch, quantize_falcon kwargs, smooth alpha, salient features given
    ("falcon_parallel_defaults", "parallel_mq", dict(), 0.5, False),
    ("falcon_newarch_group", "new_arch",
     dict(weight_quant="per_group", act_quant="per_group", quantize_bmm_input=False,
          salient_prop=0.1, quant_bits=4, group_size=32), 0.5, True),
    ("falcon_sequential_token", "sequential",
     dict(weight_quant="per_channel", act_quant="per_token", quantize_bmm_input=False,
          salient_prop=0.05, quant_bits=4, group_size=128), None, True),
    ("falcon_bmm_salient_raises", "sequential",
     dict(weight_quant="per_channel", act_quant="per_token", quantize_bmm_input=True,
          salient_prop=0.1, quant_bits=4, group_size=128), None, True),
]


def w_hat_digests(model):
    """sha256 of each W4A4Linear's W_hat (fp32 bytes, -0.0 folded to +0.0 as config_cases.
    what_digest: the packed path dequantizes integer code 0 to +0.0) and of its
    salient_indices (int64)."""
    out = {}
    for n, m in model.named_modules():
        if type(m).__name__ == "W4A4Linear":
            w = (m.weight.detach().float().contiguous() + 0.0).numpy()
            out[n] = hashlib.sha256(w.tobytes()).hexdigest()
            si = m.salient_indices
            out[n + "#salient"] = (None if si is None else
                                   hashlib.sha256(si.to(torch.int64).numpy().tobytes()).hexdigest())
    return out


def main():
    ref = load_reference()
    sys.dont_write_bytecode = True
    spec = importlib.util.spec_from_file_location("_ref_smooth", REF_SMOOTH)
    smooth = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(smooth)
    arrays, meta = {}, []
    for i, (key, arch, kw, alpha, with_feat) in enumerate(CASES):
        seed = 500 + i
        m = copy.deepcopy(tiny_falcon(arch, seed))
        cal = [tokens(1000 + seed * 10 + b, 32) for b in range(CAL_BLOCKS)]
        x = tokens(2000 + seed, SEQ)
        ev = tokens(3000 + seed, 2 * EVAL_WINDOW)
        if alpha is not None:
            sc = act_scales(m, cal)
            for n, v in sc.items():
                arrays[f"{key}__scale__{n}"] = v.numpy()
            before = {n: t.detach().clone() for n, t in m.state_dict().items()}
            smooth.smooth_lm(m, sc, alpha)
            # the smoothed tensors themselves: smooth_lm's fp32 pow is vectorised per CPU ISA
            # (AVX2 here, maybe AVX-512 on the GPU box's host), so the GPU test checks its own
            # smoothing against these to 1e-6 and then quantizes exactly these values
            for n, t in m.state_dict().items():
                if not torch.equal(t, before[n]):
                    arrays[f"{key}__smoothed__{n}"] = t.detach().clone().numpy()  # not a view: quantize_falcon rewrites per_channel weights in place
        feat = None
        if with_feat:
            # quantize_falcon looks features up as "model." + name (it walks model.named_modules())
            feat = {"model." + n: v for n, v in calib_feat(m, cal).items()}
            for n, lst in feat.items():
                arrays[f"{key}__feat__{n}"] = torch.stack(lst).numpy()
        q = ref.quantize_falcon(m, input_feat=feat, **kw)
        entry = dict(key=key, arch=arch, seed=seed, kwargs=kw, alpha=alpha,
                     cal_seeds=[1000 + seed * 10 + b for b in range(CAL_BLOCKS)], cal_len=32,
                     eval_window=EVAL_WINDOW, w_hat=w_hat_digests(q))
        arrays[f"{key}__x"] = x.numpy()
        arrays[f"{key}__ev"] = ev.numpy()
        try:
            with torch.no_grad():
                logits = q(x).logits.float()
        except Exception as e:  # the reference's own failure mode, kept as the expectation
            entry.update(raises=type(e).__name__, message=str(e))
            print(key, "raises", type(e).__name__, str(e)[:100])
        else:
            arrays[f"{key}__logits"] = logits.numpy()
            entry["ppl"] = evaluator_ppl(q, ev, EVAL_WINDOW)
            print(key, "ppl", entry["ppl"], "logits", tuple(logits.shape))
        meta.append(entry)
    info = dict(source="adithyab100/smoothquant-mixedprecision (reference quantize_falcon + "
                       "smooth_lm, CPU fp32, argsort pinned stable)",
                torch=torch.__version__, vocab=VOCAB, seq=SEQ, archs=ARCHS, cases=meta)
    arrays["meta_json"] = np.frombuffer(json.dumps(info).encode(), dtype=np.uint8)
    np.savez_compressed(OUT, **arrays)
    print("wrote", OUT)


if __name__ == "__main__":
    main()
