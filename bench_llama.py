"""Config 4 of BASELINE.json: Llama-2-7B W4A4 end-to-end prefill tokens/s on 1 MI355X.

    python bench_llama.py [--layers 32] [--windows 8] [--seq 2048] [--group 64]
                          [--salient 0.05] [--act per_group] [--cal-blocks 4]

Llama-2-7B architecture (hidden 4096, intermediate 11008, 32 layers, 32 heads, vocab
32000) with random-init fp16 weights built directly on the GPU -- there are no
checkpoints offline, so perplexities are those of a random model and only their DELTA
between the fp16 and W4A4 runs of the same weights is meaningful.  Importance: the
reference's mean|x| calibration features (smoothquant.calibration.get_calib_feat) over
synthetic 512-token blocks; quantization: quantize_llama_like(weight per_group, act
per_group, group_size=64, 5 % salient) -- every nn.Linear of the decoder becomes a HIP
W4A4Linear.  Timing: Evaluator-style prefill windows of `seq` tokens, batch 1, wall
clock around the whole window loop (after one warm-up window), for the fp16 model and
then the W4A4 model.  Prints one JSON line.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
for _p in (ROOT, os.path.join(ROOT, "smoothquant-mixedprecision_amd")):
    if _p not in sys.path:
        sys.path.insert(0, _p)

import torch  # noqa: E402
import torch.nn as nn  # noqa: E402


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--layers", type=int, default=32)
    ap.add_argument("--windows", type=int, default=8)
    ap.add_argument("--seq", type=int, default=2048)
    ap.add_argument("--group", type=int, default=64)
    ap.add_argument("--salient", type=float, default=0.05)
    ap.add_argument("--act", default="per_group")
    ap.add_argument("--weight", default="per_group")
    ap.add_argument("--cal-blocks", type=int, default=4)
    return ap.parse_args()


@torch.no_grad()
def run_windows(model, ids, seq, n):
    """Evaluator loop (run_experiments.py:86-123): returns (ppl, seconds for n windows)."""
    nlls = []
    model(ids[:, :seq])  # warm-up window (kernel selection, allocator)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(n):
        batch = ids[:, i * seq:(i + 1) * seq]
        logits = model(batch).logits
        sl = logits[:, :-1, :].contiguous().float()
        loss = nn.CrossEntropyLoss()(sl.view(-1, sl.size(-1)), batch[:, 1:].reshape(-1))
        nlls.append(loss.float() * seq)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    return float(torch.exp(torch.stack(nlls).sum() / (n * seq))), dt


def main():
    args = parse()
    from transformers import LlamaConfig, LlamaForCausalLM
    from smoothquant.calibration import get_calib_feat
    from smoothquant.fake_quant import W4A4Linear, quantize_llama_like
    dev = torch.device("cuda")
    cfg = LlamaConfig(vocab_size=32000, hidden_size=4096, intermediate_size=11008,
                      num_hidden_layers=args.layers, num_attention_heads=32,
                      num_key_value_heads=32, max_position_embeddings=4096, rms_norm_eps=1e-5,
                      attn_implementation="sdpa")
    torch.manual_seed(0)
    t_build = time.perf_counter()
    prev = torch.get_default_dtype()
    torch.set_default_dtype(torch.float16)
    with torch.device(dev):
        model = LlamaForCausalLM(cfg).eval()
    torch.set_default_dtype(prev)
    t_build = time.perf_counter() - t_build
    g = torch.Generator(device=dev).manual_seed(1)
    ids = torch.randint(0, cfg.vocab_size, (1, args.windows * args.seq), generator=g, device=dev)
    cal = [torch.randint(0, cfg.vocab_size, (1, 512), generator=g, device=dev)
           for _ in range(args.cal_blocks)]

    ppl16, dt16 = run_windows(model, ids, args.seq, args.windows)

    t_q = time.perf_counter()
    feat = get_calib_feat(model, None, samples=cal, device=dev)
    model = quantize_llama_like(model, weight_quant=args.weight, act_quant=args.act,
                                input_feat=feat, salient_prop=args.salient, quant_bits=4,
                                group_size=args.group)
    torch.cuda.synchronize()
    t_q = time.perf_counter() - t_q
    n_w4 = sum(isinstance(m, W4A4Linear) for m in model.modules())
    ppl4, dt4 = run_windows(model, ids, args.seq, args.windows)

    # reference point: every W4A4Linear replaced by the reference's fake-quant forward
    # (restated in PyTorch ops, tools/torch_fakequant.py) on the same W_hat / salient set
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    from torch_fakequant import TorchFakeQuantLinear

    class RefLinear(nn.Module):
        def __init__(self, q):
            super().__init__()
            b = None if q.bias is None else q.bias.reshape(-1)
            self.f = TorchFakeQuantLinear(q.weight, b, q.salient_indices, q.act_quant_name,
                                          q.quant_bits, q.group_size)

        def forward(self, x):
            return self.f(x)

    for name, m in list(model.named_modules()):
        for attr, child in list(m.named_children()):
            if isinstance(child, W4A4Linear):
                setattr(m, attr, RefLinear(child))
    pplr, dtr = run_windows(model, ids, args.seq, args.windows)

    tokens = args.windows * args.seq
    lin_flops_per_token = 2 * args.layers * (4 * 4096 * 4096 + 3 * 4096 * 11008)
    out = {
        "metric": "Llama-2-7B W4A4 prefill tokens/s (1 GPU)",
        "value": round(tokens / dt4, 1),
        "unit": "tokens/s",
        "higher_is_better": True,
        "n_gpus": 1,
        "fp16_tokens_per_s": round(tokens / dt16, 1),
        "w4a4_over_fp16": round(dt16 / dt4, 4),
        "reference_fakequant_tokens_per_s": round(tokens / dtr, 1),
        "speedup_vs_reference_fakequant": round(dtr / dt4, 2),
        "ppl_reference_fakequant": round(pplr, 4),
        "ppl_fp16": round(ppl16, 4),
        "ppl_w4a4": round(ppl4, 4),
        "ppl_delta": round(ppl4 - ppl16, 4),
        "linear_TFLOP_per_s_w4a4": round(lin_flops_per_token * tokens / dt4 / 1e12, 1),
        "data": "synthetic: random-init fp16 weights (Llama-2-7B shapes), random tokens; "
                "PPL values are of a random model -- only the delta is meaningful",
        "config": {"workload": "Llama-2-7B prefill, batch 1", "layers": args.layers,
                   "seq_len": args.seq, "windows": args.windows, "group_size": args.group,
                   "salient_prop": args.salient, "weight_quant": args.weight,
                   "act_quant": args.act, "w4a4_linears": n_w4,
                   "calibration": f"{args.cal_blocks} x 512 random tokens"},
        "setup_s": {"build": round(t_build, 1), "calibrate_and_quantize": round(t_q, 1)},
    }
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
