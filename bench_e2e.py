"""End-to-end W4A4 prefill benchmarks of BASELINE.json configs 3 and 4 on 1 MI355X.

    python bench_e2e.py --model llama2-7b [--layers 32] [--windows 8] [--seq 2048] [--group 64]
                        [--salient 0.05] [--act per_group] [--weight per_group] [--cal-blocks 4]
    python bench_e2e.py --model opt-1.3b   (config 3: G=128, 5 % salient, quantize_opt with
                                            its default bmm-input output quantization)
    python bench_e2e.py --model llama2-7b --flow ppl_eval   (the reference's SmoothQuant
        baseline evaluation, smoothquant/ppl_eval.py:69-83 / examples/ppl_eval.sh: bf16 model,
        quantize_model(weight_quant="per_channel", act_quant="per_token",
        quantize_bmm_input=True), no calibration features, so no salient channels)

The architecture of the named model with random-init weights built directly on the GPU
(there are no checkpoints offline), random token windows, in the reference's dtype for that
model (run_experiments.py:146-154: Llama fp16, OPT the default fp32; --dtype overrides).  Importance: the reference's
mean|x| calibration features (smoothquant.calibration.get_calib_feat) on synthetic
512-token blocks; quantization: the reference's entry point (quantize_llama_like /
quantize_opt, fake_quant.py:377-561) with every nn.Linear of the decoder becoming a HIP
W4A4Linear.  Timing: Evaluator-style prefill (run_experiments.py:86-123), batch 1, wall
clock around the whole window loop after one warm-up window, for (1) the unquantized model,
(2) the W4A4 model (1 and 2 in interleaved rounds, best of each), (3) the reference's fake-quant forward restated in PyTorch ops
(tools/torch_fakequant.py) on the same W_hat and salient sets, with the model-dtype GEMM,
and (4) the same with a higher-precision GEMM (fp32 for fp16 / bf16 models, fp64 for fp32
models) -- (3) vs (4) is the reference's own sensitivity to GEMM accumulation, the noise
floor against which the W4A4 kernel's PPL delta reads.
Perplexities are of a random model: only differences are meaningful.

CPU baseline (north star: e2e tokens/s "next to the CPU baseline"): the same architecture
with the reference's fake-quant layers (oracle/torch_cpu.py, bit-exact to the reference's
goldens) on PyTorch-CPU in fp32, every host thread; 1 and 2 decoder layers are timed on
one window (median of 2 after a warm-up) and the whole model's time is extrapolated as
t(1) + (L - 1) * (t(2) - t(1)) -- a bounded sample, stated in the output.
"""
from __future__ import annotations

import argparse
import copy
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
for _p in (ROOT, os.path.join(ROOT, "smoothquant-mixedprecision_amd"), os.path.join(ROOT, "tools")):
    if _p not in sys.path:
        sys.path.insert(0, _p)

import torch  # noqa: E402
import torch.nn as nn  # noqa: E402

MODELS = {
    # name: (family, config kwargs, default group size, linear FLOP/token per layer factor)
    "llama2-7b": ("llama", dict(vocab_size=32000, hidden_size=4096, intermediate_size=11008,
                                num_hidden_layers=32, num_attention_heads=32,
                                num_key_value_heads=32, max_position_embeddings=4096,
                                rms_norm_eps=1e-5), 64, "fp16"),
    "opt-1.3b": ("opt", dict(vocab_size=50272, hidden_size=2048, ffn_dim=8192,
                             num_hidden_layers=24, num_attention_heads=32,
                             max_position_embeddings=2048, word_embed_proj_dim=2048,
                             do_layer_norm_before=True), 128, "fp32"),
}


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama2-7b", choices=sorted(MODELS))
    ap.add_argument("--layers", type=int, default=None)
    ap.add_argument("--windows", type=int, default=8)
    ap.add_argument("--seq", type=int, default=2048)
    ap.add_argument("--group", type=int, default=None)
    ap.add_argument("--salient", type=float, default=0.05)
    ap.add_argument("--act", default="per_group")
    ap.add_argument("--weight", default="per_group")
    ap.add_argument("--act-bits", type=int, default=4, help="8 = W4A8 (act_quant rebound)")
    ap.add_argument("--cal-blocks", type=int, default=4)
    ap.add_argument("--no-ref", action="store_true", help="skip the reference fake-quant legs")
    ap.add_argument("--dtype", default=None, choices=["fp16", "bf16", "fp32"],
                    help="model dtype (default: the reference's for this model)")
    ap.add_argument("--no-cpu", action="store_true", help="skip the CPU baseline leg")
    ap.add_argument("--flow", default="experiments", choices=["experiments", "ppl_eval"],
                    help="experiments: run_experiments.py's quantize_llama_like / quantize_opt "
                         "flow (configs 3-5); ppl_eval: smoothquant/ppl_eval.py's quantize_model "
                         "flow (bf16, per_channel W, per_token A, bmm-input output quant)")
    ap.add_argument("--rounds", type=int, default=2,
                    help="interleaved (unquantized, W4A4) timing rounds; the best of each")
    args = ap.parse_args(argv)
    if args.flow == "ppl_eval":
        # ppl_eval.py:69-83: torch_dtype=torch.bfloat16, quantize_model(...) with its
        # input_feat / salient_prop defaults (no importance -> no salient channels)
        args.dtype = args.dtype or "bf16"
        args.weight, args.act, args.salient = "per_channel", "per_token", 0.0
    return args


@torch.no_grad()
def run_windows(model, ids, seq, n, warm=1, warm_s=0.0):
    """Evaluator loop (run_experiments.py:86-123): returns (ppl, seconds for n windows) after
    `warm` untimed windows, and more until `warm_s` seconds have passed (kernel selection,
    allocator, the clock the chip settles at)."""
    nlls = []
    t_w = time.perf_counter()
    k = 0
    while k < warm or time.perf_counter() - t_w < warm_s:
        model(ids[:, :seq])
        torch.cuda.synchronize()
        k += 1
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


TDT = {"fp16": torch.float16, "bf16": torch.bfloat16, "fp32": torch.float32}


def build(name, layers, dtype=torch.float16, device="cuda"):
    family, cfg_kw, _, _ = MODELS[name]
    cfg_kw = dict(cfg_kw)
    if layers:
        cfg_kw["num_hidden_layers"] = layers
    if family == "llama":
        from transformers import LlamaConfig, LlamaForCausalLM
        cfg, cls = LlamaConfig(attn_implementation="sdpa", **cfg_kw), LlamaForCausalLM
    else:
        from transformers import OPTConfig, OPTForCausalLM
        cfg, cls = OPTConfig(attn_implementation="sdpa", **cfg_kw), OPTForCausalLM
    prev = torch.get_default_dtype()
    torch.set_default_dtype(dtype)
    with torch.device(device):
        model = cls(cfg).eval()
    torch.set_default_dtype(prev)
    return family, cfg, model


class CPURefLinear(nn.Module):
    """nn.Linear -> the reference's fake-quant layer on the host (oracle/torch_cpu.py)."""

    def __init__(self, lin, weight_quant, act, G, p, output_quant):
        super().__init__()
        from oracle.torch_cpu import CPUFakeQuantLinear
        imp = torch.rand(lin.in_features, generator=torch.Generator().manual_seed(7))
        self.f = CPUFakeQuantLinear(lin.weight.detach(), None if lin.bias is None else lin.bias.detach(),
                                    weight_quant, act, 4, G, imp, p, output_quant)

    def forward(self, x):
        return self.f(x)


@torch.no_grad()
def cpu_baseline(args, G):
    """Reference fake-quant model on PyTorch-CPU, fp32: t(1 layer), t(2 layers) on one
    window -> extrapolated whole-model tokens/s (see the module docstring)."""
    family, cfg_kw, _, _ = MODELS[args.model]
    L = args.layers or cfg_kw["num_hidden_layers"]
    seq = args.seq
    times = {}
    for nl in (1, 2):
        _, _, m = build(args.model, nl, torch.float32, "cpu")
        for name, mod in list(m.named_modules()):
            for attr, child in list(mod.named_children()):
                if isinstance(child, nn.Linear) and "lm_head" not in f"{name}.{attr}":
                    outq = ((family == "opt" or args.flow == "ppl_eval")
                            and attr in ("q_proj", "k_proj", "v_proj"))
                    setattr(mod, attr, CPURefLinear(child, args.weight, args.act, G,
                                                    args.salient, outq))
        ids = torch.randint(0, m.config.vocab_size, (1, seq),
                            generator=torch.Generator().manual_seed(3))
        m(ids[:, :128])  # warm-up
        ts = []
        for _ in range(2):
            t0 = time.perf_counter()
            m(ids)
            ts.append(time.perf_counter() - t0)
        times[nl] = sorted(ts)[0] if len(ts) == 1 else sum(ts) / len(ts)
        del m
    per_layer = max(times[2] - times[1], 1e-9)
    total = times[1] + (L - 1) * per_layer
    return {
        "tokens_per_s": round(seq / total, 2),
        "cores": torch.get_num_threads(),
        "kind": "torch-cpu-fp32 (reference fake_quant ops, oracle/torch_cpu.py)",
        "sample": (f"1 window of {seq} tokens through 1 and 2 decoder layers: {times[1]:.2f} s, "
                   f"{times[2]:.2f} s -> {L} layers extrapolated {total:.1f} s per window"),
    }


def linear_flops_per_token(model):
    return 2 * sum(m.in_features * m.out_features for n, m in model.named_modules()
                   if isinstance(m, nn.Linear) and "lm_head" not in n)


class RefLinear(nn.Module):
    """A W4A4Linear replaced by the reference's fake-quant forward on its W_hat / salient
    set and bound quantizers (tools/torch_fakequant.py)."""

    def __init__(self, q, accum32):
        super().__init__()
        from smoothquant.fake_quant import resolve_quantizer
        from torch_fakequant import TorchFakeQuantLinear
        b = None if q.bias is None else q.bias.reshape(-1)
        mode, bits, g = resolve_quantizer(q.act_quant)
        self.f = TorchFakeQuantLinear(q.weight, b, q.salient_indices, mode, bits, g,
                                      accum32=accum32,
                                      output_quant=resolve_quantizer(q.output_quant))

    def forward(self, x):
        return self.f(x)


def swap_reference(model, accum32):
    """Every W4A4Linear -> RefLinear; existing RefLinears switch their GEMM accumulation."""
    from smoothquant.fake_quant import W4A4Linear
    for _, m in list(model.named_modules()):
        for attr, child in list(m.named_children()):
            if isinstance(child, W4A4Linear):
                setattr(m, attr, RefLinear(child, accum32))
            elif isinstance(child, RefLinear):
                child.f.accum32 = accum32


def main(argv=None):
    out = run(parse(argv))
    print(json.dumps(out), flush=True)
    return out


def run(args):
    """The measurements of the module docstring for parsed `args`; returns the JSON dict."""
    from functools import partial

    from smoothquant import fake_quant as FQ
    from smoothquant.calibration import get_calib_feat
    dtn = args.dtype or MODELS[args.model][3]
    family, cfg, model = build(args.model, args.layers, TDT[dtn])
    G = args.group or MODELS[args.model][2]
    dev = torch.device("cuda")
    torch.manual_seed(0)
    g = torch.Generator(device=dev).manual_seed(1)
    ids = torch.randint(0, cfg.vocab_size, (1, args.windows * args.seq), generator=g, device=dev)
    cal = [torch.randint(0, cfg.vocab_size, (1, 512), generator=g, device=dev)
           for _ in range(args.cal_blocks)]
    flops_tok = linear_flops_per_token(model)

    t_q = time.perf_counter()
    # the unquantized model stays alive beside its quantized copy, so the two are timed in
    # interleaved rounds on the same warmed-up chip (separate runs drifted by up to 25 %)
    if args.flow == "ppl_eval":
        qfn = FQ.quantize_model
        qmodel = qfn(copy.deepcopy(model), weight_quant="per_channel", act_quant="per_token",
                     quantize_bmm_input=True)
    else:
        feat = get_calib_feat(model, None, samples=cal, device=dev)
        qfn = FQ.quantize_llama_like if family == "llama" else FQ.quantize_opt
        qmodel = qfn(copy.deepcopy(model), weight_quant=args.weight, act_quant=args.act,
                     input_feat=feat, salient_prop=args.salient, quant_bits=4, group_size=G)
    if args.act_bits != 4:
        # W4A8 (config 5): rebind the bound activation quantizer, as a reference user would
        fn = FQ._ACT_FNS[args.act]
        kw = {"group_size": G} if args.act.startswith("per_group") else {}
        for m in qmodel.modules():
            if isinstance(m, FQ.W4A4Linear):
                m.act_quant = partial(fn, n_bits=args.act_bits, **kw)
    torch.cuda.synchronize()
    t_q = time.perf_counter() - t_q
    n_w4 = sum(isinstance(m, FQ.W4A4Linear) for m in qmodel.modules())
    runs16, runs4 = [], []
    for _ in range(args.rounds):
        runs16.append(run_windows(model, ids, args.seq, args.windows))
        runs4.append(run_windows(qmodel, ids, args.seq, args.windows))
    ppl16, dt16 = min(runs16, key=lambda r: r[1])
    ppl4, dt4 = min(runs4, key=lambda r: r[1])
    del model
    model = qmodel

    tokens = args.windows * args.seq
    out = {
        "metric": f"{args.model} W4A4 prefill tokens/s (1 GPU)",
        "value": round(tokens / dt4, 1),
        "unit": "tokens/s",
        "higher_is_better": True,
        "n_gpus": 1,
        "dtype": dtn,
        "unquantized_tokens_per_s": round(tokens / dt16, 1),
        "w4a4_over_unquantized": round(dt16 / dt4, 4),
        "ppl_unquantized": round(ppl16, 4),
        "ppl_w4a4": round(ppl4, 4),
        "linear_TFLOP_per_s_w4a4": round(flops_tok * tokens / dt4 / 1e12, 1),
        "rounds_s": {"unquantized": [round(r[1], 4) for r in runs16],
                     "w4a4": [round(r[1], 4) for r in runs4]},
    }
    if not args.no_ref:
        swap_reference(model, accum32=False)
        pplr, dtr = run_windows(model, ids, args.seq, args.windows)
        swap_reference(model, accum32=True)
        pplr32, _ = run_windows(model, ids, args.seq, args.windows)
        out.update({
            "reference_fakequant_tokens_per_s": round(tokens / dtr, 1),
            "speedup_vs_reference_fakequant": round(dtr / dt4, 2),
            "ppl_reference_fakequant": round(pplr, 4),
            "ppl_reference_fakequant_fp32_gemm": round(pplr32, 4),
            "ppl_delta_vs_reference": round(ppl4 - pplr, 4),
            "reference_gemm_order_noise": round(pplr32 - pplr, 4),
            "noise_gemm_dtype": "fp64" if dtn == "fp32" else "fp32",
        })
    out.update({
        "data": f"synthetic: random-init {dtn} weights of the named architecture, random tokens; "
                "PPL values are of a random model -- only differences are meaningful",
        "config": {"workload": f"{args.model} prefill, batch 1", "layers": cfg.num_hidden_layers,
                   "seq_len": args.seq, "windows": args.windows, "group_size": G,
                   "salient_prop": args.salient, "weight_quant": args.weight,
                   "act_quant": args.act, "act_bits": args.act_bits, "w4a4_linears": n_w4,
                   "quantizer": qfn.__name__, "flow": args.flow,
                   "calibration": f"{args.cal_blocks} x 512 random tokens"},
        "setup_s": {"calibrate_and_quantize": round(t_q, 1)},
    })
    if not args.no_cpu:
        del model
        torch.cuda.empty_cache()
        cpu = cpu_baseline(args, G)
        cpu["w4a4_gpu_over_cpu"] = round(out["value"] / cpu["tokens_per_s"], 1)
        out["cpu_baseline"] = cpu
    return out


if __name__ == "__main__":
    main()
