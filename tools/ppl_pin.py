"""Multi-seed pin of the end-to-end W4A4 forward against the reference fake-quant.

One e2e run gives one PPL delta, and on a random-init model one delta cannot be told apart
from the reference's own sensitivity to GEMM accumulation order (bench_e2e.py's
`reference_gemm_order_noise`).  This tool repeats the comparison over S random models and
token streams and reports, per seed and as mean / spread over seeds, four views of
"ours vs the reference" beside the same four of "the reference with a higher-precision GEMM
vs the reference" (the noise floor: identical operands, another accumulation -- fp32 for the
fp16 Llama, fp64 for the fp32 OPT):

  * the PPL delta, and its share of the reference PPL;
  * the mean |ΔNLL| per token;
  * the top-1 agreement of the next-token predictions;
  * the relative L2 distance of the hidden states after decoder layers 1, 2, 4, ... (window
    0), which shows how the two forwards part from layer to layer beside how the noise
    floor's do.

The W4A4 model is quantize_llama_like's / quantize_opt's (fake_quant.py:377-561, OPT with
its default bmm-input output quantization) with the HIP W4A4Linear;
the reference legs are tools/torch_fakequant.py's restatement of the reference forward
(fake_quant.py:280-375) on the same W_hat, salient sets and bound quantizers
(bench_e2e.swap_reference).  Random-init weights of the named architecture (no checkpoints
offline), random tokens.

    python tools/ppl_pin.py [--seeds 6] [--windows 2] [--layers 32] [--act-bits 4|8] [--out FILE]
"""
from __future__ import annotations

import argparse
import copy
import json
import math
import os
import sys
import time
from functools import partial

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for _p in (ROOT, os.path.join(ROOT, "smoothquant-mixedprecision_amd"), os.path.join(ROOT, "tools")):
    if _p not in sys.path:
        sys.path.insert(0, _p)

import torch  # noqa: E402

import bench_e2e as E  # noqa: E402

LAYER_MARKS = (1, 2, 4, 8, 16, 24, 32)


@torch.no_grad()
def forward_stats(model, ids, seq, n):
    """Per-token NLL and argmax over n windows, hidden states of window 0 (every layer)."""
    nll, top1, hid = [], [], None
    for i in range(n):
        x = ids[:, i * seq:(i + 1) * seq]
        out = model(x, output_hidden_states=(i == 0))
        lg = out.logits[0, :-1].float()
        lp = torch.log_softmax(lg, -1)
        nll.append(-lp.gather(1, x[0, 1:, None])[:, 0])
        top1.append(lg.argmax(-1))
        if i == 0:
            hid = [h[0].float() for h in out.hidden_states[1:]]  # after decoder layer 1..L
        del out, lg, lp
    return torch.cat(nll), torch.cat(top1), hid


def compare(a, b):
    """View of forward a against forward b (both forward_stats tuples)."""
    nll_a, top_a, hid_a = a
    nll_b, top_b, hid_b = b
    ppl_a, ppl_b = math.exp(nll_a.mean().item()), math.exp(nll_b.mean().item())
    rel = [((ha - hb).norm() / hb.norm().clamp_min(1e-30)).item() for ha, hb in zip(hid_a, hid_b)]
    return {
        "ppl_delta": ppl_a - ppl_b,
        "ppl_delta_rel": (ppl_a - ppl_b) / ppl_b,
        "mean_abs_dnll": (nll_a - nll_b).abs().mean().item(),
        "top1_agree": (top_a == top_b).float().mean().item(),
        "hidden_rel_l2": {str(l): rel[l - 1] for l in LAYER_MARKS if l <= len(rel)},
    }


def one_seed(args, seed):
    from smoothquant import fake_quant as FQ
    from smoothquant.calibration import get_calib_feat
    dev = torch.device("cuda")
    torch.manual_seed(seed)
    family, cfg, model = E.build(args.model, args.layers, E.TDT[E.MODELS[args.model][3]])
    qfn = FQ.quantize_llama_like if family == "llama" else FQ.quantize_opt
    G = E.MODELS[args.model][2]
    g = torch.Generator(device=dev).manual_seed(1000 + seed)
    ids = torch.randint(0, cfg.vocab_size, (1, args.windows * args.seq), generator=g, device=dev)
    cal = [torch.randint(0, cfg.vocab_size, (1, 512), generator=g, device=dev) for _ in range(4)]
    feat = get_calib_feat(model, None, samples=cal, device=dev)
    fp16 = forward_stats(model, ids, args.seq, args.windows)
    qmodel = qfn(copy.deepcopy(model), weight_quant="per_group", act_quant="per_group",
                 input_feat=feat, salient_prop=args.salient, quant_bits=4, group_size=G)
    if args.act_bits != 4:
        # W4A8: rebind the bound activation quantizer, as bench_e2e.py --act-bits does
        fn = FQ._ACT_FNS["per_group"]
        for m in qmodel.modules():
            if isinstance(m, FQ.W4A4Linear):
                m.act_quant = partial(fn, n_bits=args.act_bits, group_size=G)
    del model
    ours = forward_stats(qmodel, ids, args.seq, args.windows)
    E.swap_reference(qmodel, accum32=False)
    ref = forward_stats(qmodel, ids, args.seq, args.windows)
    E.swap_reference(qmodel, accum32=True)
    ref32 = forward_stats(qmodel, ids, args.seq, args.windows)
    del qmodel
    torch.cuda.empty_cache()
    return {
        "seed": seed,
        "ppl_reference": math.exp(ref[0].mean().item()),
        "ours_vs_reference": compare(ours, ref),
        "reference_fp32_gemm_vs_reference": compare(ref32, ref),
        "unquantized_vs_reference": compare(fp16, ref),
    }


def summarize(rows):
    out = {}
    for leg in ("ours_vs_reference", "reference_fp32_gemm_vs_reference", "unquantized_vs_reference"):
        d = {}
        for key in ("ppl_delta", "ppl_delta_rel", "mean_abs_dnll", "top1_agree"):
            v = torch.tensor([r[leg][key] for r in rows], dtype=torch.float64)
            d[key] = {"mean": v.mean().item(), "std": v.std().item() if len(v) > 1 else 0.0,
                      "mean_abs": v.abs().mean().item()}
        d["hidden_rel_l2_mean"] = {l: sum(r[leg]["hidden_rel_l2"][l] for r in rows) / len(rows)
                                   for l in rows[0][leg]["hidden_rel_l2"]}
        out[leg] = d
    return out


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama2-7b", choices=sorted(E.MODELS))
    ap.add_argument("--seeds", type=int, default=6)
    ap.add_argument("--windows", type=int, default=2)
    ap.add_argument("--seq", type=int, default=2048)
    ap.add_argument("--layers", type=int, default=None)
    ap.add_argument("--salient", type=float, default=0.05)
    ap.add_argument("--act-bits", type=int, default=4, help="8 = W4A8 (act_quant rebound)")
    ap.add_argument("--out", default=None)
    args = ap.parse_args(argv)
    rows = []
    t0 = time.perf_counter()
    for s in range(args.seeds):
        r = one_seed(args, s)
        rows.append(r)
        o, n = r["ours_vs_reference"], r["reference_fp32_gemm_vs_reference"]
        print(f"seed {s}: ppl_ref {r['ppl_reference']:.1f}  ours-ref {o['ppl_delta']:+.1f} "
              f"(|dNLL| {o['mean_abs_dnll']:.4f}, top1 {o['top1_agree']:.4f})  "
              f"ref32-ref {n['ppl_delta']:+.1f} (|dNLL| {n['mean_abs_dnll']:.4f}, "
              f"top1 {n['top1_agree']:.4f})  {time.perf_counter() - t0:.0f} s", flush=True)
    res = {"model": args.model, "act_bits": args.act_bits, "seeds": args.seeds, "windows": args.windows, "seq": args.seq,
           "layers": args.layers or E.MODELS[args.model][1]["num_hidden_layers"],
           "dtype": E.MODELS[args.model][3],
           "data": "random-init weights of the named architecture, random tokens, "
                   "4 x 512-token random calibration blocks per seed",
           "summary": summarize(rows), "per_seed": rows}
    text = json.dumps(res, indent=1)
    if args.out:
        with open(args.out, "w") as f:
            f.write(text + "\n")
    print(json.dumps(res["summary"], indent=1), flush=True)


if __name__ == "__main__":
    main()
