"""Golden fixtures for BASELINE configs 1, 3 and 4 at their real layer dimensions, from the
REFERENCE (run on this container's CPU; tests/config_cases.py defines the cases).

For every case: build the seeded random-init model (config_cases.build), collect the
mean|x| calibration features with the reference's hook formula (run_experiments.py:55-84)
and sum them into each Linear's importance (fake_quant.py:396 / :486), quantize with the
reference's own `quantize_opt` / `quantize_llama_like` (argsort pinned stable, as in
gen_golden.py) and run the eval sequence.  Stored (small; no model tensors):
  <key>__imp__<linear>    fp32 importance the quantizer consumed (fed back as [imp])
  <key>__sal__<linear>    the reference's salient_indices (int32)
  meta: per linear the sha256 of W_hat (-0.0 folded to +0.0) and its fp64 sum, shapes and
        modes; per case the eval loss (mean next-token CE, fp64) and the logits norm
  meta noise_*: the reference's own spread when its F.linear accumulates in fp64 instead
        (logits / logsumexp relative, |loss difference|): the model-level noise floor
  <key>__logits, __lse    fp32 logits[:, :VOCAB_SLICE] and the fp64 logsumexp over the
                          vocabulary at config_cases.positions(case)

Usage:  python tests/golden/gen_config_golden.py     (needs /root/reference)
"""
from __future__ import annotations

import json
import os
import sys
import time

import numpy as np
import torch
import torch.nn as nn

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.dirname(HERE))
from gen_golden import _StableTorch, load_reference  # noqa: E402

REF_SMOOTH = "/root/reference/smoothquant/smooth.py"
import config_cases as C  # noqa: E402


@torch.no_grad()
def importance_of(model, blocks):
    """{linear name: sum over blocks of mean_m |x| (model dtype), cast to fp32}."""
    feat = {}

    def hook(name, m, inp, out):
        x = inp[0] if isinstance(inp, tuple) else inp
        feat.setdefault(name, []).append(x.view(-1, x.shape[-1]).abs().mean(dim=0).cpu())

    hs = [m.register_forward_hook(lambda m, i, o, n=n: hook(n, m, i, o))
          for n, m in model.named_modules() if isinstance(m, nn.Linear)]
    for b in blocks:
        model(b)
    for h in hs:
        h.remove()
    return {n: sum(v).float() for n, v in feat.items()}


@torch.no_grad()
def eval_loss(logits, ids):
    pred = logits[:, :-1].double()
    return float(nn.functional.cross_entropy(pred.reshape(-1, pred.shape[-1]),
                                             ids[:, 1:].reshape(-1)))


class _F64LinearTorch(_StableTorch):
    """The reference's `torch` with F.linear accumulated in fp64 (rounded once to the
    model dtype): the same fake-quant model under another GEMM accumulation order."""

    class _Functional:
        class F:
            @staticmethod
            def linear(x, w, b=None):
                y = nn.functional.linear(x.double(), w.double(), None if b is None else b.double())
                return y.to(x.dtype)

    functional = _Functional


def _rel(a, b):
    return float((a.double() - b.double()).norm() / b.double().norm())


@torch.no_grad()
def act_scales_of(model, blocks):
    """{linear name: per-channel max|x| over the blocks, fp32} -- the statistic of
    calibration.get_act_scales (calibration.py:13-51) on the given token blocks."""
    scales = {}

    def hook(name, m, inp, out):
        x = inp[0] if isinstance(inp, tuple) else inp
        cur = x.view(-1, x.shape[-1]).abs().max(dim=0)[0].float().cpu()
        scales[name] = cur if name not in scales else torch.max(scales[name], cur)

    hs = [m.register_forward_hook(lambda m, i, o, n=n: hook(n, m, i, o))
          for n, m in model.named_modules() if isinstance(m, nn.Linear)]
    for b in blocks:
        model(b)
    for h in hs:
        h.remove()
    return scales


def load_smooth():
    import importlib.util
    sys.dont_write_bytecode = True
    spec = importlib.util.spec_from_file_location("_ref_smooth", REF_SMOOTH)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def main():
    ref = load_reference()
    torch.set_num_threads(os.cpu_count() or 8)
    arrays, cases = {}, {}
    only = None
    if "--only" in sys.argv:
        # regenerate the named cases, keep every other case of the existing fixture
        only = set(sys.argv[sys.argv.index("--only") + 1].split(","))
        old = np.load(C.GOLDEN, allow_pickle=False)
        old_meta = json.loads(bytes(old["meta_json"]).decode())
        for k in old.files:
            if k != "meta_json" and k.split("__")[0] not in only:
                arrays[k] = old[k]
        cases = {k: v for k, v in old_meta["cases"].items() if k not in only}
    for case in C.CASES:
        t0 = time.time()
        key = case["key"]
        if only is not None and key not in only:
            continue
        model = C.build(case)
        if case.get("smooth") is not None:
            sc = act_scales_of(model, C.tokens(case, "cal"))
            for n, v in sc.items():
                arrays[f"{key}__act__{n}"] = v.numpy()
            load_smooth().smooth_lm(model, sc, case["smooth"])
        w_orig = {n: m.weight.detach().clone() for n, m in model.named_modules()
                  if isinstance(m, nn.Linear)}
        if case.get("input_feat", True):
            imp = importance_of(model, C.tokens(case, "cal"))
            for n, v in imp.items():
                arrays[f"{key}__imp__{n}"] = v.numpy()
            # input_feat as the quantizers index it ("model." + module path); one-element
            # lists so sum(...) returns the stored fp32 importance unchanged
            feat = {n: [v] for n, v in imp.items()}
            q = getattr(ref, case["quantizer"])(model, input_feat=feat, **case["kwargs"])
        else:
            q = getattr(ref, case["quantizer"])(model, **case["kwargs"])
        C.post_quantize(q, case, ref, w_orig)
        linears = {}
        for n, m in q.named_modules():
            if type(m).__name__ != "W4A4Linear":
                continue
            sal = m.salient_indices
            if sal is not None:
                arrays[f"{key}__sal__{n}"] = sal.numpy().astype(np.int32)
            w = m.weight
            linears[n] = dict(N=int(w.shape[0]), K=int(w.shape[1]),
                              weight_quant=m.weight_quant_name, act_quant=m.act_quant_name,
                              output_quant=m.output_quant_name,
                              n_salient=0 if sal is None else int(sal.numel()),
                              what_sha256=C.what_digest(w),
                              what_sum=float(w.double().sum()))
        ids = C.tokens(case, "eval")
        with torch.no_grad():
            logits = q(ids).logits.float()
        # the reference's own accumulation-order noise on this model: the same quantized
        # model with every F.linear (fake_quant.py:306) accumulated in fp64
        real_torch = ref.torch
        ref.torch = _F64LinearTorch(torch)
        with torch.no_grad():
            logits64 = q(ids).logits.float()
        ref.torch = real_torch
        pos = C.positions(case)
        # a vocabulary slice of the logits at the stored positions + the full-vocabulary
        # logsumexp there (keeps the fixture small for the 50272-entry OPT-125M head)
        arrays[f"{key}__logits"] = logits[0, pos, :C.VOCAB_SLICE].numpy()
        arrays[f"{key}__lse"] = torch.logsumexp(logits[0, pos].double(), dim=-1).numpy()
        cases[key] = dict(n_linears=len(linears), linears=linears,
                          loss=eval_loss(logits, ids),
                          logits_norm=float(logits.double().norm()),
                          noise_logits_rel=_rel(logits64[0, pos, :C.VOCAB_SLICE],
                                                logits[0, pos, :C.VOCAB_SLICE]),
                          noise_lse_rel=_rel(torch.logsumexp(logits64[0, pos].double(), -1),
                                             torch.logsumexp(logits[0, pos].double(), -1)),
                          noise_loss=abs(eval_loss(logits64, ids) - eval_loss(logits, ids)),
                          positions=pos.tolist())
        print(f"{key}: {len(linears)} W4A4Linear, loss {cases[key]['loss']:.5f}, noise "
              f"logits {cases[key]['noise_logits_rel']:.3e} loss {cases[key]['noise_loss']:.3e}, "
              f"{time.time() - t0:.1f} s", flush=True)
        del model, q, logits
    meta = dict(source="adithyab100/smoothquant-mixedprecision reference fake_quant.py on CPU "
                       "(argsort pinned stable=True)", torch=torch.__version__, cases=cases)
    arrays["meta_json"] = np.frombuffer(json.dumps(meta).encode(), dtype=np.uint8)
    np.savez_compressed(C.GOLDEN, **arrays)
    print(f"wrote {C.GOLDEN}: {os.path.getsize(C.GOLDEN) / 1e6:.2f} MB")


if __name__ == "__main__":
    main()
