"""Perplexity harness with the reference's Evaluator interface.

    Evaluator(dataset, tokenizer, device, n_samples=10, batch_size=2048)
        behaviour of run_experiments/run_experiments.py:86-123 (smoothquant/ppl_eval.py:32-61
        is the same with n_samples=40)

The split is joined with "\\n\\n" and tokenized once into a [1, T] id stream.  Window i is
ids[:, i*B:(i+1)*B]; its negative log-likelihood is B x the mean cross-entropy of the
B-1 next-token predictions (fp32 logits) -- B = batch_size for every window, a short last
window included, as the reference computes it -- and PPL = exp(sum of window NLLs / (n*B)).
n_samples=None/0 means size // 2048 windows (the reference's count, whatever B is).
Without hub access pass a dataset with a
"text" column, or the token ids directly (`input_ids=`).  `last_tokens_per_s` is the
throughput of the last evaluate() (windows x B tokens over its wall time).
"""
from __future__ import annotations

import time

import torch
import torch.nn.functional as F

try:
    from tqdm import tqdm as _progress
except ImportError:  # pragma: no cover
    def _progress(it, **_kw):
        return it


def window_nll(model, window: torch.Tensor, batch_size=None) -> torch.Tensor:
    """batch_size x mean next-token cross-entropy of one [1, B] window (fp32 scalar tensor).
    The reference scales EVERY window by self.batch_size (run_experiments.py:120), also a
    short last window; batch_size=None uses the window's own length."""
    logits = model(window).logits
    pred = logits[:, :-1, :].float()
    target = window[:, 1:].to(pred.device)
    ce = F.cross_entropy(pred.reshape(-1, pred.shape[-1]), target.reshape(-1))
    return ce.float() * (window.shape[1] if batch_size is None else batch_size)


def _model_device(model, fallback):
    for p in model.parameters():
        return p.device
    return fallback


class Evaluator:
    def __init__(self, dataset, tokenizer, device, n_samples=10, batch_size=2048, input_ids=None):
        self.tokenizer = tokenizer
        self.device = device
        ids = input_ids
        if ids is None:
            ids = tokenizer("\n\n".join(dataset["text"]), return_tensors="pt").input_ids
        self.dataset = ids.to(device)
        self.n_samples = n_samples
        self.batch_size = batch_size
        self.last_tokens_per_s = None

    def windows(self):
        B = self.batch_size
        # n_samples falsy: the reference counts 2048-token windows whatever batch_size is
        # (run_experiments.py:103), then slices windows of batch_size
        n = self.n_samples or self.dataset.shape[1] // 2048
        return [self.dataset[:, i * B:(i + 1) * B] for i in range(n)]

    @torch.no_grad()
    def evaluate(self, model):
        model.eval()
        dev = _model_device(model, self.device)
        wins = self.windows()
        start = time.perf_counter()
        total = torch.stack([window_nll(model, w.to(dev), self.batch_size)
                             for w in _progress(wins, desc="Evaluating")]).sum()
        if torch.cuda.is_available():
            torch.cuda.synchronize()
        tokens = len(wins) * self.batch_size
        self.last_tokens_per_s = tokens / (time.perf_counter() - start)
        return torch.exp(total / tokens)


__all__ = ["Evaluator", "window_nll"]
