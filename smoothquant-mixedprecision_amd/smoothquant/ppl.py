"""Perplexity harness: the reference's Evaluator.

    Evaluator(dataset, tokenizer, device, n_samples=10, batch_size=2048)
        run_experiments/run_experiments.py:86-123 (smoothquant/ppl_eval.py:32-61 is the same
        with n_samples=40 and batch_size fixed at 2048)

The whole split is joined with "\\n\\n" and tokenized once; window i is tokens
[i*B, (i+1)*B); the loss is the mean cross-entropy over the B-1 shifted labels, scaled by
B, and PPL = exp(sum(nll) / (n * B)).  n_samples=None (or 0) evaluates every full window.
`dataset` is anything with a "text" column (a `datasets.Dataset`, or {"text": [...]}) --
pass local data when the hub is not reachable; `input_ids` may also be given directly.
"""
import time

import torch
import torch.nn as nn

try:
    from tqdm import tqdm as _tqdm
except ImportError:  # pragma: no cover
    def _tqdm(it, **_kw):
        return it


class Evaluator:
    def __init__(self, dataset, tokenizer, device, n_samples=10, batch_size=2048, input_ids=None):
        self.dataset = dataset
        self.tokenizer = tokenizer
        self.device = device
        if input_ids is None:
            input_ids = tokenizer("\n\n".join(dataset["text"]), return_tensors="pt").input_ids
        self.dataset = input_ids.to(device)
        self.n_samples = n_samples
        self.batch_size = batch_size
        self.last_tokens_per_s = None

    @torch.no_grad()
    def evaluate(self, model):
        model.eval()
        nlls = []
        B = self.batch_size
        n_samples = self.n_samples if self.n_samples else self.dataset.size(1) // B
        dev = next(model.parameters()).device if any(True for _ in model.parameters()) else self.device
        t0 = time.perf_counter()
        for i in _tqdm(range(n_samples), desc="Evaluating"):
            batch = self.dataset[:, i * B:(i + 1) * B].to(dev)
            lm_logits = model(batch).logits
            shift_logits = lm_logits[:, :-1, :].contiguous().float()
            shift_labels = self.dataset[:, i * B:(i + 1) * B][:, 1:].to(shift_logits.device)
            loss = nn.CrossEntropyLoss()(shift_logits.view(-1, shift_logits.size(-1)),
                                         shift_labels.reshape(-1))
            nlls.append(loss.float() * B)
        if torch.cuda.is_available():
            torch.cuda.synchronize()
        self.last_tokens_per_s = n_samples * B / (time.perf_counter() - t0)
        return torch.exp(torch.stack(nlls).sum() / (n_samples * B))


__all__ = ["Evaluator"]
