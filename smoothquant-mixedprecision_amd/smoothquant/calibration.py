"""Calibration statistics for the W4A4 path.

All of this is offline, host-orchestrated PyTorch: one `LinearInputStats` object hooks
every nn.Linear of a model and folds a per-module statistic of its input (or output)
over the calibration batches.  The statistics feed `W4A4Linear.from_float(importance=)`
and `smooth_lm`; none of it runs on the per-token hot path.

Reference semantics kept (names and return values are the reference's API):
  get_act_scales                   smoothquant/calibration.py:13-51  running max over
                                   batches of the per-channel absmax, fp32 on the CPU
  get_static_decoder_layer_scales  smoothquant/calibration.py:54-130 whole-tensor absmax
                                   of each Linear's input and output; per layer / 127
  get_calib_dataset                run_experiments/run_experiments.py:30-53
  get_calib_feat                   run_experiments/run_experiments.py:55-84 one mean|x|
                                   vector per batch (model dtype, CPU) per Linear

Datasets: with a path / no dataset the reference's own `load_dataset` calls are made;
without hub access pass a `datasets.Dataset` or a list of rows ({"text": ...} or plain
strings) and the reference's `shuffle(seed=42)` order is applied to it.
"""
from __future__ import annotations

import functools
from collections import defaultdict
from typing import Callable, Dict, Iterable, List

import torch
import torch.nn as nn

try:  # progress bars only
    from tqdm import tqdm as _progress
except ImportError:  # pragma: no cover
    def _progress(it, **_kw):
        return it


# ------------------------------------------------------------------ datasets
def _shuffled_rows(source, default_loader: Callable):
    """The calibration rows in the reference's order: `shuffle(seed=42)` of the dataset."""
    if source is None or isinstance(source, str):
        ds = default_loader(source)
    elif hasattr(source, "shuffle"):
        ds = source
    else:
        from datasets import Dataset
        ds = Dataset.from_list([r if isinstance(r, dict) else {"text": r} for r in source])
    return ds.shuffle(seed=42)


def _json_rows(path):
    from datasets import load_dataset
    return load_dataset("json", data_files=path, split="train")


def _wikitext_validation(_unused):
    from datasets import load_dataset
    return load_dataset("wikitext", "wikitext-2-raw-v1", split="validation")


# ------------------------------------------------------------------ statistics
def _first(t):
    return t[0] if isinstance(t, tuple) else t


def _is_linear_like(m: nn.Module) -> bool:
    """nn.Linear, and the transformers-5 MoE router (MixtralTopKRouter: an [E, H] weight
    applied by F.linear -- an nn.Linear named `gate` in the reference's transformers 4.x)."""
    return isinstance(m, nn.Linear) or type(m).__name__ == "MixtralTopKRouter"


class LinearInputStats:
    """Forward hooks on every nn.Linear of `model`; `fold(name, old, x, y)` returns the
    module's new statistic (old is None on its first call)."""

    def __init__(self, model: nn.Module, fold: Callable):
        self.stats: Dict[str, object] = {}
        self._fold = fold
        self._handles = [m.register_forward_hook(functools.partial(self._on_forward, name))
                         for name, m in model.named_modules() if _is_linear_like(m)]

    def _on_forward(self, name, module, inputs, output):
        self.stats[name] = self._fold(name, self.stats.get(name), _first(inputs), _first(output))

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        for h in self._handles:
            h.remove()
        self._handles = []
        return False


def _fold_channel_absmax(_name, old, x, _y):
    # per-channel absmax of this batch, fp32 on the host; running max over batches
    cur = x.reshape(-1, x.shape[-1]).abs().detach().amax(dim=0).float().cpu()
    return cur if old is None else torch.maximum(old, cur)


def _fold_channel_mean_list(_name, old, x, _y):
    # one mean_m |x[m, k]| vector per batch, kept in the model dtype on the host
    cur = x.reshape(-1, x.shape[-1]).abs().mean(dim=0).detach().cpu()
    return [cur] if old is None else old + [cur]


def _fold_io_absmax(_name, old, x, y):
    xin = x.detach().abs().max().item()
    xout = y.detach().abs().max().item()
    if old is None:
        return {"input": xin, "output": xout}
    return {"input": max(old["input"], xin), "output": max(old["output"], xout)}


def _run_text_rows(model, tokenizer, rows, num_samples, seq_len):
    device = next(model.parameters()).device
    for i in _progress(range(num_samples)):
        ids = tokenizer(rows[i]["text"], return_tensors="pt", max_length=seq_len,
                        truncation=True).input_ids
        model(ids.to(device))


@torch.no_grad()
def get_act_scales(model, tokenizer, dataset_path, num_samples=512, seq_len=512):
    """{Linear name: fp32 CPU (K,)} per-input-channel absmax over the calibration rows."""
    model.eval()
    rows = _shuffled_rows(dataset_path, _json_rows)
    with LinearInputStats(model, _fold_channel_absmax) as col:
        _run_text_rows(model, tokenizer, rows, num_samples, seq_len)
    return col.stats


@torch.no_grad()
def get_static_decoder_layer_scales(model, tokenizer, dataset_path, num_samples=512,
                                    seq_len=512):
    """(per-layer static int8 scales of an OPT decoder, {name: {"input", "output"}})."""
    model.eval()
    rows = _shuffled_rows(dataset_path, _json_rows)
    with LinearInputStats(model, _fold_io_absmax) as col:
        _run_text_rows(model, tokenizer, rows, num_samples, seq_len)
    act_dict = defaultdict(dict, col.stats)
    fields = (("attn_input_scale", "self_attn.q_proj", "input"),
              ("q_output_scale", "self_attn.q_proj", "output"),
              ("k_output_scale", "self_attn.k_proj", "output"),
              ("v_output_scale", "self_attn.v_proj", "output"),
              ("out_input_scale", "self_attn.out_proj", "input"),
              ("fc1_input_scale", "fc1", "input"),
              ("fc2_input_scale", "fc2", "input"))
    layers = []
    for idx in range(model.config.num_hidden_layers):
        base = f"model.decoder.layers.{idx}."
        layers.append({key: act_dict[base + mod][io] / 127 for key, mod, io in fields})
    return layers, act_dict


def _kept_lines(rows: Iterable, tokenizer, n_samples: int, block_size: int):
    """Token lists of the first `n_samples` stripped lines with 1..block_size tokens."""
    kept = 0
    for row in rows:
        ids = tokenizer.encode(row["text"].strip())
        if not ids or len(ids) > block_size:
            continue
        yield ids
        kept += 1
        if kept == n_samples:
            return


def get_calib_dataset(tokenizer=None, n_samples=256, block_size=512, dataset=None):
    """[1, block_size] LongTensor blocks cut from the concatenation of the kept lines."""
    rows = _shuffled_rows(dataset, _wikitext_validation)
    stream: List[int] = []
    for ids in _kept_lines(rows, tokenizer, n_samples, block_size):
        stream.extend(ids)
    flat = torch.tensor([stream], dtype=torch.long)
    n_blocks = flat.shape[1] // block_size
    return list(flat[:, :n_blocks * block_size].split(block_size, dim=1))


@torch.no_grad()
def get_calib_feat(model, tokenizer, samples=None, device=None, **dataset_kw):
    """{Linear name: [mean_m |x| per calibration block]} -- the salient-channel importance
    inputs that quantize_* sum and cast to fp32 (fake_quant.py:396)."""
    if device is None:
        device = torch.device("cuda" if torch.cuda.is_available() else "cpu")
    blocks = get_calib_dataset(tokenizer, **dataset_kw) if samples is None else samples
    with LinearInputStats(model, _fold_channel_mean_list) as col:
        for ids in _progress(blocks):
            model(ids.to(device))
    return col.stats


__all__ = ["get_act_scales", "get_static_decoder_layer_scales", "get_calib_dataset",
           "get_calib_feat", "LinearInputStats"]
