"""Calibration statistics for the W4A4 path (§8f rows 1 and 4).

Everything here is offline, host-orchestrated PyTorch (forward hooks on the model's
nn.Linear modules); the statistics feed `W4A4Linear.from_float(importance=...)` and
`smooth_lm`, never the per-token hot path.

  get_act_scales                   the reference's smoothquant/calibration.py:13-51
  get_static_decoder_layer_scales  smoothquant/calibration.py:54-133
  get_calib_dataset                run_experiments/run_experiments.py:30-53
  get_calib_feat                   run_experiments/run_experiments.py:55-84

Datasets: the reference reads `load_dataset("json", data_files=...)` (act scales) and
`load_dataset("wikitext", "wikitext-2-raw-v1", split="validation")` (calibration
features).  The same calls are made here when no dataset is passed; callers without hub
access pass any `datasets.Dataset` (or a list of {"text": ...} rows, which is wrapped
into one) and get the reference's `shuffle(seed=42)` order over it.
"""
import functools
from collections import defaultdict

import torch
import torch.nn as nn

try:  # tqdm is optional: progress bars only
    from tqdm import tqdm as _tqdm
except ImportError:  # pragma: no cover
    def _tqdm(it, **_kw):
        return it


def _as_dataset(dataset):
    """A `datasets.Dataset` for `dataset` (a Dataset already, or a list of rows)."""
    if hasattr(dataset, "shuffle"):
        return dataset
    from datasets import Dataset
    rows = [r if isinstance(r, dict) else {"text": r} for r in dataset]
    return Dataset.from_list(rows)


def _linear_hooks(model, hook):
    hooks = []
    for name, m in model.named_modules():
        if isinstance(m, nn.Linear):
            hooks.append(m.register_forward_hook(functools.partial(hook, name=name)))
    return hooks


@torch.no_grad()
def get_act_scales(model, tokenizer, dataset_path, num_samples=512, seq_len=512):
    """Per-input-channel absmax of every nn.Linear input (calibration.py:13-51).

    `dataset_path` is a JSON(-lines) file with a "text" field, as in the reference; a
    `datasets.Dataset` or a list of rows is accepted too.  Returns {name: fp32 CPU (K,)}.
    """
    model.eval()
    device = next(model.parameters()).device
    act_scales = {}

    def stat_tensor(name, tensor):
        hidden_dim = tensor.shape[-1]
        tensor = tensor.view(-1, hidden_dim).abs().detach()
        coming_max = torch.max(tensor, dim=0)[0].float().cpu()
        if name in act_scales:
            act_scales[name] = torch.max(act_scales[name], coming_max)
        else:
            act_scales[name] = coming_max

    def stat_input_hook(m, x, y, name):
        if isinstance(x, tuple):
            x = x[0]
        stat_tensor(name, x)

    hooks = _linear_hooks(model, stat_input_hook)
    try:
        if isinstance(dataset_path, str):
            from datasets import load_dataset
            dataset = load_dataset("json", data_files=dataset_path, split="train")
        else:
            dataset = _as_dataset(dataset_path)
        dataset = dataset.shuffle(seed=42)
        for i in _tqdm(range(num_samples)):
            input_ids = tokenizer(dataset[i]["text"], return_tensors="pt", max_length=seq_len,
                                  truncation=True).input_ids.to(device)
            model(input_ids)
    finally:
        for h in hooks:
            h.remove()
    return act_scales


@torch.no_grad()
def get_static_decoder_layer_scales(model, tokenizer, dataset_path, num_samples=512, seq_len=512):
    """Per-layer static int8 scales of an OPT decoder (calibration.py:54-133).

    Returns (decoder_layer_scales, act_dict): act_dict[name] = {"input": absmax,
    "output": absmax} over all samples; the per-layer dict divides by 127.
    """
    model.eval()
    device = next(model.parameters()).device
    act_dict = defaultdict(dict)

    def stat_io_hook(m, x, y, name):
        if isinstance(x, tuple):
            x = x[0]
        v = x.detach().abs().max().item()
        act_dict[name]["input"] = max(act_dict[name].get("input", v), v)
        if isinstance(y, tuple):
            y = y[0]
        v = y.detach().abs().max().item()
        act_dict[name]["output"] = max(act_dict[name].get("output", v), v)

    hooks = _linear_hooks(model, stat_io_hook)
    try:
        if isinstance(dataset_path, str):
            from datasets import load_dataset
            dataset = load_dataset("json", data_files=dataset_path, split="train")
        else:
            dataset = _as_dataset(dataset_path)
        dataset = dataset.shuffle(seed=42)
        for i in _tqdm(range(num_samples)):
            input_ids = tokenizer(dataset[i]["text"], return_tensors="pt", max_length=seq_len,
                                  truncation=True).input_ids.to(device)
            model(input_ids)
    finally:
        for h in hooks:
            h.remove()

    decoder_layer_scales = []
    for idx in range(model.config.num_hidden_layers):
        pre = f"model.decoder.layers.{idx}."
        decoder_layer_scales.append({
            "attn_input_scale": act_dict[pre + "self_attn.q_proj"]["input"] / 127,
            "q_output_scale": act_dict[pre + "self_attn.q_proj"]["output"] / 127,
            "k_output_scale": act_dict[pre + "self_attn.k_proj"]["output"] / 127,
            "v_output_scale": act_dict[pre + "self_attn.v_proj"]["output"] / 127,
            "out_input_scale": act_dict[pre + "self_attn.out_proj"]["input"] / 127,
            "fc1_input_scale": act_dict[pre + "fc1"]["input"] / 127,
            "fc2_input_scale": act_dict[pre + "fc2"]["input"] / 127,
        })
    return decoder_layer_scales, act_dict


def get_calib_dataset(tokenizer=None, n_samples=256, block_size=512, dataset=None):
    """Calibration blocks (run_experiments.py:30-53): shuffle(seed=42), keep stripped lines
    of at most `block_size` tokens (and at least one), stop after `n_samples` lines,
    concatenate, split into `block_size`-token blocks [1, block_size]."""
    if dataset is None:
        from datasets import load_dataset
        dataset = load_dataset("wikitext", "wikitext-2-raw-v1", split="validation")
    dataset = _as_dataset(dataset).shuffle(seed=42)
    samples = []
    n_run = 0
    for data in dataset:
        line_encoded = tokenizer.encode(data["text"].strip())
        if len(line_encoded) > block_size:
            continue
        sample = torch.tensor([line_encoded])
        if sample.numel() == 0:
            continue
        samples.append(sample)
        n_run += 1
        if n_run == n_samples:
            break
    cat_samples = torch.cat(samples, dim=1)
    n_split = cat_samples.shape[1] // block_size
    return [cat_samples[:, i * block_size:(i + 1) * block_size] for i in range(n_split)]


@torch.no_grad()
def get_calib_feat(model, tokenizer, samples=None, device=None, **dataset_kw):
    """Salient-channel importance features (run_experiments.py:55-84): for every nn.Linear,
    one mean_m |x[m, k]| vector (model dtype, on the CPU) per calibration block.  The
    quantize_* functions sum the list and cast to fp32 (fake_quant.py:396)."""
    input_dict = {}

    def stat_input_max_hook(m, x, y, name):
        if isinstance(x, tuple):
            x = x[0]
        x_max = x.view(-1, x.shape[-1]).abs().mean(dim=0).cpu().detach()
        input_dict.setdefault(name, []).append(x_max)

    if device is None:
        device = torch.device("cuda" if torch.cuda.is_available() else "cpu")
    if samples is None:
        samples = get_calib_dataset(tokenizer, **dataset_kw)
    hooks = _linear_hooks(model, stat_input_max_hook)
    try:
        for input_ids in _tqdm(samples):
            model(input_ids.to(device))
    finally:
        for h in hooks:
            h.remove()
    return input_dict


__all__ = ["get_act_scales", "get_static_decoder_layer_scales", "get_calib_dataset",
           "get_calib_feat"]
