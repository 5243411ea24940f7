"""Quantized-model checkpoints (persistent packed format).

    save_quantized(model, path)      torch.save of {"format", "state_dict"}; every W4A4Linear
                                     contributes its packed buffers + `_extra_state`
    load_quantized(model, path)      replaces the nn.Linear modules named in the checkpoint
                                     with W4A4Linear and loads the packed state (no
                                     calibration, no re-packing); safe loader only

The reference has no such format: its quantized models exist only in memory (weights
stored dequantized, salient_indices not in state_dict).
"""
import torch
import torch.nn as nn

from .fake_quant import W4A4Linear

FORMAT = "sqmp-w4a4-model/1"


def save_quantized(model: nn.Module, path: str) -> None:
    torch.save({"format": FORMAT, "state_dict": model.state_dict()}, path)


def _swap_in(model: nn.Module, name: str, extra: dict) -> None:
    parent_name, _, attr = name.rpartition(".")
    parent = model.get_submodule(parent_name) if parent_name else model
    old = getattr(parent, attr)
    if isinstance(old, W4A4Linear):
        return
    if not isinstance(old, nn.Linear):
        raise RuntimeError(f"{name}: expected nn.Linear or W4A4Linear, found {type(old).__name__}")
    new = W4A4Linear(extra["in_features"], extra["out_features"], old.bias is not None,
                     act_quant=extra["act_quant"],
                     quantize_output=extra["output_quant"] != "None",
                     quant_bits=extra["quant_bits"], group_size=extra["group_size"])
    setattr(parent, attr, new)


def load_quantized(model: nn.Module, path: str, map_location=None, strict: bool = True) -> nn.Module:
    ckpt = torch.load(path, map_location=map_location, weights_only=True)
    if not isinstance(ckpt, dict) or ckpt.get("format") != FORMAT:
        raise RuntimeError(f"{path}: not a {FORMAT} checkpoint")
    sd = ckpt["state_dict"]
    for key, val in sd.items():
        if key.endswith("._extra_state") and isinstance(val, dict) and \
                val.get("format") == W4A4Linear.EXTRA_FORMAT:
            _swap_in(model, key[: -len("._extra_state")], val)
    model.load_state_dict(sd, strict=strict)
    return model


__all__ = ["save_quantized", "load_quantized", "FORMAT"]
