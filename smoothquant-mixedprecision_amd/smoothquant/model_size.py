"""Analytic model size (the reference's smoothquant/model_size.py:5-16, same formula).

Non-salient elements cost `data_width + (16 + 4) / group_size` bits and salient ones
`16 + (16 + 4) / group_size`, over every parameter of the model.
"""
import torch.nn as nn


def get_model_size(model: nn.Module, data_width=16, salient_prop=0, group_size=-1):
    width_q = float(data_width)
    width_s = 16.0
    if group_size != -1:
        width_q += (16 + 4) / group_size
        width_s += (16 + 4) / group_size
    avg = width_q * (1 - salient_prop) + width_s * salient_prop
    return sum(p.numel() for p in model.parameters()) * avg
