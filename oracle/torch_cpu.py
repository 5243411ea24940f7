"""TEST INFRASTRUCTURE (CPU baseline + checker) -- never imported by the product path.

A PyTorch-CPU restatement of the reference's fake-quant W4A4 layer, the "reference
PyTorch-CPU fake_quant path" BASELINE.md §3 prices the MI355X operator against: the same
torch ops at the same rounding points as /root/reference/smoothquant/fake_quant.py, run
on the host cores.  `bench.py`'s cpu_baseline leg times it (fp32, all host threads,
median of 3 after 1 warm-up); `tests/test_torch_cpu_golden.py` pins it bit-exact to the
reference-generated goldens (tests/golden/fake_quant_golden.npz), so the baseline is the
reference's computation, not an approximation of it.

Reference map (fake_quant.py):
  _absmax_fq              the shared `s = absmax.clamp(1e-5) / q_max; t/s -> round -> *s`
                          of :9-26, :56-75, :137-142, :188-193
  group_fq                per-group quantizer over a column order (sorted :104-154 /
                          :156-207, unsorted :29-53 / :77-101), zero padding to G
  quantize_weight         from_float's weight step :347-365 (salient columns restored)
  forward                 :279-322 (salient mask, act quant, F.linear, output quant)
Ties in the column sort use a STABLE argsort (the fixtures' rule).
"""
from __future__ import annotations

from typing import Optional

import torch
import torch.nn.functional as F


def _qmax(n_bits: int) -> int:
    return 2 ** (n_bits - 1) - 1


def _absmax_fq(t: torch.Tensor, amax: torch.Tensor, n_bits: int) -> torch.Tensor:
    s = amax.clamp(min=1e-5).div(_qmax(n_bits))
    return t.div(s).round().mul(s)


def group_fq(t: torch.Tensor, n_bits: int, group_size: int, sort: bool) -> torch.Tensor:
    """Per-(row, group) fake quantization of t [R, C]; groups of `group_size` consecutive
    columns in ascending column-absmax order (sort=True) or natural order."""
    R, C = t.shape
    order = (torch.argsort(t.abs().amax(dim=0), stable=True) if sort
             else torch.arange(C, device=t.device))
    pad = (-C) % group_size
    ts = F.pad(t[:, order], (0, pad))
    g = ts.view(R, -1, group_size)
    q = _absmax_fq(g, g.abs().amax(dim=-1, keepdim=True), n_bits).view(R, -1)[:, :C]
    out = torch.empty_like(t)
    out[:, order] = q
    return out


def act_quant(t2: torch.Tensor, mode: str, n_bits: int, group_size: int) -> torch.Tensor:
    """The bound act_quant of W4A4Linear (fake_quant.py:246-256) on a 2-D tensor."""
    if mode == "per_token":
        return _absmax_fq(t2, t2.abs().amax(dim=-1, keepdim=True), n_bits)
    if mode == "per_tensor":
        return _absmax_fq(t2, t2.abs().amax(), n_bits)
    if mode == "per_group":
        return group_fq(t2, n_bits, group_size, sort=True)
    if mode == "per_group_unsorted":
        return group_fq(t2, n_bits, group_size, sort=False)
    raise ValueError(f"Invalid act_quant: {mode}")


def select_salient(importance: Optional[torch.Tensor], salient_prop: float):
    """fake_quant.py:265-270 (descending importance, stable ties)."""
    if importance is None or not salient_prop > 0:
        return None
    order = torch.argsort(importance, descending=True, stable=True)
    return order[:max(1, int(salient_prop * len(order)))]


def quantize_weight(w: torch.Tensor, weight_quant: str, n_bits: int, group_size: int,
                    salient: Optional[torch.Tensor]) -> torch.Tensor:
    """W_hat of from_float (fake_quant.py:347-365): a new tensor, salient columns exact."""
    if weight_quant == "per_channel":
        w_hat = _absmax_fq(w, w.abs().amax(dim=-1, keepdim=True), n_bits)
    elif weight_quant == "per_tensor":
        w_hat = _absmax_fq(w, w.abs().amax(), n_bits)
    elif weight_quant == "per_group":
        w_hat = group_fq(w, n_bits, group_size, sort=True)
    elif weight_quant == "per_group_unsorted":
        w_hat = group_fq(w, n_bits, group_size, sort=False)
    else:
        raise ValueError(f"Invalid weight_quant: {weight_quant}")
    if salient is not None:
        w_hat[:, salient] = w[:, salient]
    return w_hat


class CPUFakeQuantLinear:
    """The reference layer on the host: construct from W [N, K] (+ bias) once, call on x."""

    def __init__(self, w, bias, weight_quant="per_group", act_mode="per_group", n_bits=4,
                 group_size=128, importance=None, salient_prop=0.0, quantize_output=False):
        self.salient = select_salient(importance, salient_prop)
        self.w_hat = quantize_weight(w, weight_quant, n_bits, group_size, self.salient)
        self.bias = bias
        self.mode, self.n_bits, self.G = act_mode, n_bits, group_size
        self.quantize_output = quantize_output
        self.keep = None
        if self.salient is not None:
            self.keep = torch.ones(w.shape[1], dtype=torch.bool)
            self.keep[self.salient] = False

    def quantize_input(self, x2: torch.Tensor) -> torch.Tensor:
        """q_x of fake_quant.py:291-304 (a new tensor; the caller's x is left alone)."""
        if self.keep is None:
            return act_quant(x2.clone(), self.mode, self.n_bits, self.G)
        q_x = x2.clone()
        if bool(self.keep.any()):
            q_x[:, self.keep] = act_quant(x2[:, self.keep], self.mode, self.n_bits, self.G)
        return q_x

    @torch.no_grad()
    def __call__(self, x: torch.Tensor) -> torch.Tensor:
        x2 = x.reshape(-1, x.shape[-1])
        y = F.linear(self.quantize_input(x2), self.w_hat, self.bias)
        if self.quantize_output:
            if self.keep is not None:
                y[:, self.keep] = act_quant(y[:, self.keep], self.mode, self.n_bits, self.G)
            else:
                y = act_quant(y, self.mode, self.n_bits, self.G)
        return y.view(*x.shape[:-1], -1)
