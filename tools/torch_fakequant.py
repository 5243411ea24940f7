"""GPU reference point: the reference's fake-quant forward restated in
plain PyTorch ops, run through PyTorch-ROCm on the same MI355X.  Benchmark-only: it is
what the reference's W4A4Linear.forward costs on this GPU (the reference itself cannot
travel to the box), never part of the product path.

Follows /root/reference/smoothquant/fake_quant.py:
  forward              :279-322 (salient mask, q_x = x.clone(), q_x[:, ~S] = act_quant(A),
                                 F.linear with the stored dequantized weight)
  per_group (sorted)   :104-154 (batch column absmax, argsort, pad to G, per-(row, group)
                                 scales, round, unsort)
  per_token            :56-64
"""
import torch
import torch.nn.functional as F


@torch.no_grad()
def act_per_token(t, n_bits):
    q_max = 2 ** (n_bits - 1) - 1
    s = t.abs().max(dim=-1, keepdim=True)[0].clamp(min=1e-5).div(q_max)
    return t.div(s).round().mul(s)


@torch.no_grad()
def act_per_group_sorted(t, n_bits, group_size):
    q_max = 2 ** (n_bits - 1) - 1
    M, C = t.shape
    idx = torch.argsort(t.abs().max(dim=0)[0], stable=True)
    ts = t[:, idx]
    pad = (-C) % group_size
    if pad:
        ts = torch.cat([ts, ts.new_zeros(M, pad)], dim=1)
    g = ts.view(M, -1, group_size)
    s = g.abs().amax(dim=-1, keepdim=True).clamp(min=1e-5).div(q_max)
    g = g.div(s).round().mul(s)
    ts = g.view(M, -1)[:, :C]
    out = torch.empty_like(t)
    out[:, idx] = ts
    return out


class TorchFakeQuantLinear:
    """The reference forward on given W_hat (dequantized weight), bias, salient set."""

    def __init__(self, w_hat, bias, salient, act_quant="per_group", n_bits=4, group_size=128):
        self.w = w_hat
        self.b = bias
        K = w_hat.shape[1]
        self.mask = None
        if salient is not None:
            self.mask = torch.ones(K, dtype=torch.bool, device=w_hat.device)
            self.mask[salient.to(w_hat.device)] = False
        self.act = act_quant
        self.n_bits = n_bits
        self.G = group_size

    def _aq(self, t):
        if self.act == "per_group":
            return act_per_group_sorted(t, self.n_bits, self.G)
        return act_per_token(t, self.n_bits)

    @torch.no_grad()
    def __call__(self, x):
        x2 = x.reshape(-1, x.shape[-1])
        if self.mask is not None:
            q_x = x2.clone()
            q_x[:, self.mask] = self._aq(x2[:, self.mask])
        else:
            q_x = self._aq(x2)
        y = F.linear(q_x, self.w, self.b)
        return y.view(*x.shape[:-1], -1)
