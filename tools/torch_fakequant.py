"""GPU reference point: the reference's fake-quant forward restated in
plain PyTorch ops, run through PyTorch-ROCm on the same MI355X.  Benchmark-only: it is
what the reference's W4A4Linear.forward costs on this GPU (the reference itself cannot
travel to the box), never part of the product path.

Follows /root/reference/smoothquant/fake_quant.py:
  forward              :279-322 (salient mask, q_x = x.clone(), q_x[:, ~S] = act_quant(A),
                                 F.linear with the stored dequantized weight)
  per_group (sorted)   :104-154 (batch column absmax, argsort, pad to G, per-(row, group)
                                 scales, round, unsort)
  per_token / tensor   :56-75
  output quantization  :308-316 (OPT q/k/v with quantize_bmm_input)
plus the config-5 variants (unsorted groups :77-101, the mean+3sigma sort key).
`accum32` runs F.linear at a higher precision than the model's -- fp32 copies for fp16 / bf16
models, fp64 for fp32 models -- : the same fake-quant math with another GEMM accumulation
(the noise floor of PPL comparisons).
"""
import torch
import torch.nn.functional as F


@torch.no_grad()
def act_per_token(t, n_bits):
    q_max = 2 ** (n_bits - 1) - 1
    s = t.abs().max(dim=-1, keepdim=True)[0].clamp(min=1e-5).div(q_max)
    return t.div(s).round().mul(s)


@torch.no_grad()
def act_per_tensor(t, n_bits):
    q_max = 2 ** (n_bits - 1) - 1
    s = t.abs().max().clamp(min=1e-5).div(q_max)
    return t.div(s).round().mul(s)


def _mean3std(t):
    a = t.abs().double()
    mean = a.mean(0)
    var = ((a * a).mean(0) - mean * mean).clamp(min=0)
    return (mean + 3 * var.sqrt()).float()


@torch.no_grad()
def act_per_group_sorted(t, n_bits, group_size, key="max"):
    q_max = 2 ** (n_bits - 1) - 1
    M, C = t.shape
    if key == "none":
        idx = torch.arange(C, device=t.device)
    elif key == "mean3std":
        idx = torch.argsort(_mean3std(t), stable=True)
    else:
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

    def __init__(self, w_hat, bias, salient, act_quant="per_group", n_bits=4, group_size=128,
                 accum32=False, output_quant=None):
        self.w = w_hat
        self.accum32 = accum32
        self.out_spec = output_quant  # (mode, bits, group) or None
        self.b = bias
        K = w_hat.shape[1]
        self.mask = None
        if salient is not None:
            self.mask = torch.ones(K, dtype=torch.bool, device=w_hat.device)
            self.mask[salient.to(w_hat.device)] = False
        self.act = act_quant
        self.n_bits = n_bits
        self.G = group_size

    @staticmethod
    def _quant(t, mode, bits, G):
        if mode == "per_group":
            return act_per_group_sorted(t, bits, G)
        if mode == "per_group_unsorted":
            return act_per_group_sorted(t, bits, G, "none")
        if mode == "per_group_mean3std":
            return act_per_group_sorted(t, bits, G, "mean3std")
        if mode == "per_tensor":
            return act_per_tensor(t, bits)
        return act_per_token(t, bits)

    def _aq(self, t):
        return self._quant(t, self.act, self.n_bits, self.G)

    @torch.no_grad()
    def __call__(self, x):
        x2 = x.reshape(-1, x.shape[-1])
        if self.mask is not None:
            q_x = x2.clone()
            q_x[:, self.mask] = self._aq(x2[:, self.mask])
        else:
            q_x = self._aq(x2)
        if self.accum32:
            hi = torch.float64 if q_x.dtype == torch.float32 else torch.float32
            y = F.linear(q_x.to(hi), self.w.to(hi),
                         None if self.b is None else self.b.to(hi)).to(q_x.dtype)
        else:
            y = F.linear(q_x, self.w, self.b)
        if self.out_spec is not None:
            mode, bits, G = self.out_spec
            if self.mask is not None:
                y = y.clone()
                y[:, self.mask] = self._quant(y[:, self.mask], mode, bits, G)
            else:
                y = self._quant(y, mode, bits, G)
        return y.view(*x.shape[:-1], -1)
