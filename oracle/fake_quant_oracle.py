"""CPU ORACLE for the W4A4 mixed-precision linear -- TEST INFRASTRUCTURE ONLY.

This module restates, in numpy, the numerics of the reference's fake-quant path
(`/root/reference/smoothquant/fake_quant.py`, adithyab100/smoothquant-mixedprecision
@ 2024-12-20).  It is the *checker*: only `tests/`, `__graft_entry__.smoke()` and
`bench.py`'s `cpu_baseline` leg may import it.  The product path
(`smoothquant-mixedprecision_amd/smoothquant`) never calls it and fails loudly when the
HIP library is missing.

Parity status: PINNED.  `tests/golden/*.npz` were produced by running the reference
itself in the survey container (`tests/golden/gen_golden.py`, which loads
`fake_quant.py` by file path with the sort pinned to `stable=True`, see below), and
`tests/test_oracle_golden.py` checks every function here against them bit-exactly.

Numerics contract (what "bit-exact" means):
  * D is the model dtype (fp32, fp16 or bf16).  Every elementwise op is computed in fp32
    and rounded to D, exactly as PyTorch's CPU kernels do for reduced float types
    (opmath = float).  bf16 values are held in float32 arrays and rounded with RNE.
  * round() is round-half-to-even (torch.round_ / np.rint).
  * argsort ties: the reference calls `torch.argsort(col_max)` (unstable).  We pin the
    STABLE ascending order (ties -> lower column index first); fixtures were generated
    with the same pin.  In fp32 with continuous data the two agree.
  * F.linear (fake_quant.py:306) is restated as an fp64 accumulation of the exact
    products of the dequantized operands, plus bias, rounded once to D.  Any fp32-
    accumulating GEMM (cuBLAS, MKL, our MFMA kernels) differs from it only by
    accumulation order; tests state that tolerance explicitly.
"""
from __future__ import annotations

import numpy as np

__all__ = [
    "DT", "quantize_weight_per_channel_absmax", "quantize_weight_per_tensor_absmax",
    "quantize_weight_per_group_absmax", "quantize_activation_per_token_absmax",
    "quantize_activation_per_tensor_absmax", "quantize_activation_per_group_absmax",
    "quantize_activation_per_group_absmax_sort", "quantize_weight_per_group_absmax_sort",
    "select_salient", "w4a4_from_float", "w4a4_forward", "linear", "act_quant_fn",
    "weight_quant_fn", "mean3std_key", "quantize_activation_per_group_mean3std_sort",
    "quantize_weight_per_group_mean3std_sort",
]


# --------------------------------------------------------------------------------------
# dtype emulation
# --------------------------------------------------------------------------------------
def _bf16_round(a32: np.ndarray) -> np.ndarray:
    """Round float32 values to the nearest bf16 (RNE), returned as float32."""
    a32 = np.ascontiguousarray(a32, dtype=np.float32)
    u = a32.view(np.uint32).astype(np.uint64)
    r = ((u + 0x7FFF + ((u >> 16) & 1)) >> 16) << 16
    return (r & 0xFFFFFFFF).astype(np.uint32).view(np.float32).reshape(a32.shape)


class DT:
    """Storage dtype D.  `rnd` rounds an fp32 array to D; `f32` widens D to fp32."""

    def __init__(self, name: str):
        if name not in ("fp32", "fp16", "bf16"):
            raise ValueError(name)
        self.name = name

    def rnd(self, a) -> np.ndarray:
        a = np.asarray(a, dtype=np.float32)
        if self.name == "fp32":
            return a.copy()
        if self.name == "fp16":
            return a.astype(np.float16)
        return _bf16_round(a)

    @staticmethod
    def f32(a) -> np.ndarray:
        return np.asarray(a).astype(np.float32)

    def clamp_min(self, a, lo: float) -> np.ndarray:
        """`t.clamp_(min=lo)` on a D tensor (fake_quant.py:14 etc.)."""
        return self.rnd(np.maximum(self.f32(a), np.float32(lo)))

    def __repr__(self):
        return f"DT({self.name})"


def _scales(absmax, q_max: int, dt: DT):
    """`scales.clamp_(min=1e-5).div_(q_max)` in D (e.g. fake_quant.py:14, 139, 190)."""
    c = dt.clamp_min(absmax, 1e-5)
    return dt.rnd(dt.f32(c) / np.float32(q_max))


def _fq(t, s, dt: DT):
    """`t.div_(s).round_().mul_(s)` in D (e.g. fake_quant.py:15, 142, 193).

    Returns (dequantized values in D, integer codes as int32)."""
    q = dt.rnd(dt.f32(t) / dt.f32(s))
    code = np.rint(dt.f32(q))
    return dt.rnd(code.astype(np.float32) * dt.f32(s)), code.astype(np.int32)


def _qmax(n_bits: int) -> int:
    return 2 ** (n_bits - 1) - 1


# --------------------------------------------------------------------------------------
# quantizer primitives (fake_quant.py:9-207)
# --------------------------------------------------------------------------------------
def quantize_weight_per_channel_absmax(w, n_bits, dt: DT):
    """fake_quant.py:9-16 -- one scale per output row."""
    s = _scales(np.abs(w).max(axis=-1, keepdims=True), _qmax(n_bits), dt)
    return _fq(w, s, dt)[0]


def quantize_weight_per_tensor_absmax(w, n_bits, dt: DT):
    """fake_quant.py:19-26 -- one scale for the whole matrix."""
    s = _scales(np.abs(w).max(), _qmax(n_bits), dt)
    return _fq(w, s, dt)[0]


def _group_quant_rows(t, n_bits, group_size, dt: DT):
    """Pad columns with zeros to a multiple of group_size, quantize each
    (row, group), drop the padding (fake_quant.py:32-53 / 123-147 / 175-199)."""
    R, C = t.shape
    ng = (C + group_size - 1) // group_size
    pad = ng * group_size - C
    tp = np.concatenate([t, np.zeros((R, pad), dtype=t.dtype)], axis=1) if pad else t
    tg = tp.reshape(R, ng, group_size)
    s = _scales(np.abs(tg).max(axis=-1, keepdims=True), _qmax(n_bits), dt)
    deq, code = _fq(tg, s, dt)
    return (deq.reshape(R, -1)[:, :C], code.reshape(R, -1)[:, :C], s[..., 0])


def quantize_weight_per_group_absmax(w, n_bits, dt: DT, group_size=128):
    """fake_quant.py:29-53 -- unsorted groups (not wired into W4A4Linear)."""
    return _group_quant_rows(w, n_bits, group_size, dt)[0]


def quantize_activation_per_token_absmax(t, n_bits, dt: DT):
    """fake_quant.py:56-64 -- one scale per token row (returns 2-D like the reference)."""
    t2 = t.reshape(-1, t.shape[-1])
    s = _scales(np.abs(t2).max(axis=-1, keepdims=True), _qmax(n_bits), dt)
    return _fq(t2, s, dt)[0]


def quantize_activation_per_tensor_absmax(t, n_bits, dt: DT):
    """fake_quant.py:67-75 -- one scale for the whole batch (returns 2-D)."""
    t2 = t.reshape(-1, t.shape[-1])
    s = _scales(np.abs(t2).max(), _qmax(n_bits), dt)
    return _fq(t2, s, dt)[0]


def quantize_activation_per_group_absmax(t, n_bits, dt: DT, group_size=128):
    """fake_quant.py:77-101 -- unsorted per-row groups."""
    t2 = t.reshape(-1, t.shape[-1])
    return _group_quant_rows(t2, n_bits, group_size, dt)[0].reshape(t.shape)


def stable_argsort(keys) -> np.ndarray:
    """Ascending argsort, ties -> lower index first (the pinned torch.argsort rule)."""
    return np.argsort(np.asarray(keys, dtype=np.float64), kind="stable")


def mean3std_key(t2, dt: DT):
    """The mean + 3 sigma column key (README.md:36 "statistical sorting"; absent from the
    reference's code, so defined here -- PARITY UNPINNED): mean|x| + 3 std|x| over the
    rows (population std) from fp64 sums of |x| and x^2, rounded once to fp32.  The HIP
    key kernel (sqmp_stats.hip) computes the same formula with the same rounding points."""
    a = np.abs(dt.f32(t2)).astype(np.float64)
    R = a.shape[0]
    mean = a.sum(axis=0) / R
    var = np.maximum((a * a).sum(axis=0) / R - mean * mean, 0.0)
    return (mean + 3.0 * np.sqrt(var)).astype(np.float32)


def _sorted_group_quant(t2, n_bits, group_size, dt: DT, key: str = "max"):
    """Shared body of fake_quant.py:104-154 and :156-207: sort columns ascending by
    column absmax, group, quantize, unsort.  Returns (dequant, codes, scales, perm).
    key="mean3std" sorts by mean3std_key instead (the config-5 extension)."""
    if key == "mean3std":
        col_max = mean3std_key(t2, dt)
    else:
        col_max = np.abs(t2).max(axis=0)                # :113 / :164
    perm = stable_argsort(dt.f32(col_max))              # :116 / :167
    deq, code, s = _group_quant_rows(t2[:, perm], n_bits, group_size, dt)
    inv = np.argsort(perm, kind="stable")               # :150 / :204
    return deq[:, inv], code[:, inv], s, perm


def quantize_activation_per_group_absmax_sort(t, n_bits, dt: DT, group_size=128):
    """fake_quant.py:104-154 -- groups over columns sorted by the batch's column absmax."""
    t2 = t.reshape(-1, t.shape[-1])
    return _sorted_group_quant(t2, n_bits, group_size, dt)[0].reshape(t.shape)


def quantize_weight_per_group_absmax_sort(w, n_bits, dt: DT, group_size=128):
    """fake_quant.py:156-207 -- groups over columns sorted by the weight column absmax."""
    return _sorted_group_quant(w, n_bits, group_size, dt)[0]


def quantize_activation_per_group_mean3std_sort(t, n_bits, dt: DT, group_size=128):
    """Config-5 extension: :104-154 with the mean3std_key sort (parity unpinned)."""
    t2 = t.reshape(-1, t.shape[-1])
    return _sorted_group_quant(t2, n_bits, group_size, dt, "mean3std")[0].reshape(t.shape)


def quantize_weight_per_group_mean3std_sort(w, n_bits, dt: DT, group_size=128):
    """Config-5 extension: :156-207 with the mean3std_key sort (parity unpinned)."""
    return _sorted_group_quant(w, n_bits, group_size, dt, "mean3std")[0]


def act_quant_fn(name: str, n_bits: int, group_size: int, dt: DT):
    """The `act_quant` binding of W4A4Linear.__init__ (fake_quant.py:246-256), plus the
    config-5 rebindings: "per_group_unsorted" = :77-101, "per_group_mean3std"."""
    if name == "per_token":
        return lambda t: quantize_activation_per_token_absmax(t, n_bits, dt)
    if name == "per_tensor":
        return lambda t: quantize_activation_per_tensor_absmax(t, n_bits, dt)
    if name == "per_group":
        return lambda t: quantize_activation_per_group_absmax_sort(t, n_bits, dt, group_size)
    if name == "per_group_unsorted":
        return lambda t: quantize_activation_per_group_absmax(t, n_bits, dt, group_size)
    if name == "per_group_mean3std":
        return lambda t: quantize_activation_per_group_mean3std_sort(t, n_bits, dt, group_size)
    raise ValueError(f"Invalid act_quant: {name}")


def weight_quant_fn(name: str, n_bits: int, group_size: int, dt: DT):
    """The weight quantizer choice of from_float (fake_quant.py:348-361), plus the
    config-5 compositions: "per_group_unsorted" = :29-53, "per_group_mean3std"."""
    if name == "per_channel":
        return lambda w: quantize_weight_per_channel_absmax(w, n_bits, dt)
    if name == "per_tensor":
        return lambda w: quantize_weight_per_tensor_absmax(w, n_bits, dt)
    if name == "per_group":
        return lambda w: quantize_weight_per_group_absmax_sort(w, n_bits, dt, group_size)
    if name == "per_group_unsorted":
        return lambda w: quantize_weight_per_group_absmax(w, n_bits, dt, group_size)
    if name == "per_group_mean3std":
        return lambda w: quantize_weight_per_group_mean3std_sort(w, n_bits, dt, group_size)
    raise ValueError(f"Invalid weight_quant: {name}")


# --------------------------------------------------------------------------------------
# W4A4Linear (fake_quant.py:209-374)
# --------------------------------------------------------------------------------------
def select_salient(importance, salient_prop):
    """fake_quant.py:265-270: top max(1, int(p*K)) channels by importance, descending
    (ties -> lower index first, the pinned rule).  None when disabled."""
    if importance is None or not salient_prop or salient_prop <= 0:
        return None
    imp = np.asarray(importance, dtype=np.float64)
    order = np.argsort(-imp, kind="stable")
    n = max(1, int(salient_prop * len(order)))
    return order[:n].astype(np.int64)


def w4a4_from_float(w, weight_quant, n_bits, group_size, salient, dt: DT):
    """fake_quant.py:324-371: quantize W (salient columns included in the scale
    computation), then restore the salient columns to their original values."""
    w = dt.rnd(dt.f32(w))
    outl = w[:, salient].copy() if salient is not None else None   # :347
    wq = weight_quant_fn(weight_quant, n_bits, group_size, dt)(w.copy())
    if salient is not None:
        wq[:, salient] = outl                                       # :363-365
    return wq


def linear(x, w, b, dt: DT):
    """F.linear(q_x, W, b) in D (fake_quant.py:306): fp64 accumulate, one rounding."""
    acc = dt.f32(x).astype(np.float64) @ dt.f32(w).astype(np.float64).T
    if b is not None:
        acc = acc + dt.f32(b).reshape(1, -1).astype(np.float64)
    return dt.rnd(acc.astype(np.float32)) if dt.name != "fp32" else acc.astype(np.float32)


def quantize_input(x2, act_quant, n_bits, group_size, salient, dt: DT):
    """The pre-GEMM half of forward (fake_quant.py:291-304): returns q_x (M,K) in D."""
    aq = act_quant_fn(act_quant, n_bits, group_size, dt)
    if salient is not None:
        mask = np.ones(x2.shape[-1], dtype=bool)
        mask[salient] = False
        q_x = x2.copy()
        a = x2[:, mask]
        if a.size > 0:
            q_x[:, mask] = aq(a)
        return q_x
    return aq(x2.copy())


def w4a4_forward(x, w_hat, bias, act_quant, n_bits, group_size, salient,
                 quantize_output, dt: DT, act_bits=None):
    """fake_quant.py:279-322 (forward) with the weights already fake-quantized.
    act_bits: the activation quantizer's n_bits when it was rebound (W4A8, config 5);
    output quantization keeps the constructor's binding (n_bits), as in the reference."""
    shape = x.shape
    if len(shape) not in (2, 3):
        raise ValueError(f"Unsupported input shape: {shape}")
    K = shape[-1]
    x2 = dt.rnd(dt.f32(x.reshape(-1, K)))
    q_x = quantize_input(x2, act_quant, n_bits if act_bits is None else act_bits, group_size,
                         salient, dt)
    y = linear(q_x, w_hat, bias, dt)
    if quantize_output and salient is not None:
        mask = np.ones(K, dtype=bool)
        mask[salient] = False
        if mask.shape[0] != y.shape[1]:
            raise IndexError("output quantization with salient channels needs N == K")
        q_y = y.copy()
        if mask.any():
            ys = y[:, mask]
            if ys.size > 0:
                q_y[:, mask] = act_quant_fn(act_quant, n_bits, group_size, dt)(ys)
    elif quantize_output:
        q_y = act_quant_fn(act_quant, n_bits, group_size, dt)(y.copy())
    else:
        q_y = y
    if len(shape) == 3:
        return q_y.reshape(shape[0], shape[1], -1)
    return q_y
