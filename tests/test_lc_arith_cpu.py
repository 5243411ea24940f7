"""Exhaustive proof (CPU, numpy) of the division-free scale arithmetic of the lane-contiguous
quantizer (csrc/sqmp_actquant_lc.hip, pair_scale / nib_pair):

  * s32 = fl32(a / q) as  q0 = a * rq,  e = fma(-q0, q, a),  s32 = fma(e, rq, q0)
    with rq = fl32(1 / q)   (Markstein) -- equal to the IEEE quotient for every D value a
    the scale can see (D = fp16: all of them from the 1e-5 clamp up; bf16: up to 2^100)
    and every q_max = 2^(b-1) - 1, b = 2 .. 8;
  * r = fl32(1 / s) as  e = fma(-s, y0, 1),  r = fma(e, y0, y0)  for EVERY y0 within one
    ulp of 1 / s (v_rcp_f32's bound), for every D scale s that can occur;
  * the 4-bit code as the low byte of D(q) + 1544 (fp16) / fl32(D(q) + 2^23 + 8) (bf16):
    code + 8 for every D value q that rounds to a code in [-8, 7] (bf16: |q| <= 7.5, as
    |x| <= absmax keeps |x / s| under 7.03 at q_max = 7).

fma is emulated exactly: every product below is exact in fp64, and the one sum that is not
is re-done in exact rationals whenever its fp64 value sits on an fp32 rounding midpoint
(the only case where rounding twice differs from rounding once).  The reference quotient
is numpy's correctly rounded fp32 division, as PyTorch's D(D(x) / q_max) computes it
(/root/reference/smoothquant/fake_quant.py:139-142)."""
from fractions import Fraction

import numpy as np

F32 = np.float32


def _rn32_exact(x: Fraction) -> np.float32:
    # round an exact rational to the nearest fp32 (normal range), ties to even
    if x == 0:
        return F32(0.0)
    sign = -1 if x < 0 else 1
    x = abs(x)
    e = x.numerator.bit_length() - x.denominator.bit_length()
    if Fraction(2) ** e > x:
        e -= 1
    scaled = x * Fraction(2) ** (23 - e)  # in [2^23, 2^24)
    n = scaled.numerator // scaled.denominator
    rem = scaled - n
    if rem > Fraction(1, 2) or (rem == Fraction(1, 2) and n % 2 == 1):
        n += 1
    return F32(sign * float(Fraction(n) * Fraction(2) ** (e - 23)))


def _fma_sum(p64: np.ndarray, a: np.ndarray, b: np.ndarray, c: np.ndarray) -> np.ndarray:
    """RN32(a * b + c) given p64 = a * b exact in fp64; exact fallback on fp32 midpoints."""
    v64 = p64 + c.astype(np.float64)
    r = v64.astype(F32)
    # a midpoint of two fp32 neighbours: v64 halfway between r and its neighbour
    lo = np.nextafter(r, F32(-np.inf)).astype(np.float64)
    hi = np.nextafter(r, F32(np.inf)).astype(np.float64)
    r64 = r.astype(np.float64)
    mid = (v64 == (r64 + lo) / 2) | (v64 == (r64 + hi) / 2)
    for i in np.nonzero(mid)[0]:
        r[i] = _rn32_exact(Fraction(float(a[i])) * Fraction(float(b[i])) + Fraction(float(c[i])))
    return r


def _fma(a, b, c):
    # a * b exact in fp64 for the operand widths used here (<= 24 + 24 bits)
    return _fma_sum(a.astype(np.float64) * b.astype(np.float64), a, b, c)


def _d_values(dtype):
    if dtype == "fp16":
        bits = np.arange(0, 0x7C00, dtype=np.uint16)  # +0 .. max finite
        v = bits.view(np.float16).astype(F32)
    else:
        bits = np.arange(0, 0x7F80, dtype=np.uint32)
        v = (bits << 16).astype(np.uint32).view(F32)
        v = v[v < F32(2.0 ** 100)]
    return v


def _rd(v, dtype):
    if dtype == "fp16":
        return v.astype(np.float16).astype(F32)
    b = v.view(np.uint32).astype(np.uint64)
    b = (b + 0x7FFF + ((b >> 16) & 1)) >> 16 << 16  # RNE to bf16 (finite values)
    return b.astype(np.uint32).view(F32)


def test_markstein_scale_division_exhaustive():
    for dtype in ("fp16", "bf16"):
        lo = _rd(np.array([1e-5], F32), dtype)[0]
        a = _d_values(dtype)
        a = a[a >= lo]
        for b in range(2, 9):
            qm = F32(2 ** (b - 1) - 1)
            rq = F32(1.0) / qm
            q = np.full_like(a, qm)
            rqv = np.full_like(a, rq)
            q0 = (a * rq).astype(F32)
            e = _fma(-q0, q, a)
            s32 = _fma(e, rqv, q0)
            ref = a / qm
            bad = np.nonzero(s32 != ref)[0]
            assert bad.size == 0, (dtype, b, a[bad[:4]], s32[bad[:4]], ref[bad[:4]])


def test_newton_reciprocal_exhaustive():
    for dtype in ("fp16", "bf16"):
        lo = _rd(np.array([1e-5], F32), dtype)[0]
        s = np.unique(np.concatenate([_rd(_d_values(dtype)[_d_values(dtype) >= lo] / F32(q), dtype)
                                      for q in (1, 3, 7, 15, 31, 63, 127)]))
        s = s[s > 0]
        ref = F32(1.0) / s
        one = np.ones_like(s)
        for y0 in (np.nextafter(ref, F32(0)), ref, np.nextafter(ref, F32(np.inf))):
            y0 = y0.astype(F32)
            e = _fma(-s, y0, one)
            r = _fma(e, y0, y0)
            bad = np.nonzero(r != ref)[0]
            assert bad.size == 0, (dtype, s[bad[:4]], r[bad[:4]], ref[bad[:4]])


def test_magic_code_bytes():
    # fp16: every D value that rounds (half-even) to a code in [-8, 7]
    d = np.arange(0, 0x10000, dtype=np.uint32).astype(np.uint16).view(np.float16)
    d = d[np.isfinite(d)]
    code = np.rint(d.astype(np.float64))
    d, code = d[(code >= -8) & (code <= 7)], code[(code >= -8) & (code <= 7)]
    m = (d + np.float16(1544)).view(np.uint16)
    assert np.array_equal(m & 0xFF, (code + 8).astype(np.uint16))
    assert np.all((m >> 8) == 0x66)
    # bf16: the same through fp32 with 2^23 + 8
    b = (np.arange(0, 0x10000, dtype=np.uint32) << 16).astype(np.uint32).view(F32)
    b = b[np.isfinite(b)]
    code = np.rint(b.astype(np.float64))
    keep = np.abs(b) <= 7.5
    b, code = b[keep], code[keep]
    m = (b + F32(8388616.0)).view(np.uint32)
    assert np.array_equal(m & 0xFF, (code + 8).astype(np.uint32))
