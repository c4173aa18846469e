"""Correctly rounded fused multiply-add on torch tensors, without an FMA op.

The native backends evaluate the FTCS update of heat3D.cu:128-131 the way
nvcc compiles the reference kernel (every ``acc + D*a`` one fused
multiply-add, csrc/kernels/kernels.hpp ``ftcs_update``).  Eager PyTorch has
no fused multiply-add that is guaranteed to round once, so the test oracles
emulate it with error-free transformations:

* fp64: Dekker's TwoProduct gives ``a*b = p + e`` exactly, Knuth's TwoSum
  ``p + c = s + t`` exactly, so ``a*b + c = s + (t + e)``; the small part is
  summed with round-to-odd (``u = RN(t + e)``, sticky bit from its exact
  error) and one round-to-nearest add finishes — round-to-odd followed by
  round-to-nearest into a narrower-or-equal format is the Boldo–Melquiond
  construction for correctly rounded sums.
* fp32: ``a*b`` is exact in fp64; ``s = RN64(a*b + c)`` plus its TwoSum error
  rounded to odd in fp64 (53 >= 24 + 2 bits) then rounded to fp32.

Every op used here is one IEEE operation with one rounding, so the results
match ``fma()`` on the CPU and ``v_fma_f64``/``v_fma_f32`` on gfx950 bitwise
for finite operands without overflow (the stencil's range).
"""
from __future__ import annotations

import torch

_SPLIT = 134217729.0  # 2^27 + 1 (Veltkamp split of a 53-bit significand)


def _two_sum(a, b):
    s = a + b
    bb = s - a
    err = (a - (s - bb)) + (b - bb)
    return s, err


def _split(a):
    c = _SPLIT * a
    hi = c - (c - a)
    return hi, a - hi


def _two_prod(a, b):
    p = a * b
    ah, al = _split(a)
    bh, bl = _split(b)
    err = ((ah * bh - p) + ah * bl + al * bh) + al * bl
    return p, err


def _round_to_odd(u, v):
    """RO(u + v) for u = RN(u + v) and its exact error v (float64)."""
    bits = u.view(torch.int64)
    toward_zero = (v != 0) & ((v < 0) != (u < 0))
    # truncation toward zero of u + v: u itself, or u's neighbour toward zero
    trunc = torch.where(toward_zero & (u != 0), bits - 1, bits)
    odd = torch.where(v != 0, trunc | 1, trunc)
    return odd.view(torch.float64)


def fma(a, b, c) -> torch.Tensor:
    """round(a * b + c) elementwise (float64 or float32 tensors / scalars)."""
    ref = next(x for x in (a, b, c) if isinstance(x, torch.Tensor))
    dt = ref.dtype

    def t64(x):
        # python scalars take the tensor dtype first (as in torch's own binary ops)
        x = x if isinstance(x, torch.Tensor) else torch.tensor(float(x), dtype=dt)
        return x.to(torch.float64)

    a64, b64, c64 = t64(a), t64(b), t64(c)
    if dt == torch.float32:
        p = a64 * b64                       # exact: 24 + 24 bits
        s, t = _two_sum(p, c64)             # p + c = s + t exactly
        return _round_to_odd(s, t).to(torch.float32)
    if dt != torch.float64:
        raise TypeError(f"fma: unsupported dtype {dt}")
    p, e = _two_prod(a64, b64)
    s, t = _two_sum(p, c64)
    u, v = _two_sum(t, e)                   # t + e = u + v exactly
    return s + _round_to_odd(u, v)


def ftcs_update(c, xm, xp, ym, yp, zm, zp, D):
    """FTCS update in the native backends' arithmetic (kernels.hpp ftcs_update)."""
    ax = fma(-2.0, c, xp) + xm
    ay = fma(-2.0, c, yp) + ym
    az = fma(-2.0, c, zp) + zm
    return fma(D[2], az, fma(D[1], ay, fma(D[0], ax, c)))
