"""Exact IEEE binary32 helpers in numpy — TEST INFRASTRUCTURE ONLY.

The HIP kernels contract the basis with the weights as a k-ordered chain of single-rounding
f32 FMAs (``v_fma_f32`` on the VALU, and the f32-input MFMA, which cdna_hip_programming.md §3
documents as bit-for-bit the same k-ordered ``fmaf`` chain).  numpy has no fma, so
``fma32`` emulates it exactly: a*b is exact in f64 for f32 inputs, ``two_sum`` gives the f64
sum s and its exact error e, and rounding s to f32 differs from rounding the exact value s+e
only when s sits exactly on an f32 midpoint (then the sign of e decides).
"""
import numpy as np

f32 = np.float32
f64 = np.float64


def _two_sum(a, b):
    s = a + b
    bb = s - a
    return s, (a - (s - bb)) + (b - bb)


def _round_exact(s, e):
    r = s.astype(f32)
    r64 = r.astype(f64)
    below = r64 < s
    above = r64 > s
    lo = np.where(above, np.nextafter(r, f32(-np.inf)), r)
    hi = np.where(below, np.nextafter(r, f32(np.inf)), r)
    mid = (lo.astype(f64) + hi.astype(f64)) * 0.5
    fix = (below | above) & (s == mid) & (e != 0)
    if np.any(fix):
        r = np.where(fix, np.where(e > 0, hi, lo), r)
    return np.asarray(r, dtype=f32)


def fma32(a, b, c):
    """Exact single-rounding f32 fma(a, b, c) for f32 inputs (vectorised)."""
    a = np.asarray(a, dtype=f32).astype(f64)
    b = np.asarray(b, dtype=f32).astype(f64)
    c = np.asarray(c, dtype=f32).astype(f64)
    s, e = _two_sum(a * b, c)          # a*b exact in f64
    return _round_exact(s, e)


def fma_chain32(A, B, c0=None):
    """sum_k A[..., k] * B[..., k] as the k-ordered f32 fma chain starting from c0 (default 0)."""
    A = np.asarray(A, dtype=f32)
    B = np.asarray(B, dtype=f32)
    shape = np.broadcast_shapes(A.shape[:-1], B.shape[:-1])
    acc = np.zeros(shape, f32) if c0 is None else np.broadcast_to(np.asarray(c0, f32), shape).copy()
    for k in range(A.shape[-1]):
        acc = fma32(A[..., k], B[..., k], acc)
    return acc
