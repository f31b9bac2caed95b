"""Comparison helpers shared by the parity tests."""
import numpy as np

import cases as C


def same_bits_nan_aware(a, b, op):
    """Byte equality, except that a NaN element matches any NaN (payload bits of a
    NaN produced by arithmetic are not pinned by the reference or IEEE)."""
    if np.array_equal(a, b):
        return True
    rt = np.dtype(C.REAL[op])
    if rt.kind != "f":
        return False
    n = (a.size // rt.itemsize) * rt.itemsize
    if not np.array_equal(a[n:], b[n:]):
        return False
    x, y = a[:n].view(rt), b[:n].view(rt)
    xn, yn = np.isnan(x), np.isnan(y)
    if not np.array_equal(xn, yn):
        return False
    it = np.int64 if rt.itemsize == 8 else np.int32
    return np.array_equal(x[~xn].view(it), y[~yn].view(it))


def first_mismatch(a, b, op):
    rt = np.dtype(C.REAL[op])
    n = (min(a.size, b.size) // rt.itemsize) * rt.itemsize
    x, y = a[:n].view(rt), b[:n].view(rt)
    bad = np.nonzero(~((x == y) | (np.isnan(x) & np.isnan(y)) if rt.kind == "f" else (x == y)))[0]
    if bad.size == 0:
        return "tail bytes differ"
    i = bad[0]
    return f"{bad.size} elements differ, first at {i}: got {x[i]!r} want {y[i]!r}"
