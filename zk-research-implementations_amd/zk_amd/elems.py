"""Field element marshalling: Python ints <-> numpy uint64[n, 4] (LE limbs)."""
from __future__ import annotations

import ctypes as C

import numpy as np

MASK64 = (1 << 64) - 1


def as_limbs(values) -> np.ndarray:
    """Python ints or an existing uint64[n,4] array -> C-contiguous uint64[n,4]."""
    if isinstance(values, np.ndarray):
        a = np.ascontiguousarray(values, dtype=np.uint64)
        if a.ndim == 1 and a.shape[0] == 4:
            a = a.reshape(1, 4)
        if a.ndim != 2 or a.shape[1] != 4:
            raise ValueError("expected a uint64 array of shape [n, 4]")
        return a
    vals = [int(v) for v in values]
    out = np.empty((len(vals), 4), dtype=np.uint64)
    for i, v in enumerate(vals):
        if v < 0:
            raise ValueError("field elements are non-negative canonical integers")
        out[i, 0] = v & MASK64
        out[i, 1] = (v >> 64) & MASK64
        out[i, 2] = (v >> 128) & MASK64
        out[i, 3] = (v >> 192) & MASK64
    return out


def to_ints(a: np.ndarray) -> list[int]:
    a = np.asarray(a, dtype=np.uint64).reshape(-1, 4)
    return [int(r[0]) | int(r[1]) << 64 | int(r[2]) << 128 | int(r[3]) << 192 for r in a]


def one(v: int) -> np.ndarray:
    return as_limbs([v])


def ptr(a: np.ndarray) -> C.c_void_p:
    """Pointer to a's data that keeps a alive (numpy's data_as holds a reference),
    so `f(ptr(as_limbs(x)))` cannot hand the C side a freed temporary."""
    return a.ctypes.data_as(C.c_void_p)
