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
    try:
        buf = b"".join(int(v).to_bytes(32, "little") for v in values)
    except OverflowError:
        raise ValueError("field elements are non-negative canonical integers below 2^256") from None
    return np.frombuffer(bytearray(buf), dtype="<u8").reshape(-1, 4)


def to_ints(a: np.ndarray) -> list[int]:
    b = np.ascontiguousarray(a, dtype="<u8").reshape(-1, 4).tobytes()
    return [int.from_bytes(b[i: i + 32], "little") for i in range(0, len(b), 32)]


def one(v: int) -> np.ndarray:
    return as_limbs([v])


def ptr(a: np.ndarray) -> C.c_void_p:
    """Pointer to a's data that keeps a alive (numpy's data_as holds a reference),
    so `f(ptr(as_limbs(x)))` cannot hand the C side a freed temporary."""
    return a.ctypes.data_as(C.c_void_p)
