"""ORACLE — TEST INFRASTRUCTURE ONLY.

ctypes binding of oracle/build/liboracle.so (the C restatement in
zk_oracle.c). Imported only by tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg. Elements cross this boundary as canonical numpy uint64[...,4].
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "build", "liboracle.so")
_lib = None


def build() -> str:
    subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return _LIB_PATH


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH) or os.path.getmtime(_LIB_PATH) < os.path.getmtime(
            os.path.join(_HERE, "zk_oracle.c")
        ):
            build()
        L = C.CDLL(_LIB_PATH)
        P = C.c_void_p
        u32, u64, i32 = C.c_uint32, C.c_uint64, C.c_int
        L.or_transcript_new.restype = P
        L.or_transcript_free.argtypes = [P]
        L.or_transcript_append.argtypes = [P, P, C.c_size_t]
        L.or_transcript_challenge.argtypes = [P, i32, P]
        L.or_keccak256.argtypes = [P, C.c_size_t, P]
        L.or_mle_partial_evaluate.argtypes = [i32, P, u32, u32, P, P]
        L.or_mle_evaluate.argtypes = [i32, P, u32, P, P]
        L.or_interpolate.argtypes = [i32, P, P, i32, P]
        L.or_sumcheck_prove.argtypes = [i32, P, u32, P, P]
        L.or_sumcheck_verify.argtypes = [i32, P, u32, P, u32, u32, P]
        L.or_gkr_prove.argtypes = [i32, P, u32, P, P, P, P]
        L.or_gkr_prove_fast.argtypes = [i32, P, u32, P, P, P, P]
        L.or_threads.restype = i32
        L.or_gkr_verify.argtypes = [i32, P, P, u32, P, P, P, P]
        L.or_synth_fill.argtypes = [i32, u64, u32, u64, u64, P]
        L.or_fe_from_le_bytes_mod_order.argtypes = [i32, P, C.c_size_t, P]
        L.or_fe_to_mont.argtypes = [i32, P, P]
        L.or_fe_add.argtypes = [i32, P, P, P]
        L.or_fe_mul.argtypes = [i32, P, P, P]
        _lib = L
    return _lib


def _ptr(a: np.ndarray):
    return a.ctypes.data_as(C.c_void_p)


def to_limbs(values) -> np.ndarray:
    out = np.zeros((len(values), 4), dtype=np.uint64)
    for i, v in enumerate(values):
        v = int(v)
        for k in range(4):
            out[i, k] = (v >> (64 * k)) & 0xFFFFFFFFFFFFFFFF
    return out


def from_limbs(a: np.ndarray) -> list[int]:
    a = np.asarray(a, dtype=np.uint64).reshape(-1, 4)
    return [int(r[0]) | int(r[1]) << 64 | int(r[2]) << 128 | int(r[3]) << 192 for r in a]


class Transcript:
    def __init__(self):
        self.h = lib().or_transcript_new()

    def __del__(self):
        if getattr(self, "h", None):
            lib().or_transcript_free(self.h)
            self.h = None

    def append(self, b: bytes) -> None:
        buf = np.frombuffer(bytes(b), dtype=np.uint8).copy()
        lib().or_transcript_append(self.h, _ptr(buf), len(buf))

    def get_random_challenge(self, field: int) -> int:
        out = np.zeros((1, 4), np.uint64)
        lib().or_transcript_challenge(self.h, field, _ptr(out))
        return from_limbs(out)[0]


def keccak256(data: bytes) -> bytes:
    buf = np.frombuffer(bytes(data) or b"\0", dtype=np.uint8).copy()
    out = np.zeros(32, np.uint8)
    lib().or_keccak256(_ptr(buf), len(data), _ptr(out))
    return out.tobytes()


def synth(field: int, seed: int, table: int, index0: int, count: int) -> np.ndarray:
    out = np.zeros((count, 4), np.uint64)
    lib().or_synth_fill(field, seed, table, index0, count, _ptr(out))
    return out


def partial_evaluate(field: int, evals: np.ndarray, bit: int, r: int) -> np.ndarray:
    evals = np.ascontiguousarray(evals, dtype=np.uint64)
    n = evals.shape[0].bit_length() - 1
    out = np.zeros((evals.shape[0] // 2, 4), np.uint64)
    rr = to_limbs([r])
    assert lib().or_mle_partial_evaluate(field, _ptr(evals), n, bit, _ptr(rr), _ptr(out)) == 0
    return out


def evaluate(field: int, evals: np.ndarray, point) -> int:
    evals = np.ascontiguousarray(evals, dtype=np.uint64)
    n = evals.shape[0].bit_length() - 1
    pt = to_limbs(point) if len(point) else np.zeros((1, 4), np.uint64)
    out = np.zeros((1, 4), np.uint64)
    assert lib().or_mle_evaluate(field, _ptr(evals), n, _ptr(pt), _ptr(out)) == 0
    return from_limbs(out)[0]


def interpolate(field: int, xs, ys) -> list[int]:
    X, Y = to_limbs(xs), to_limbs(ys)
    out = np.zeros((8, 4), np.uint64)
    k = lib().or_interpolate(field, _ptr(X), _ptr(Y), len(xs), _ptr(out))
    return from_limbs(out[:k])


def prove(field: int, evals: np.ndarray):
    evals = np.ascontiguousarray(evals, dtype=np.uint64)
    n = evals.shape[0].bit_length() - 1
    rp = np.zeros((max(2 * n, 1), 4), np.uint64)
    cs = np.zeros((1, 4), np.uint64)
    assert lib().or_sumcheck_prove(field, _ptr(evals), n, _ptr(rp), _ptr(cs)) == 0
    return rp[: 2 * n].reshape(n, 2, 4), from_limbs(cs)[0]


def verify(field: int, evals: np.ndarray, round_polys: np.ndarray, claimed: int) -> int:
    evals = np.ascontiguousarray(evals, dtype=np.uint64)
    n = evals.shape[0].bit_length() - 1
    rp = np.ascontiguousarray(round_polys, dtype=np.uint64)
    nrounds, plen = (rp.shape[0], rp.shape[1]) if rp.ndim == 3 else (0, 2)
    buf = rp.reshape(-1, 4) if rp.size else np.zeros((1, 4), np.uint64)
    return lib().or_sumcheck_verify(field, _ptr(evals), n, _ptr(buf), nrounds, plen, _ptr(to_limbs([claimed])))


def threads() -> int:
    return int(lib().or_threads())


def gkr_prove(field: int, tables, transcript: Transcript, fast: bool = False):
    """or_gkr_prove (reference-faithful, 1 thread) or, with fast=True,
    or_gkr_prove_fast (fused, in place, OpenMP; identical outputs)."""
    tabs = [np.ascontiguousarray(t, dtype=np.uint64) for t in tables]
    n = tabs[0].shape[0].bit_length() - 1
    arr = (C.c_void_p * 4)(*[t.ctypes.data for t in tabs])
    coeffs = np.zeros((max(n, 1), 3, 4), np.uint64)
    nco = np.zeros(max(n, 1), np.uint8)
    ch = np.zeros((max(n, 1), 4), np.uint64)
    fn = lib().or_gkr_prove_fast if fast else lib().or_gkr_prove
    assert fn(field, arr, n, transcript.h, _ptr(coeffs), _ptr(nco), _ptr(ch)) == 0
    polys = [from_limbs(coeffs[k, : nco[k]]) for k in range(n)]
    return polys, from_limbs(ch[:n])


def gkr_verify(field: int, round_polys, claimed: int, transcript: Transcript):
    n = len(round_polys)
    coeffs = np.zeros((max(n, 1), 3, 4), np.uint64)
    nco = np.zeros(max(n, 1), np.uint8)
    for k, rp in enumerate(round_polys):
        nco[k] = len(rp)
        if rp:
            coeffs[k, : len(rp)] = to_limbs(rp)
    fin = np.zeros((1, 4), np.uint64)
    ch = np.zeros((max(n, 1), 4), np.uint64)
    ok = lib().or_gkr_verify(field, _ptr(coeffs), _ptr(nco), n, _ptr(to_limbs([claimed])), transcript.h, _ptr(fin), _ptr(ch))
    return bool(ok), from_limbs(fin)[0], (from_limbs(ch[:n]) if ok else [0])
