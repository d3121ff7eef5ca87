"""Mirror of the reference multilinear KZG (pcs/src/kzg_pcs/kzg.rs) over
BLS12-381 G1, on the GPU through the C ABI.

Points are (x, y) canonical integers, None for the point at infinity (ark's
affine identity); G2 points are ((x0, x1), (y0, y1)) over Fq2 = Fq[u]/(u^2+1).
Scalars are BLS12-381 Fr integers. The G1 work (setup basis, commit, get_proof)
runs on the GPU; the verifier half (G2 taus, pairings) is host code in the
library (csrc/pairing.hpp), O(nvars) like gkr_verify.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from ._lib import lib
from .api import Field, _call, default_context
from .context import REPR_CANONICAL, Context
from .elems import as_limbs, ptr, to_ints

FIELD = Field.BLS12_381_FR


def _points(a: np.ndarray) -> list:
    out = []
    for row in a:
        x = sum(int(row[i]) << (64 * i) for i in range(6))
        y = sum(int(row[6 + i]) << (64 * i) for i in range(6))
        out.append(None if x == 0 and y == 0 else (x, y))
    return out


def _g1_array(points: list) -> np.ndarray:
    a = np.zeros((max(len(points), 1), 12), np.uint64)
    for k, pt in enumerate(points):
        if pt is None:
            continue
        for j, v in enumerate(pt):
            for i in range(6):
                a[k, 6 * j + i] = (v >> (64 * i)) & 0xFFFFFFFFFFFFFFFF
    return a


def _g2_array(points: list) -> np.ndarray:
    a = np.zeros((max(len(points), 1), 24), np.uint64)
    for k, pt in enumerate(points):
        if pt is None:
            continue
        for j, v in enumerate((pt[0][0], pt[0][1], pt[1][0], pt[1][1])):
            for i in range(6):
                a[k, 6 * j + i] = (int(v) >> (64 * i)) & 0xFFFFFFFFFFFFFFFF
    return a


def _g2_points(a: np.ndarray) -> list:
    out = []
    for row in a:
        c = [sum(int(row[6 * j + i]) << (64 * i) for i in range(6)) for j in range(4)]
        out.append(None if not any(c) else ((c[0], c[1]), (c[2], c[3])))
    return out


class KZG:  # kzg.rs:10-49
    def __init__(self, taus: list[int], ctx: Context | None = None):
        self.ctx = ctx or default_context()
        self.nvars = len(taus)
        h = C.c_void_p()
        _call(lib().zk_kzg_setup(self.ctx.h, REPR_CANONICAL, ptr(as_limbs([int(t) for t in taus])), self.nvars,
                                 C.byref(h)))
        self.h = h

    def close(self) -> None:
        if self.h:
            lib().zk_kzg_free(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @property
    def g2_taus(self) -> list:  # pub g2_taus (:13, :43-46)
        out = np.zeros((self.nvars, 24), np.uint64)
        _call(lib().zk_kzg_g2_taus(self.h, ptr(out)))
        return _g2_points(out)

    @staticmethod
    def verify(commitment, opened_value: int, proof: list, opening_values: list[int], g2_taus: list) -> bool:
        """KZG::verify (:97-129); ValueError where the reference panics (:104-106)."""
        ok = C.c_int(0)
        n = len(opening_values)
        _call(lib().zk_kzg_verify(REPR_CANONICAL, ptr(_g1_array([commitment])), ptr(as_limbs([int(opened_value)])),
                                  ptr(_g1_array(proof)), len(proof),
                                  ptr(as_limbs([int(v) for v in opening_values]) if n else np.zeros((1, 4), np.uint64)),
                                  n, ptr(_g2_array(list(g2_taus)[:n])), C.byref(ok)))
        return bool(ok.value)

    def lagrange_basis(self, nvars_suffix: int | None = None) -> list:  # get_lagrange_basis (:183-212)
        v = self.nvars if nvars_suffix is None else nvars_suffix
        out = np.zeros((1 << v, 12), np.uint64)
        _call(lib().zk_kzg_lagrange_basis(self.ctx.h, self.h, v, ptr(out)))
        return _points(out)

    def commit(self, evals: list[int]):  # :51-53
        out = np.zeros((1, 12), np.uint64)
        _call(lib().zk_kzg_commit(self.ctx.h, self.h, REPR_CANONICAL, ptr(as_limbs([int(e) for e in evals])),
                                  ptr(out)))
        return _points(out)[0]

    def open(self, opening_values: list[int], evals: list[int]) -> int:  # :55-57 (MultilinearPoly::evaluate)
        res = np.zeros((1, 4), np.uint64)
        pt = as_limbs([int(v) for v in opening_values])
        _call(lib().zk_mle_evaluate(self.ctx.h, int(FIELD), REPR_CANONICAL, ptr(as_limbs([int(e) for e in evals])),
                                    self.nvars, ptr(pt), len(opening_values), ptr(res)))
        return to_ints(res)[0]

    def get_proof(self, opened_value: int, opening_values: list[int], evals: list[int]) -> list:  # :59-95
        out = np.zeros((self.nvars, 12), np.uint64)
        _call(lib().zk_kzg_get_proof(self.ctx.h, self.h, REPR_CANONICAL, ptr(as_limbs([int(e) for e in evals])),
                                     ptr(as_limbs([int(opened_value)])),
                                     ptr(as_limbs([int(v) for v in opening_values])), ptr(out)))
        return _points(out)


    def get_proof_device(self, opened_value: int, opening_values: list[int], table) -> list:
        """get_proof over evaluations already on the device (a DeviceTable of
        2^nvars BLS12-381 Fr values, e.g. Context.upload / synth): no host
        upload (zk_dev_kzg_get_proof)."""
        if table.count != 1 << self.nvars or int(table.field) != int(FIELD):
            raise ValueError("the device table must hold 2^nvars BLS12-381 Fr values")
        out = np.zeros((self.nvars, 12), np.uint64)
        _call(lib().zk_dev_kzg_get_proof(self.ctx.h, self.h, REPR_CANONICAL, table.ptr,
                                         ptr(as_limbs([int(opened_value)])),
                                         ptr(as_limbs([int(v) for v in opening_values])), ptr(out)))
        return _points(out)


def release_fixed_base_cache(device: int = -1) -> None:
    """Free the per-device fixed-base table large setups share (654 MB of HBM;
    -1: every device). ZkError while a setup is using it."""
    _call(lib().zk_kzg_release_fixed_base_cache(int(device)))


def msm_g1(bases: list, scalars: list[int], ctx: Context | None = None):
    """sum_i scalars[i] * bases[i] (bases must be on the curve)."""
    ctx = ctx or default_context()
    out = np.zeros((1, 12), np.uint64)
    sc = as_limbs([int(s) for s in scalars]) if scalars else np.zeros((1, 4), np.uint64)
    _call(lib().zk_msm_g1(ctx.h, REPR_CANONICAL, ptr(_g1_array(bases)), ptr(sc), len(scalars), ptr(out)))
    return _points(out)[0]


def g2_mul_generator(scalars: list[int]) -> list:
    """scalars[i] * G2 (G2Projective::mul_bigint), host."""
    out = np.zeros((max(len(scalars), 1), 24), np.uint64)
    sc = as_limbs([int(s) for s in scalars]) if scalars else np.zeros((1, 4), np.uint64)
    _call(lib().zk_g2_mul_generator(REPR_CANONICAL, ptr(sc), len(scalars), ptr(out)))
    return _g2_points(out)[: len(scalars)]


def pairing(p, q) -> list[int]:
    """Bls12_381::pairing(p, q): the Fq12 value as 12 canonical Fq integers in
    ark's order (c0.c0.re, c0.c0.im, c0.c1.re, ..., c1.c2.im)."""
    out = np.zeros(72, np.uint64)
    _call(lib().zk_bls12_381_pairing(ptr(_g1_array([p])), ptr(_g2_array([q])), ptr(out)))
    return [sum(int(out[6 * k + i]) << (64 * i) for i in range(6)) for k in range(12)]


def pairing_check(pairs: list) -> bool:
    """prod_i e(p_i, q_i) == 1 (one final exponentiation)."""
    ok = C.c_int(0)
    _call(lib().zk_bls12_381_pairing_check(ptr(_g1_array([p for p, _ in pairs])),
                                           ptr(_g2_array([q for _, q in pairs])), len(pairs), C.byref(ok)))
    return bool(ok.value)
