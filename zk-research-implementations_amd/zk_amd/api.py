"""Reference-shaped API (same names, argument meaning and panic points as the
Rust crates), backed by the HIP library.

Reference item -> here:
  fiat_shamir_transcript.rs:5-30   Transcript{new, append, get_random_challenge}, Clone
  fiat_shamir_transcript.rs:32-37  fq_vec_to_bytes
  multilinear_polynomial_evaluation.rs:19-91   MultilinearPoly{new, partial_evaluate,
                                               multi_partial_evaluate, evaluate}
  composed_polynomial.rs:5-103     ProductPoly, SumPoly{new, evaluate, partial_evaluate, get_degree}
  univariate_polynomial_dense.rs   UnivariatePoly{coefficient, evaluate, degree, interpolate}
  sum_check_protocol.rs:8-150      Proof, GkrProof, GkrVerify, prove, verify, gkr_prove, gkr_verify
Where the reference panics, these raise ValueError (the C ABI's ZK_EINVAL).
"""
from __future__ import annotations

import ctypes as C
import os
from dataclasses import dataclass, field as dc_field
from enum import IntEnum

import numpy as np

from ._lib import ZK_BLOB_GKR, ZK_BLOB_SUMCHECK, ZK_EINVAL, ZkError, check, lib
from .context import REPR_CANONICAL, Context
from .elems import as_limbs, one, ptr, to_ints

MLE_ADD, MLE_MUL, MLE_SUB = 0, 1, 2  # zk_mle_op


class Field(IntEnum):
    BN254_FR = 0
    BN254_FQ = 1
    BLS12_381_FR = 2


_MODULI = {
    Field.BN254_FR: 0x30644E72E131A029B85045B68181585D2833E84879B9709143E1F593F0000001,
    Field.BN254_FQ: 0x30644E72E131A029B85045B68181585D97816A916871CA8D3C208C16D87CFD47,
    Field.BLS12_381_FR: 0x73EDA753299D7D483339D80809A1D80553BDA402FFFE5BFEFFFFFFFF00000001,
}


def modulus(field: int) -> int:
    return _MODULI[Field(field)]


_contexts: dict[int, Context] = {}


def default_context(device: int | None = None) -> Context:
    """Process-wide context for `device` (default: $ZK_DEVICE, else $LOCAL_RANK, else 0)."""
    if device is None:
        device = int(os.environ.get("ZK_DEVICE", os.environ.get("LOCAL_RANK", "0")))
    if device not in _contexts:
        _contexts[device] = Context(device)
    return _contexts[device]


def _call(code: int) -> None:
    try:
        check(code)
    except ZkError as e:
        if e.code == ZK_EINVAL:
            raise ValueError(str(e)) from None
        raise


# ---------------------------------------------------------------------------
# fiat_shamir
# ---------------------------------------------------------------------------
class Transcript:
    """Keccak256 Fiat-Shamir transcript (host side of the library)."""

    def __init__(self, field: int = Field.BN254_FR, _handle=None):
        self.field = Field(field)
        self.h = _handle if _handle is not None else lib().zk_transcript_new()
        if not self.h:
            raise MemoryError("zk_transcript_new failed")

    def __del__(self):
        try:
            if getattr(self, "h", None):
                lib().zk_transcript_free(self.h)
                self.h = None
        except Exception:  # interpreter shutdown: module globals may already be gone
            pass

    def append(self, preimage: bytes) -> None:
        b = bytes(preimage)
        buf = (C.c_uint8 * max(1, len(b))).from_buffer_copy(b or b"\0")
        _call(lib().zk_transcript_append(self.h, buf, len(b)))

    def get_random_challenge(self) -> int:
        out = np.zeros((1, 4), np.uint64)
        _call(lib().zk_transcript_get_random_challenge(self.h, int(self.field), REPR_CANONICAL, ptr(out)))
        return to_ints(out)[0]

    def clone(self) -> "Transcript":
        return Transcript(self.field, _handle=lib().zk_transcript_clone(self.h))

    def to_bytes(self) -> bytes:
        """Checkpoint: the byte image of `clone()` (zk_transcript_serialize)."""
        out = (C.c_uint8 * 352)()
        n = C.c_size_t(0)
        _call(lib().zk_transcript_serialize(self.h, out, len(out), C.byref(n)))
        return bytes(out[: n.value])

    @classmethod
    def from_bytes(cls, state: bytes, field: int = Field.BN254_FR) -> "Transcript":
        """Resume from `to_bytes()`; ValueError on a malformed state."""
        b = bytes(state)
        buf = (C.c_uint8 * max(1, len(b))).from_buffer_copy(b or b"\0")
        h = lib().zk_transcript_deserialize(buf, len(b))
        if not h:
            raise ValueError("malformed transcript state")
        return cls(field, _handle=h)


def fq_vec_to_bytes(values, field: int = Field.BN254_FR) -> bytes:
    a = as_limbs(values)
    out = np.zeros(32 * a.shape[0], np.uint8)
    if a.shape[0]:
        _call(lib().zk_fe_vec_to_bytes(int(field), REPR_CANONICAL, ptr(a), a.shape[0], ptr(out)))
    return out.tobytes()


# ---------------------------------------------------------------------------
# multilinear_polynomial
# ---------------------------------------------------------------------------
class MultilinearPoly:
    def __init__(self, evaluations, field: int = Field.BN254_FR, ctx: Context | None = None):
        self.field = Field(field)
        self.limbs = as_limbs(evaluations)
        n = self.limbs.shape[0]
        if n == 0 or n & (n - 1):
            raise ValueError("Invalid evaluations")  # :27-31
        self.num_of_vars = n.bit_length() - 1
        self.ctx = ctx

    @property
    def evaluation(self) -> list[int]:
        return to_ints(self.limbs)

    def _ctx(self) -> Context:
        return self.ctx or default_context()

    def partial_evaluate(self, bit: int, value: int) -> "MultilinearPoly":  # :52-63
        out = np.zeros((self.limbs.shape[0] // 2, 4), np.uint64)
        _call(
            lib().zk_mle_partial_evaluate(
                self._ctx().h, int(self.field), REPR_CANONICAL, ptr(self.limbs), self.num_of_vars, int(bit),
                ptr(one(value)), ptr(out),
            )
        )
        return MultilinearPoly(out, self.field, self.ctx)

    def multi_partial_evaluate(self, values) -> "MultilinearPoly":  # :65-77
        if len(values) > self.num_of_vars:
            raise ValueError("Invalid number of values")
        poly = self
        for v in values:
            poly = poly.partial_evaluate(0, v)
        return poly

    def evaluate(self, values) -> int:  # :79-91
        pt = as_limbs(list(values)) if len(values) else np.zeros((1, 4), np.uint64)
        out = np.zeros((1, 4), np.uint64)
        _call(
            lib().zk_mle_evaluate(
                self._ctx().h, int(self.field), REPR_CANONICAL, ptr(self.limbs), self.num_of_vars, ptr(pt),
                len(values), ptr(out),
            )
        )
        return to_ints(out)[0]

    def scale(self, value: int) -> "MultilinearPoly":  # :93-97
        out = np.zeros_like(self.limbs)
        _call(lib().zk_mle_scale(self._ctx().h, int(self.field), REPR_CANONICAL, ptr(self.limbs), self.num_of_vars,
                                 ptr(one(value)), ptr(out)))
        return MultilinearPoly(out, self.field, self.ctx)

    def _binop(self, other: "MultilinearPoly", op: int) -> "MultilinearPoly":  # impl Add/Mul/Sub :113-151
        if not isinstance(other, MultilinearPoly):
            return NotImplemented
        out = np.zeros((min(self.limbs.shape[0], other.limbs.shape[0]), 4), np.uint64)
        _call(lib().zk_mle_binop(self._ctx().h, int(self.field), REPR_CANONICAL, op, ptr(self.limbs),
                                 self.num_of_vars, ptr(other.limbs), other.num_of_vars, ptr(out)))
        return MultilinearPoly(out, self.field, self.ctx)

    def __add__(self, other):
        return self._binop(other, MLE_ADD)

    def __mul__(self, other):
        return self._binop(other, MLE_MUL)

    def __sub__(self, other):
        return self._binop(other, MLE_SUB)

    @staticmethod
    def tensor_add_mul_polynomials(poly_a, poly_b, op, field: int = Field.BN254_FR,
                                   ctx: Context | None = None) -> "MultilinearPoly":  # :99-110
        """op: gkr.Operation (Add = 0, Mul = 1) or the strings "add" / "mul"."""
        code = {"add": MLE_ADD, "mul": MLE_MUL}[op] if isinstance(op, str) else int(op)
        a, b = as_limbs(poly_a), as_limbs(poly_b)
        out = np.zeros((a.shape[0] * b.shape[0], 4), np.uint64)
        _call(lib().zk_mle_tensor((ctx or default_context()).h, int(field), REPR_CANONICAL, code, ptr(a),
                                  a.shape[0], ptr(b), b.shape[0], ptr(out)))
        return MultilinearPoly(out, field, ctx)

    def __eq__(self, other) -> bool:
        return (
            isinstance(other, MultilinearPoly)
            and self.field == other.field
            and np.array_equal(self.limbs, other.limbs)
        )


class ProductPoly:
    def __init__(self, evaluations, field: int = Field.BN254_FR, ctx: Context | None = None):  # :16-28
        evs = [as_limbs(e) for e in evaluations]
        if not evs:
            raise ValueError("index out of bounds: evaluations[0]")
        if any(e.shape[0] != evs[0].shape[0] for e in evs):
            raise ValueError("all evaluations must have same length")
        self.evaluation = [MultilinearPoly(e, field, ctx) for e in evs]
        self.field = Field(field)

    def get_degree(self) -> int:  # :56-58
        return len(self.evaluation)

    def evaluate(self, values) -> int:  # :31-36
        p = modulus(self.field)
        acc = 1
        for poly in self.evaluation:
            acc = acc * poly.evaluate(values) % p
        return acc

    def reduce(self) -> list[int]:  # :52-54: evaluation[0] * evaluation[1]
        return (self.evaluation[0] * self.evaluation[1]).evaluation

    def partial_evaluate(self, value: int) -> "ProductPoly":  # :38-50
        return ProductPoly([poly.partial_evaluate(0, value).limbs for poly in self.evaluation], self.field,
                           self.evaluation[0].ctx)


class SumPoly:
    def __init__(self, polys: list[ProductPoly]):  # :61-68
        if not polys:
            raise ValueError("index out of bounds: polys[0]")
        d = polys[0].get_degree()
        if any(pp.get_degree() != d for pp in polys):
            raise ValueError("all product polys must have same degree")
        self.polys = list(polys)
        self.field = polys[0].field

    def get_degree(self) -> int:  # :101-103
        return self.polys[0].get_degree()

    def evaluate(self, values) -> int:  # :71-76
        p = modulus(self.field)
        return sum(pp.evaluate(values) for pp in self.polys) % p

    def partial_evaluate(self, value: int) -> "SumPoly":  # :78-86
        return SumPoly([pp.partial_evaluate(value) for pp in self.polys])

    def reduce(self) -> list[int]:  # :88-99: polys[0].reduce() + polys[1].reduce() (zip)
        p = modulus(self.field)
        return [(x + y) % p for x, y in zip(self.polys[0].reduce(), self.polys[1].reduce())]

    def gkr_tables(self) -> list[np.ndarray]:
        """The four tables SumPoly::reduce reads (:88-99 with :52-54):
        polys[0].evaluation[0..2] and polys[1].evaluation[0..2]."""
        if len(self.polys) < 2:
            raise ValueError("index out of bounds: polys[1] (SumPoly::reduce)")
        if self.get_degree() < 2:
            raise ValueError("index out of bounds: evaluation[1] (ProductPoly::reduce)")
        t = [self.polys[0].evaluation[0], self.polys[0].evaluation[1], self.polys[1].evaluation[0],
             self.polys[1].evaluation[1]]
        n = t[0].limbs.shape[0]
        for pp in self.polys:
            for mle in pp.evaluation:
                if mle.limbs.shape[0] != n:
                    # the reference zips (truncates) or panics once a smaller table is exhausted
                    raise ValueError("all tables of a SumPoly must have the same length")
        return [m.limbs for m in t]


# ---------------------------------------------------------------------------
# univariate_polynomial (host scalar helper for proof polynomials)
# ---------------------------------------------------------------------------
@dataclass
class UnivariatePoly:
    coefficient: list[int]
    field: int = Field.BN254_FR

    def evaluate(self, x: int) -> int:  # :20-26
        p = modulus(self.field)
        return sum(c * pow(x, i, p) for i, c in enumerate(self.coefficient)) % p

    def degree(self) -> int:  # :28-32
        while self.coefficient and self.coefficient[-1] == 0:
            self.coefficient.pop()
        if not self.coefficient:
            raise ValueError("attempt to subtract with overflow")
        return len(self.coefficient) - 1


# ---------------------------------------------------------------------------
# sum_check
# ---------------------------------------------------------------------------
@dataclass
class Proof:  # :8-12
    proof_polynomials: list[list[int]]
    claimed_sum: int

    def to_bytes(self, field: int = Field.BN254_FR) -> bytes:
        """Canonical proof blob (include/zk_sumcheck.h "Proof blob", kind ZK_BLOB_SUMCHECK)."""
        polys = self.proof_polynomials
        plen = len(polys[0]) if polys else 2
        if any(len(p) != plen for p in polys):
            raise ValueError("round polynomials of different lengths")
        flat = as_limbs([v for p in polys for v in p]) if polys and plen else np.zeros((1, 4), np.uint64)
        return _blob(lambda out, cap, n: lib().zk_sumcheck_proof_to_blob(
            int(field), REPR_CANONICAL, ptr(flat), len(polys), plen, ptr(one(self.claimed_sum)), out, cap, n))

    @staticmethod
    def from_bytes(blob: bytes) -> "Proof":
        kind, _, n = blob_info(blob)
        if kind != ZK_BLOB_SUMCHECK:
            raise ValueError("ZK_EINVAL: not a sum-check proof blob")
        cap = max(1, (len(blob) - 44) // 32)
        rp = np.zeros((cap, 4), np.uint64)
        plen = C.c_uint32(0)
        cs = np.zeros((1, 4), np.uint64)
        _call(lib().zk_sumcheck_proof_from_blob(blob, len(blob), REPR_CANONICAL, ptr(rp), cap, C.byref(plen), ptr(cs)))
        vals = to_ints(rp[: n * plen.value])
        m = plen.value
        return Proof([vals[m * k: m * k + m] for k in range(n)], to_ints(cs)[0])


@dataclass
class GkrProof:  # :13-17
    proof_polynomials: list[UnivariatePoly]
    claimed_sum: int
    random_challenges: list[int]

    def to_bytes(self, field: int | None = None) -> bytes:
        """Canonical proof blob (kind ZK_BLOB_GKR): per round exactly the bytes the
        transcript absorbs. The challenges are not stored (a verifier re-derives them)."""
        if field is None:
            field = self.proof_polynomials[0].field if self.proof_polynomials else Field.BN254_FR
        coeffs, nco = _gkr_coeff_arrays(self.proof_polynomials)
        return _blob(lambda out, cap, n: lib().zk_gkr_proof_to_blob(
            int(field), REPR_CANONICAL, ptr(coeffs), ptr(nco), len(self.proof_polynomials),
            ptr(one(self.claimed_sum)), out, cap, n))

    @staticmethod
    def from_bytes(blob: bytes) -> "GkrProof":
        kind, field, n = blob_info(blob)
        if kind != ZK_BLOB_GKR:
            raise ValueError("ZK_EINVAL: not a GKR sum-check proof blob")
        coeffs = np.zeros((max(n, 1), 3, 4), np.uint64)
        nco = np.zeros(max(n, 1), np.uint8)
        cs = np.zeros((1, 4), np.uint64)
        _call(lib().zk_gkr_proof_from_blob(blob, len(blob), REPR_CANONICAL, ptr(coeffs), ptr(nco), max(n, 1), ptr(cs)))
        polys = [UnivariatePoly(to_ints(coeffs[k, : nco[k]]), field) for k in range(n)]
        return GkrProof(polys, to_ints(cs)[0], [])


def _gkr_coeff_arrays(round_polys) -> tuple[np.ndarray, np.ndarray]:
    n = len(round_polys)
    coeffs = np.zeros((max(n, 1), 3, 4), np.uint64)
    nco = np.zeros(max(n, 1), np.uint8)
    for k, rp in enumerate(round_polys):
        c = rp.coefficient if isinstance(rp, UnivariatePoly) else list(rp)
        if len(c) > 3:
            raise ValueError("round polynomial of degree > 2")
        nco[k] = len(c)
        if c:
            coeffs[k, : len(c)] = as_limbs(c)
    return coeffs, nco


def _blob(fill) -> bytes:
    n = C.c_size_t(0)
    _call(fill(None, 0, C.byref(n)))
    buf = (C.c_uint8 * n.value)()
    _call(fill(buf, n.value, C.byref(n)))
    return bytes(buf)


def blob_info(blob: bytes) -> tuple[int, "Field", int]:
    """(kind, field, nrounds) of a proof blob; raises ZkError on a malformed header."""
    kind, field, n = C.c_int(0), C.c_int(0), C.c_uint32(0)
    _call(lib().zk_proof_blob_info(blob, len(blob), C.byref(kind), C.byref(field), C.byref(n)))
    return kind.value, Field(field.value), n.value


def keccak256(data: bytes) -> bytes:
    out = (C.c_uint8 * 32)()
    _call(lib().zk_keccak256(data, len(data), out))
    return bytes(out)


@dataclass
class GkrVerify:  # :19-23
    verified: bool
    final_claimed_sum: int
    random_challenges: list[int] = dc_field(default_factory=list)


def prove(polynomial: MultilinearPoly, ctx: Context | None = None) -> Proof:  # :25-52
    ctx = ctx or polynomial.ctx or default_context()
    n = polynomial.num_of_vars
    rp = np.zeros((max(2 * n, 1), 4), np.uint64)
    cs = np.zeros((1, 4), np.uint64)
    _call(lib().zk_sumcheck_prove(ctx.h, int(polynomial.field), REPR_CANONICAL, ptr(polynomial.limbs), n, ptr(rp),
                                  ptr(cs)))
    vals = to_ints(rp[: 2 * n])
    return Proof([vals[2 * k: 2 * k + 2] for k in range(n)], to_ints(cs)[0])


def verify(polynomial: MultilinearPoly, proof: Proof, ctx: Context | None = None) -> bool:  # :54-84
    ctx = ctx or polynomial.ctx or default_context()
    polys = proof.proof_polynomials
    plen = len(polys[0]) if polys else 2
    if any(len(p) != plen for p in polys):
        raise ValueError("round polynomials of different lengths are not representable in this ABI")
    flat = as_limbs([v for p in polys for v in p]) if polys and plen else np.zeros((1, 4), np.uint64)
    ok = C.c_int(0)
    _call(lib().zk_sumcheck_verify(ctx.h, int(polynomial.field), REPR_CANONICAL, ptr(polynomial.limbs),
                                   polynomial.num_of_vars, ptr(flat), len(polys), plen, ptr(one(proof.claimed_sum)),
                                   C.byref(ok)))
    return bool(ok.value)


def gkr_prove(claimed_sum: int, composed_polynomial: SumPoly, transcript: Transcript,
              ctx: Context | None = None) -> GkrProof:  # :86-115
    tables = composed_polynomial.gkr_tables()
    ctx = ctx or composed_polynomial.polys[0].evaluation[0].ctx or default_context()
    n = tables[0].shape[0].bit_length() - 1
    arr = (C.c_void_p * 4)(*[t.ctypes.data for t in tables])
    coeffs = np.zeros((max(n, 1), 3, 4), np.uint64)
    nco = np.zeros(max(n, 1), np.uint8)
    ch = np.zeros((max(n, 1), 4), np.uint64)
    cs = np.zeros((1, 4), np.uint64)
    _call(lib().zk_gkr_sumcheck_prove(ctx.h, int(composed_polynomial.field), REPR_CANONICAL, arr, n,
                                      ptr(one(claimed_sum)), transcript.h, ptr(coeffs), ptr(nco), ptr(ch), ptr(cs)))
    field = composed_polynomial.field
    polys = [UnivariatePoly(to_ints(coeffs[k, : nco[k]]), field) for k in range(n)]
    return GkrProof(polys, to_ints(cs)[0], to_ints(ch[:n]))


def gkr_verify(round_polys: list[UnivariatePoly], claimed_sum: int, transcript: Transcript) -> GkrVerify:  # :117-150
    n = len(round_polys)
    field = transcript.field
    coeffs, nco = _gkr_coeff_arrays(round_polys)
    ok = C.c_int(0)
    fin = np.zeros((1, 4), np.uint64)
    ch = np.zeros((max(n, 1), 4), np.uint64)
    _call(lib().zk_gkr_sumcheck_verify(int(field), REPR_CANONICAL, ptr(coeffs), ptr(nco), n, ptr(one(claimed_sum)),
                                       transcript.h, C.byref(ok), ptr(fin), ptr(ch)))
    if not ok.value:
        return GkrVerify(False, 0, [0])
    return GkrVerify(True, to_ints(fin)[0], to_ints(ch[:n]))


def gkr_verify_blob(blob: bytes, transcript: Transcript) -> GkrVerify:
    """gkr_verify of a GKR proof blob (claimed sum from the blob)."""
    _, _, n = blob_info(blob)
    ok = C.c_int(0)
    fin = np.zeros((1, 4), np.uint64)
    ch = np.zeros((max(n, 1), 4), np.uint64)
    _call(lib().zk_gkr_verify_blob(blob, len(blob), transcript.h, C.byref(ok), ptr(fin), ptr(ch), max(n, 1)))
    if not ok.value:
        return GkrVerify(False, 0, [0])
    return GkrVerify(True, to_ints(fin)[0], to_ints(ch[:n]))
