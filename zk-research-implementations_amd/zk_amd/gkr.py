"""Mirror of the reference `gkr` crate (gkr/src/gkr_circuit.rs,
gkr/src/gkr_protocol.rs) over the C ABI: a layered circuit, `prove` (circuit
evaluation, per-layer tables and sum-checks on the GPU) and `verify` (host).

Differences from the reference:
* the input layer's KZG step (gkr_protocol.rs:92-118) runs over BLS12-381 Fr
  (the reference's KZG field, kzg.rs:3), as the reference always runs it: by
  default (`taus="entropy"`) the taus are drawn from the OS entropy source like
  the reference's `StdRng::from_entropy()` (:94-103) — a fresh, unreproducible
  setup per proof — and caller-given taus make the proof reproducible (tests).
  The proof then carries `input_proof` (commitment, both get_proofs, the opened
  values, the G2 taus) and `verify` checks it with two KZG::verify pairings
  (:155-175). `taus=None` skips the KZG step (a library extension, and the only
  mode over BN254, whose reference `gkr::prove` cannot instantiate the
  BLS12-381 KZG): the proof then carries only the two input-MLE evaluations
  KZG::open would return, and `verify` recomputes them from the inputs when
  they are given;
* only the circuit shape for which the reference's table sizes agree is
  accepted (binary tree, powers of two, 1- or 2-gate output layer);
  anything else raises ValueError (the reference panics or mis-sizes).
"""
from __future__ import annotations

import ctypes as C
import os
from dataclasses import dataclass
from enum import IntEnum

import numpy as np

from ._lib import lib
from .api import Field, UnivariatePoly, _call, default_context, modulus
from .context import REPR_CANONICAL, Context
from .elems import as_limbs, ptr, to_ints


class Operation(IntEnum):  # multilinear_polynomial_evaluation.rs:4-17
    Add = 0
    Mul = 1

    def apply(self, a: int, b: int, p: int) -> int:
        return (a + b) % p if self is Operation.Add else (a * b) % p


class Circuit:  # gkr_circuit.rs:107-144
    def __init__(self, structure: list[list[Operation]], field: int = Field.BN254_FR):
        # immutable, like the reference's Circuit after Circuit::new (gkr_circuit.rs:114-125)
        self.layers = tuple(tuple(Operation(op) for op in layer) for layer in structure)
        self.field = Field(field)

    def evaluate(self, inputs: list[int]) -> list[list[int]]:  # :127-143 (host; O(#gates))
        p = modulus(self.field)
        out, cur = [], [int(x) % p for x in inputs]
        for ops in self.layers:
            vals = [op.apply(0, 0, p) for op in ops]
            for i, op in enumerate(ops):
                if 2 * i + 1 < len(cur):
                    vals[i] = op.apply(cur[2 * i], cur[2 * i + 1], p)
            out.append(vals)
            cur = vals
        return out

    def _abi(self):
        # the C arrays of the structure, built once (the layers are tuples;
        # assigning a new `layers` rebuilds them)
        if getattr(self, "_abi_src", None) is not self.layers:  # (holds the source: no id reuse)
            gates = np.array([len(layer) for layer in self.layers], np.uint32)
            ops = np.fromiter((op for layer in self.layers for op in layer), np.uint8, int(gates.sum()))
            self._abi_cache, self._abi_src = (gates, ops), self.layers
        return self._abi_cache


@dataclass
class KzgProof:  # gkr_protocol.rs:15-21
    commitment: tuple | None              # G1 affine (x, y), None = infinity
    proof: tuple[list, list]              # get_proof at r_b, at r_c (nvars G1 points each)
    opened_evals: tuple[int, int]         # KZG::open at r_b, r_c
    g2_taus: list                         # kzg_setup.g2_taus


@dataclass
class GkrCircuitProof:  # gkr_protocol.rs:23-29
    output_poly: list[int]
    proof_polynomials: list[list[UnivariatePoly]]  # per layer, output layer first
    claimed_evaluations: list[tuple[int, int]]
    input_evaluations: tuple[int, int]
    random_challenges: list[list[int]]
    input_proof: KzgProof | None = None


def _rounds(gates: np.ndarray) -> int:
    n = C.c_uint32(0)
    _call(lib().zk_gkr_circuit_rounds(len(gates), ptr(gates), C.byref(n)))
    return n.value


def _layer_rounds(gates, coeffs, nco, ch, field):
    """Per layer (output first): its round polynomials (trimmed) and challenges,
    from the C arrays in one conversion each."""
    flat, chs, cnt = to_ints(coeffs.reshape(-1, 4)), to_ints(ch), nco.tolist()
    polys, chal, k0 = [], [], 0
    for layer in reversed(range(len(gates))):
        nv = 2 * (2 * int(gates[layer])).bit_length() - 2
        polys.append([UnivariatePoly(flat[3 * k: 3 * k + cnt[k]], field) for k in range(k0, k0 + nv)])
        chal.append(chs[k0: k0 + nv])
        k0 += nv
    return polys, chal


ENTROPY = "entropy"


def entropy_taus(nvars: int, field: int = Field.BLS12_381_FR) -> list[int]:
    """nvars field elements from the OS entropy source (the reference's
    F::rand(StdRng::from_entropy()), gkr_protocol.rs:94-101): 512 random bits
    reduced mod p each (bias < 2^-256)."""
    p = modulus(field)
    return [int.from_bytes(os.urandom(64), "little") % p for _ in range(nvars)]


def prove(circuit: Circuit, inputs: list[int] | np.ndarray, ctx: Context | None = None,
          taus: list[int] | str | None = ENTROPY) -> GkrCircuitProof:  # :31-126
    """gkr::prove. inputs: canonical ints, or a uint64[n, 4] array of them
    (little-endian limbs, the C ABI layout) which skips their conversion.
    taus: "entropy" (default; BLS12-381 Fr circuits run the input layer's KZG
    step over a fresh setup drawn from os.urandom, like the reference, and
    other fields skip it: the reference's KZG is BLS12-381-only), a list of
    one tau per input variable (reproducible; BLS12-381 Fr only), or None (no
    KZG step)."""
    ctx = ctx or default_context()
    if isinstance(taus, str):
        if taus != ENTROPY:
            raise ValueError(f'taus must be a list, None or "{ENTROPY}"')
        taus = entropy_taus(len(inputs).bit_length() - 1) if circuit.field == Field.BLS12_381_FR else None
    if taus is not None:
        return _prove_kzg(circuit, inputs, ctx, taus)
    gates, ops = circuit._abi()
    total = _rounds(gates)
    L = len(gates)
    outp = np.zeros((2, 4), np.uint64)
    coeffs = np.zeros((total, 3, 4), np.uint64)
    nco = np.zeros(total, np.uint8)
    ch = np.zeros((total, 4), np.uint64)
    claims = np.zeros((max(2 * (L - 1), 1), 4), np.uint64)
    ins = np.zeros((2, 4), np.uint64)
    x = as_limbs(inputs)
    _call(lib().zk_gkr_circuit_prove(ctx.h, int(circuit.field), REPR_CANONICAL, L, ptr(gates), ptr(ops), ptr(x),
                                     len(inputs), ptr(outp), ptr(coeffs), ptr(nco), ptr(ch), ptr(claims), ptr(ins)))
    polys, chal = _layer_rounds(gates, coeffs, nco, ch, circuit.field)
    cl = to_ints(claims[: 2 * (L - 1)])
    return GkrCircuitProof(to_ints(outp), polys, [(cl[2 * i], cl[2 * i + 1]) for i in range(L - 1)],
                           tuple(to_ints(ins)), chal)


def _prove_kzg(circuit: Circuit, inputs: list[int], ctx: Context, taus: list[int]) -> GkrCircuitProof:
    from .kzg import _g2_points, _points

    if circuit.field != Field.BLS12_381_FR:
        raise ValueError("the input layer's KZG commitment is over BLS12-381 (kzg.rs:3): use Field.BLS12_381_FR")
    gates, ops = circuit._abi()
    total = _rounds(gates)
    L = len(gates)
    nin = len(inputs).bit_length() - 1
    if len(taus) != nin:
        raise ValueError(f"need {nin} taus (one per input variable)")
    outp = np.zeros((2, 4), np.uint64)
    coeffs = np.zeros((total, 3, 4), np.uint64)
    nco = np.zeros(total, np.uint8)
    ch = np.zeros((total, 4), np.uint64)
    claims = np.zeros((max(2 * (L - 1), 1), 4), np.uint64)
    ins = np.zeros((2, 4), np.uint64)
    com = np.zeros((1, 12), np.uint64)
    prf = np.zeros((max(2 * nin, 1), 12), np.uint64)
    g2 = np.zeros((max(nin, 1), 24), np.uint64)
    x = as_limbs(inputs)  # Python ints or the C ABI layout uint64[n, 4], as on the plain path
    _call(lib().zk_gkr_circuit_prove_kzg(ctx.h, REPR_CANONICAL, L, ptr(gates), ptr(ops), ptr(x), len(inputs),
                                         ptr(as_limbs([int(t) for t in taus])), ptr(outp), ptr(coeffs), ptr(nco),
                                         ptr(ch), ptr(claims), ptr(ins), ptr(com), ptr(prf), ptr(g2)))
    polys, chal = _layer_rounds(gates, coeffs, nco, ch, circuit.field)
    cl = to_ints(claims[: 2 * (L - 1)])
    opened = tuple(to_ints(ins))
    pts = _points(prf[: 2 * nin])
    kp = KzgProof(_points(com)[0], (pts[:nin], pts[nin:]), opened, _g2_points(g2[:nin]))
    return GkrCircuitProof(to_ints(outp), polys, [(cl[2 * i], cl[2 * i + 1]) for i in range(L - 1)], opened, chal, kp)


def _verify_kzg(proof: GkrCircuitProof, circuit: Circuit, gates, ops, coeffs, nco, claims) -> bool:
    from .kzg import _g1_array, _g2_array

    kp = proof.input_proof
    nin = (2 * int(gates[0])).bit_length() - 1
    if circuit.field != Field.BLS12_381_FR or len(kp.proof) != 2 or any(len(q) != nin for q in kp.proof) \
            or len(kp.g2_taus) != nin:
        return False
    ok = C.c_int(0)
    _call(lib().zk_gkr_circuit_verify_kzg(REPR_CANONICAL, len(gates), ptr(gates), ptr(ops),
                                          ptr(as_limbs(proof.output_poly)), ptr(coeffs), ptr(nco), ptr(claims),
                                          ptr(as_limbs(list(kp.opened_evals))), ptr(_g1_array([kp.commitment])),
                                          ptr(_g1_array(list(kp.proof[0]) + list(kp.proof[1]))),
                                          ptr(_g2_array(kp.g2_taus)), C.byref(ok)))
    return bool(ok.value)


def verify(proof: GkrCircuitProof, circuit: Circuit, inputs: list[int] | None = None) -> bool:  # :128-227
    """gkr::verify. With an input-layer KZG proof (BLS12-381 Fr) the two
    pairing checks use proof.input_proof.g2_taus, as the reference does
    (gkr_protocol.rs:167,175): that setup must come from a trusted source the
    verifier holds. Taken from an untrusted prover it makes the check unsound
    (a prover who picks its own setup can satisfy both pairings). Inputs, when
    given, are checked as well: their MLE evaluations at the final points must
    equal the opened values (without a KZG proof they are the only check of
    the input layer)."""
    gates, ops = circuit._abi()
    total = _rounds(gates)
    flat = [p for layer in proof.proof_polynomials for p in layer]
    if len(flat) != total:
        return False
    coeffs = np.zeros((max(total, 1), 3, 4), np.uint64)
    nco = np.zeros(max(total, 1), np.uint8)
    for k, poly in enumerate(flat):
        c = poly.coefficient
        if len(c) > 3:
            return False
        nco[k] = len(c)
        if c:
            coeffs[k, : len(c)] = as_limbs(c)
    L = len(gates)
    cl = [v for pair in proof.claimed_evaluations for v in pair]
    if len(cl) != 2 * (L - 1):
        return False
    claims = as_limbs(cl) if cl else np.zeros((1, 4), np.uint64)
    if proof.input_proof is not None:  # the reference's verifier: KZG checks, no inputs needed
        if not _verify_kzg(proof, circuit, gates, ops, coeffs, nco, claims):
            return False
        if inputs is None:
            return True
        if tuple(proof.input_evaluations) != tuple(proof.input_proof.opened_evals):
            return False
    x = as_limbs([int(v) for v in inputs]) if inputs is not None else None
    ok = C.c_int(0)
    _call(lib().zk_gkr_circuit_verify(int(circuit.field), REPR_CANONICAL, L, ptr(gates), ptr(ops),
                                      ptr(x) if x is not None else None, len(inputs) if inputs is not None else
                                      2 * int(gates[0]), ptr(as_limbs(proof.output_poly)), ptr(coeffs), ptr(nco),
                                      ptr(claims), ptr(as_limbs(list(proof.input_evaluations))), C.byref(ok)))
    return bool(ok.value)
