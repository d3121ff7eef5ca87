"""Mirror of the reference `gkr` crate (gkr/src/gkr_circuit.rs,
gkr/src/gkr_protocol.rs) over the C ABI: a layered circuit, `prove` (circuit
evaluation, per-layer tables and sum-checks on the GPU) and `verify` (host).

Differences from the reference, all forced by SURVEY.md 8(f2)/(f3):
* the input layer is not committed with KZG (row f3); the proof carries the
  two input-MLE evaluations KZG::open would return, and `verify` recomputes
  them from the inputs when they are given;
* only the circuit shape for which the reference's table sizes agree is
  accepted (binary tree, powers of two, 1- or 2-gate output layer);
  anything else raises ValueError (the reference panics or mis-sizes).
"""
from __future__ import annotations

import ctypes as C
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
        self.layers = [[Operation(op) for op in layer] for layer in structure]
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
        gates = np.array([len(layer) for layer in self.layers], np.uint32)
        ops = np.array([int(op) for layer in self.layers for op in layer], np.uint8)
        return gates, ops


@dataclass
class GkrCircuitProof:  # gkr_protocol.rs:23-29 (input_proof -> input_evaluations)
    output_poly: list[int]
    proof_polynomials: list[list[UnivariatePoly]]  # per layer, output layer first
    claimed_evaluations: list[tuple[int, int]]
    input_evaluations: tuple[int, int]
    random_challenges: list[list[int]]


def _rounds(gates: np.ndarray) -> int:
    n = C.c_uint32(0)
    _call(lib().zk_gkr_circuit_rounds(len(gates), ptr(gates), C.byref(n)))
    return n.value


def prove(circuit: Circuit, inputs: list[int], ctx: Context | None = None) -> GkrCircuitProof:  # :31-126
    ctx = ctx or default_context()
    gates, ops = circuit._abi()
    total = _rounds(gates)
    L = len(gates)
    outp = np.zeros((2, 4), np.uint64)
    coeffs = np.zeros((total, 3, 4), np.uint64)
    nco = np.zeros(total, np.uint8)
    ch = np.zeros((total, 4), np.uint64)
    claims = np.zeros((max(2 * (L - 1), 1), 4), np.uint64)
    ins = np.zeros((2, 4), np.uint64)
    x = as_limbs([int(v) for v in inputs])
    _call(lib().zk_gkr_circuit_prove(ctx.h, int(circuit.field), REPR_CANONICAL, L, ptr(gates), ptr(ops), ptr(x),
                                     len(inputs), ptr(outp), ptr(coeffs), ptr(nco), ptr(ch), ptr(claims), ptr(ins)))
    polys, chal, k0 = [], [], 0
    for layer in reversed(range(L)):
        nv = 2 * (2 * int(gates[layer])).bit_length() - 2
        polys.append([UnivariatePoly(to_ints(coeffs[k, : nco[k]]), circuit.field) for k in range(k0, k0 + nv)])
        chal.append(to_ints(ch[k0: k0 + nv]))
        k0 += nv
    cl = to_ints(claims[: 2 * (L - 1)])
    return GkrCircuitProof(to_ints(outp), polys, [(cl[2 * i], cl[2 * i + 1]) for i in range(L - 1)],
                           tuple(to_ints(ins)), chal)


def verify(proof: GkrCircuitProof, circuit: Circuit, inputs: list[int] | None = None) -> bool:  # :128-227
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
    x = as_limbs([int(v) for v in inputs]) if inputs is not None else None
    ok = C.c_int(0)
    _call(lib().zk_gkr_circuit_verify(int(circuit.field), REPR_CANONICAL, L, ptr(gates), ptr(ops),
                                      ptr(x) if x is not None else None, len(inputs) if inputs is not None else
                                      2 * int(gates[0]), ptr(as_limbs(proof.output_poly)), ptr(coeffs), ptr(nco),
                                      ptr(claims), ptr(as_limbs(list(proof.input_evaluations))), C.byref(ok)))
    return bool(ok.value)
