"""The GKR-driver oracle (oracle/gkr_oracle.py) against the known answers the
reference's own tests hold (gkr/src/gkr_circuit.rs:146-257,
gkr/src/gkr_protocol.rs:343-571). CPU only."""
from __future__ import annotations

import gkr_oracle as go
import pyoracle as po

BN254_FQ, BLS_FR = 1, 2
A, M = go.ADD, go.MUL


def test_it_evaluates_the_circuit_correctly():  # gkr_circuit.rs:151-186 (ark_bn254::Fq)
    p = po.MODULI[BN254_FQ]
    ev = go.circuit_evaluate(p, [[M, M, M, M], [A, A], [A]], [5, 2, 2, 4, 10, 0, 3, 3])
    assert ev == [[10, 8, 0, 9], [18, 9], [27]]


def test_it_returns_right_w_polys():  # :188-202
    p = po.MODULI[BN254_FQ]
    assert go.circuit_evaluate(p, [[A, M, A, M]], [1, 2, 3, 4, 5, 6, 7, 8]) == [[3, 12, 11, 56]]


def test_add_i_and_mul_i_polys():  # :204-256
    assert go.get_add_mul_i([A], A) == [0, 1, 0, 0, 0, 0, 0, 0]
    assert go.get_add_mul_i([M], A) == [0] * 8
    assert go.get_add_mul_i([A], M) == [0] * 8
    assert go.get_add_mul_i([M], M) == [0, 1, 0, 0, 0, 0, 0, 0]


def test_wiring_positions_two_and_four_gates():  # gate_to_bits :67-104
    assert go.gate_to_bits(2) == [0b0_00_01, 0b1_10_11]
    assert go.gate_to_bits(4) == [(i << 6) | (2 * i << 3) | (2 * i + 1) for i in range(4)]
    assert go.bits_for_gates(4) == 8


def test_tensor_add_mul():  # gkr_protocol.rs:362-420
    p = po.MODULI[BLS_FR]
    assert po.tensor_add_mul(p, [0, 2], [0, 3], "add") == [0, 3, 2, 5]
    assert po.tensor_add_mul(p, [0, 3], [0, 0, 0, 2], "add") == [0, 0, 0, 2, 3, 3, 3, 5]
    assert po.tensor_add_mul(p, [0, 2], [0, 3], "mul") == [0, 0, 0, 6]
    assert po.tensor_add_mul(p, [0, 3], [0, 0, 0, 2], "mul") == [0] * 7 + [6]


def test_get_fbc_poly():  # gkr_protocol.rs:422-452
    p = po.MODULI[BLS_FR]
    tabs = go.get_fbc_poly(p, 5, [A], [2, 12], [2, 12])
    assert tabs == [[0, p - 4, 0, 0], [4, 14, 14, 24], [0, 0, 0, 0], [4, 24, 24, 144]]


def test_valid_proving_and_verification():  # gkr_protocol.rs:473-506
    structure = [[A, A, A, A], [M, A], [A]]
    inputs = [5, 2, 2, 4, 10, 0, 3, 3]
    proof = go.prove(BLS_FR, structure, inputs)
    assert go.verify(BLS_FR, proof, structure, inputs)
    assert go.verify(BLS_FR, proof, structure)  # KZG stand-in skipped: the sum-check chain alone holds


def test_verify_invalid_proof():  # gkr_protocol.rs:508-570
    p = po.MODULI[BLS_FR]
    dummy = po.interpolate(p, [0, 1], [10, 5])  # the reference's dummy round polynomial
    proof = {"output_poly": [10, 0], "proof_polynomials": [[dummy] * 2, [dummy] * 4],
             "claimed_evaluations": [(10, 5)], "input_evaluations": (1, 2)}
    assert not go.verify(BLS_FR, proof, [[M, M], [A]])


def test_tampered_claimed_evaluation_rejected():
    structure = [[M, A, M, A], [A, M], [M]]
    inputs = [3, 1, 4, 1, 5, 9, 2, 6]
    proof = go.prove(0, structure, inputs)
    assert go.verify(0, proof, structure, inputs)
    o1, o2 = proof["claimed_evaluations"][0]
    proof["claimed_evaluations"][0] = (o1 + 1, o2)
    assert not go.verify(0, proof, structure, inputs)
