"""GKR over a layered circuit: the library's host verifier
(sparse wiring evaluation) against proofs made by the dense reference
restatement (oracle/gkr_oracle.py). CPU only."""
from __future__ import annotations

import random

import pytest

import gkr_oracle as go

from zk_amd import UnivariatePoly
from zk_amd.gkr import Circuit, GkrCircuitProof, Operation, verify

A, M = go.ADD, go.MUL
OPS = {A: Operation.Add, M: Operation.Mul}


def _random_circuit(rng: random.Random, depth: int, out_gates: int) -> list[list[str]]:
    sizes = [out_gates << (depth - 1 - i) for i in range(depth)]  # input -> output
    return [[rng.choice((A, M)) for _ in range(g)] for g in sizes]


def _to_lib(field: int, proof: dict) -> GkrCircuitProof:
    polys = [[UnivariatePoly(list(p), field) for p in layer] for layer in proof["proof_polynomials"]]
    return GkrCircuitProof(list(proof["output_poly"]), polys, [tuple(c) for c in proof["claimed_evaluations"]],
                           tuple(proof["input_evaluations"]), [])


CASES = [  # (field, structure or (depth, out_gates, seed), inputs seed)
    (2, [[A, A, A, A], [M, A], [A]]),  # gkr_protocol.rs:473-506
    (0, (3, 1, 5)),
    (1, (4, 2, 6)),
    (2, (4, 1, 7)),
    (0, (1, 1, 8)),
    (2, (1, 2, 9)),
]


def _case(c):
    field, shape = c
    rng = random.Random(str(shape))
    structure = shape if isinstance(shape, list) else _random_circuit(rng, shape[0], shape[1])
    p = go.MODULI[field]
    n_in = 2 * len(structure[0])
    inputs = [5, 2, 2, 4, 10, 0, 3, 3] if isinstance(shape, list) else [rng.randrange(p) for _ in range(n_in)]
    return field, structure, inputs


@pytest.mark.parametrize("case", CASES)
def test_host_verifier_accepts_oracle_proofs(case):
    field, structure, inputs = _case(case)
    proof = go.prove(field, structure, inputs)
    circ = Circuit([[OPS[o] for o in layer] for layer in structure], field)
    lib_proof = _to_lib(field, proof)
    assert verify(lib_proof, circ, inputs)
    assert verify(lib_proof, circ)  # without the inputs: the sum-check chain alone
    assert circ.evaluate(inputs) == go.circuit_evaluate(go.MODULI[field], structure, inputs)


@pytest.mark.parametrize("case", CASES[:3])
def test_host_verifier_rejects_tampering(case):
    field, structure, inputs = _case(case)
    proof = go.prove(field, structure, inputs)
    circ = Circuit([[OPS[o] for o in layer] for layer in structure], field)
    base = _to_lib(field, proof)
    # a round coefficient
    t = _to_lib(field, proof)
    t.proof_polynomials[-1][0].coefficient[0] += 1
    assert not verify(t, circ, inputs)
    # a claimed evaluation (when there is one)
    if base.claimed_evaluations:
        t = _to_lib(field, proof)
        o1, o2 = t.claimed_evaluations[0]
        t.claimed_evaluations[0] = (o1, o2 + 1)
        assert not verify(t, circ, inputs)
    # the input evaluations: caught by the final claim and, with inputs, by recomputation
    t = _to_lib(field, proof)
    t.input_evaluations = (t.input_evaluations[0] + 1, t.input_evaluations[1])
    assert not verify(t, circ, inputs)
    # the output poly (changes r0 and m0)
    t = _to_lib(field, proof)
    t.output_poly[1] += 1
    assert not verify(t, circ, inputs)
    # a different circuit (flip one gate)
    flipped = [list(layer) for layer in circ.layers]
    flipped[0][0] = Operation.Mul if flipped[0][0] == Operation.Add else Operation.Add
    assert not verify(base, Circuit(flipped, field), inputs)


def test_unsupported_shapes_rejected():
    proof = go.prove(0, [[A, A], [M]], [1, 2, 3, 4])
    lib_proof = _to_lib(0, proof)
    with pytest.raises(ValueError, match="powers of two"):
        verify(lib_proof, Circuit([[Operation.Add] * 3, [Operation.Mul]]))
    with pytest.raises(ValueError, match="half the gates"):
        verify(lib_proof, Circuit([[Operation.Add] * 4, [Operation.Mul]]))
    with pytest.raises(ValueError, match="1 or 2 gates"):
        verify(lib_proof, Circuit([[Operation.Add] * 8, [Operation.Mul] * 4]))
