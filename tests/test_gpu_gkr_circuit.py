"""GKR over a layered circuit on the GPU: circuit evaluation,
sparse-wiring layer tables and layer sum-checks on the device, through the C
ABI. Small circuits must equal the dense reference restatement
(oracle/gkr_oracle.py) exactly; a 2^10-input circuit (input-layer sum-check
over 20 variables) must pass the verifier (size-independent property)."""
from __future__ import annotations

import random

import pytest

import gkr_oracle as go

from zk_amd.gkr import Circuit, Operation, prove, verify

pytestmark = pytest.mark.gpu
A, M = go.ADD, go.MUL
OPS = {A: Operation.Add, M: Operation.Mul}


def _circuit(rng: random.Random, depth: int, out_gates: int) -> list[list[str]]:
    return [[rng.choice((A, M)) for _ in range(out_gates << (depth - 1 - i))] for i in range(depth)]


@pytest.mark.parametrize("host_lgl", ["8", "0", "3"])
@pytest.mark.parametrize("field,depth,out_gates", [(2, 3, 1), (0, 3, 1), (1, 4, 2), (2, 5, 1), (0, 1, 1), (0, 1, 2),
                                                   (2, 2, 2), (0, 5, 2)])
def test_device_proof_equals_oracle(monkeypatch, field, depth, out_gates, host_lgl):
    """ZK_CIRCUIT_HOST_LGL: layers with tables of <= 2^this entries run on the
    host (8; the default 9 also runs these circuits entirely there), none (0:
    every layer on the device), or the top ones (3). Every split gives the
    oracle's proof."""
    import zk_amd

    monkeypatch.setenv("ZK_CIRCUIT_HOST_LGL", host_lgl)
    ctx = zk_amd.Context(0)
    try:
        _check_circuit(ctx, field, depth, out_gates)
    finally:
        ctx.close()


def _check_circuit(ctx, field, depth, out_gates):
    rng = random.Random(1000 * field + 10 * depth + out_gates)
    structure = _circuit(rng, depth, out_gates)
    p = go.MODULI[field]
    inputs = [rng.randrange(p) for _ in range(2 * len(structure[0]))]
    want = go.prove(field, structure, inputs)
    circ = Circuit([[OPS[o] for o in layer] for layer in structure], field)
    got = prove(circ, inputs, ctx)
    assert got.output_poly == want["output_poly"]
    assert [[q.coefficient for q in layer] for layer in got.proof_polynomials] == \
        [[list(q) for q in layer] for layer in want["proof_polynomials"]]
    assert got.claimed_evaluations == [tuple(c) for c in want["claimed_evaluations"]]
    assert got.input_evaluations == tuple(want["input_evaluations"])
    assert verify(got, circ, inputs)


def test_reference_circuit(ctx):  # gkr_protocol.rs:473-506
    structure = [[A, A, A, A], [M, A], [A]]
    inputs = [5, 2, 2, 4, 10, 0, 3, 3]
    circ = Circuit([[OPS[o] for o in layer] for layer in structure], 2)
    got = prove(circ, inputs, ctx)
    want = go.prove(2, structure, inputs)
    assert got.output_poly == want["output_poly"] == [58, 0]  # (5+2)(2+4) + (10+0)+(3+3)
    assert verify(got, circ, inputs)


@pytest.mark.parametrize("field", [0, 1, 2])
def test_two_phase_equals_dense_tables(monkeypatch, field):
    """The default layer prover (two phases over tables of L = 2G entries) and
    ZK_CIRCUIT_DENSE=1 (the four L^2 tables, then the generic sum-check) give
    the same proof on a 2^10-input circuit (input layer: 20 sum-check rounds);
    so do every layer on the device (ZK_CIRCUIT_HOST_LGL=0) and every layer on
    the host (10). On the device, layers of 2^9 and 2^10 entries end their
    phases in host rounds (2 and 4 of them) and take w(r_b), w(r_c) from the
    folded tables; the dense route evaluates w on the device (k_mle_eval2)."""
    import zk_amd

    rng = random.Random(5 + field)
    depth = 10
    structure = [[rng.choice((Operation.Add, Operation.Mul)) for _ in range(1 << (depth - 1 - i))] for i in range(depth)]
    p = go.MODULI[field]
    inputs = [rng.randrange(p) for _ in range(1 << depth)]
    circ = Circuit(structure, field)
    proofs = {}
    for mode in ("0", "1", "host0", "host10"):
        monkeypatch.setenv("ZK_CIRCUIT_DENSE", "1" if mode == "1" else "0")
        monkeypatch.setenv("ZK_CIRCUIT_HOST_LGL", mode[4:] if mode.startswith("host") else "8")
        c = zk_amd.Context(0)
        try:
            pr = prove(circ, inputs, c)
            proofs[mode] = ([[q.coefficient for q in layer] for layer in pr.proof_polynomials], pr.claimed_evaluations,
                            pr.input_evaluations, pr.output_poly)
        finally:
            c.close()
    assert proofs["0"] == proofs["1"] == proofs["host0"] == proofs["host10"]


def test_bench_circuit_equals_dense_tables(monkeypatch):
    """bench.py gkr_circuit's workload (4 096 inputs, seed 11, BN254 Fr): the
    default prover (layers of <= 2^9 entries on the host, device layers of 2^10
    .. 2^12 with host-round ends: 4, 2 and 4 of them, and evaluations from the
    folds) equals the dense route (ZK_CIRCUIT_DENSE=1: L^2 tables, evaluations
    by k_mle_eval2) and verifies; limb-array inputs give the same proof."""
    import zk_amd
    from zk_amd.elems import as_limbs

    rng = random.Random(11)
    log_inputs = 12
    structure = [[rng.choice((Operation.Add, Operation.Mul)) for _ in range(1 << (log_inputs - 1 - i))]
                 for i in range(log_inputs)]
    inputs = [rng.randrange(go.MODULI[0]) for _ in range(1 << log_inputs)]
    circ = Circuit(structure, 0)
    got = {}
    for dense in ("0", "1"):
        monkeypatch.setenv("ZK_CIRCUIT_DENSE", dense)
        monkeypatch.delenv("ZK_CIRCUIT_HOST_LGL", raising=False)
        c = zk_amd.Context(0)
        try:
            pr = prove(circ, inputs, c)
            got[dense] = ([[q.coefficient for q in layer] for layer in pr.proof_polynomials], pr.claimed_evaluations,
                          pr.input_evaluations, pr.random_challenges)
            if dense == "0":
                assert verify(pr, circ, inputs)
                pa = prove(circ, as_limbs(inputs), c)
                assert pa.random_challenges == pr.random_challenges and pa.input_evaluations == pr.input_evaluations
        finally:
            c.close()
    assert got["0"] == got["1"]


@pytest.mark.parametrize("field", [0, 2])
def test_large_circuit_verifies(ctx, field):
    rng = random.Random(77 + field)
    depth = 10  # 1024 inputs; input layer: 512 gates, tables of 2^20, 20 rounds
    structure = [[rng.choice((Operation.Add, Operation.Mul)) for _ in range(1 << (depth - 1 - i))] for i in range(depth)]
    p = go.MODULI[field]
    inputs = [rng.randrange(p) for _ in range(1 << depth)]
    circ = Circuit(structure, field)
    proof = prove(circ, inputs, ctx)
    assert proof.output_poly[0] == circ.evaluate(inputs)[-1][0] and proof.output_poly[1] == 0
    assert [len(layer) for layer in proof.proof_polynomials] == [2 * (i + 1) for i in range(depth)]
    assert verify(proof, circ, inputs)
    bad = list(inputs)
    bad[123] = (bad[123] + 1) % p
    assert not verify(proof, circ, bad)


@pytest.mark.parametrize("taus", [[5, 2, 3], [0x1234567, 99, 0xdeadbeefcafef00d]])
def test_reference_circuit_with_input_kzg(ctx, taus):
    """gkr::prove including the input layer's KZG step (gkr_protocol.rs:92-118)
    with caller-fixed taus, on the reference's 8-input circuit (:473-506): every
    field of the proof equals gkr_oracle + kzg_oracle (commit and both
    get_proofs against the Lagrange basis of the taus), and gkr::verify's KZG
    checks (:155-175, two pairings per opening on the host) accept it and
    reject tampered openings, commitments and proofs."""
    import dataclasses

    import kzg_oracle as ko
    import pairing_oracle as pa

    structure = [[A, A, A, A], [M, A], [A]]
    inputs = [5, 2, 2, 4, 10, 0, 3, 3]
    circ = Circuit([[OPS[o] for o in layer] for layer in structure], 2)
    got = prove(circ, inputs, ctx, taus=taus)
    want = go.prove(2, structure, inputs)
    assert [[q.coefficient for q in layer] for layer in got.proof_polynomials] == \
        [[list(q) for q in layer] for layer in want["proof_polynomials"]]
    assert got.claimed_evaluations == [tuple(c) for c in want["claimed_evaluations"]]
    kp = got.input_proof
    basis = ko.get_lagrange_basis(taus)
    assert kp.commitment == ko.commit(inputs, basis)
    assert kp.opened_evals == tuple(want["input_evaluations"])
    assert kp.opened_evals == (ko.open_(inputs, want["final_rb"]), ko.open_(inputs, want["final_rc"]))
    assert list(kp.proof[0]) == ko.get_proof(inputs, kp.opened_evals[0], want["final_rb"], basis)
    assert list(kp.proof[1]) == ko.get_proof(inputs, kp.opened_evals[1], want["final_rc"], basis)
    assert kp.g2_taus == pa.g2_taus(taus)
    assert verify(got, circ)  # no inputs: the verifier trusts only the commitment
    bad_open = dataclasses.replace(kp, opened_evals=(kp.opened_evals[0] + 1, kp.opened_evals[1]))
    assert not verify(dataclasses.replace(got, input_proof=bad_open), circ)
    bad_com = dataclasses.replace(kp, commitment=ko.add(kp.commitment, ko.G1))
    assert not verify(dataclasses.replace(got, input_proof=bad_com), circ)
    bad_prf = dataclasses.replace(kp, proof=(kp.proof[1], kp.proof[0]))
    assert not verify(dataclasses.replace(got, input_proof=bad_prf), circ)
    with pytest.raises(ValueError):
        prove(Circuit([[OPS[o] for o in layer] for layer in structure], 0), inputs, ctx, taus=taus)


def test_input_kzg_accepts_limb_array_inputs(ctx):
    """prove() documents inputs as Python ints or the C ABI's uint64[n, 4]
    limb array; with taus (the KZG path) the array must give the same proof
    as the ints (the KZG path used to int() each row)."""
    from zk_amd.elems import as_limbs

    structure = [[A, A, A, A], [M, A], [A]]
    inputs = [5, 2, 2, 4, 10, 0, 3, 3]
    circ = Circuit([[OPS[o] for o in layer] for layer in structure], 2)
    a = prove(circ, inputs, ctx, taus=[5, 2, 3])
    b = prove(circ, as_limbs(inputs), ctx, taus=[5, 2, 3])
    assert a == b


def test_circuit_with_input_kzg_at_scale(ctx):
    """gkr::prove with the input layer's KZG step on a random 10-layer circuit
    (1 024 inputs, BLS12-381 Fr): gkr::verify — the layer sum-checks and both
    KZG pairing checks, without the inputs — accepts it, and rejects a proof
    whose opened evaluation was changed."""
    import dataclasses
    import random

    rng = random.Random(1024)
    log_in = 10
    structure = [[rng.choice((A, M)) for _ in range(1 << (log_in - 1 - i))] for i in range(log_in)]
    p = 0x73EDA753299D7D483339D80809A1D80553BDA402FFFE5BFEFFFFFFFF00000001
    inputs = [rng.randrange(p) for _ in range(1 << log_in)]
    taus = [rng.randrange(p) for _ in range(log_in)]
    circ = Circuit([[OPS[o] for o in layer] for layer in structure], 2)
    got = prove(circ, inputs, ctx, taus=taus)
    assert verify(got, circ)
    assert verify(got, circ, inputs)
    kp = got.input_proof
    bad = dataclasses.replace(kp, opened_evals=(kp.opened_evals[0], (kp.opened_evals[1] + 1) % p))
    assert not verify(dataclasses.replace(got, input_proof=bad), circ)


def test_default_entropy_taus_like_the_reference(ctx):
    """gkr::prove's default matches the reference's shape (gkr_protocol.rs:92-118):
    a BLS12-381 Fr circuit always gets the input layer's KZG step, over taus
    drawn from entropy (os.urandom here, StdRng::from_entropy there), so two
    proofs of the same circuit carry different setups and commitments but the
    same layer sum-checks, and both verify (without the inputs, and with them);
    taus=None skips the step; a BN254 circuit (whose reference gkr::prove cannot
    build the BLS12-381 KZG) gets no input proof."""
    import dataclasses

    structure = [[A, A, A, A], [M, A], [A]]
    inputs = [5, 2, 2, 4, 10, 0, 3, 3]
    circ = Circuit([[OPS[o] for o in layer] for layer in structure], 2)
    a, b = prove(circ, inputs, ctx), prove(circ, inputs, ctx, taus="entropy")
    for pr in (a, b):
        assert pr.input_proof is not None and len(pr.input_proof.g2_taus) == 3
        assert verify(pr, circ) and verify(pr, circ, inputs)
        assert not verify(pr, circ, [5, 2, 2, 4, 10, 0, 3, 4])  # inputs given: checked against the openings
    assert a.input_proof.g2_taus != b.input_proof.g2_taus and a.input_proof.commitment != b.input_proof.commitment
    assert a.proof_polynomials == b.proof_polynomials and a.input_evaluations == b.input_evaluations
    bad = dataclasses.replace(a.input_proof, proof=(b.input_proof.proof[0], a.input_proof.proof[1]))
    assert not verify(dataclasses.replace(a, input_proof=bad), circ)  # an opening under another setup
    c = prove(circ, inputs, ctx, taus=None)
    assert c.input_proof is None and c.proof_polynomials == a.proof_polynomials and verify(c, circ, inputs)
    bn = prove(Circuit([[OPS[o] for o in layer] for layer in structure], 0), inputs, ctx)
    assert bn.input_proof is None and verify(bn, Circuit([[OPS[o] for o in layer] for layer in structure], 0), inputs)
    with pytest.raises(ValueError):
        prove(circ, inputs, ctx, taus="urandom")
