"""Pin the oracle: the reference's own known-answer tests, public Keccak
vectors, hashlib's SHA3 (same permutation), agreement of the two independent
restatements (C and Python), and the committed golden vectors."""
from __future__ import annotations

import hashlib

import numpy as np
import pytest

import coracle as co
import pyoracle as po
from conftest import h2i

FQ = 1  # the reference's sum_check / multilinear tests use ark_bn254::Fq
P_FQ = po.MODULI[FQ]


# --- Keccak / transcript ------------------------------------------------------
def test_keccak_public_vectors():
    assert po.keccak256(b"").hex() == "c5d2460186f7233c927e7db2dcc703c0e500b653ca82273b7bfad8045d85a470"
    assert po.keccak256(b"abc").hex() == "4e03657aea45a94fc7d47ba826c8d667c0d1e6e33a64a036ec44f58fa12d6c45"
    assert co.keccak256(b"").hex() == po.keccak256(b"").hex()


@pytest.mark.parametrize("n", [0, 1, 71, 135, 136, 137, 271, 272, 273, 1000])
def test_keccak_permutation_matches_hashlib_sha3(n):
    data = bytes((7 * i + 3) % 256 for i in range(n))
    assert po.sha3_256_via_permutation(data) == hashlib.sha3_256(data).digest()
    assert co.keccak256(data) == po.keccak256(data)


def test_transcript_challenge_is_le_digest_mod_p():
    for f in range(3):
        t = po.Transcript(f)
        t.append(b"zero knowledge")
        d = po.keccak256(b"zero knowledge")
        assert t.get_random_challenge() == int.from_bytes(d, "little") % po.MODULI[f]
        # second challenge hashes the re-absorbed digest (fiat_shamir_transcript.rs:23-29)
        assert t.get_random_challenge() == int.from_bytes(po.keccak256(d), "little") % po.MODULI[f]


def test_from_le_bytes_mod_order_c_oracle():
    L = co.lib()
    for f in range(3):
        for raw in [b"\xff" * 32, bytes(range(32)), b"\x00" * 31 + b"\x80"]:
            buf = np.frombuffer(raw, np.uint8).copy()
            out = np.zeros((1, 4), np.uint64)
            L.or_fe_from_le_bytes_mod_order(f, buf.ctypes.data, 32, out.ctypes.data)
            assert co.from_limbs(out)[0] == int.from_bytes(raw, "little") % po.MODULI[f]


# --- reference known-answer tests --------------------------------------------
def test_kat_partial_evaluate():  # multilinear_polynomial_evaluation.rs:174-186
    assert po.partial_evaluate(P_FQ, [0, 0, 3, 10], 0, 5) == [15, 50]
    assert co.from_limbs(co.partial_evaluate(FQ, co.to_limbs([0, 0, 3, 10]), 0, 5)) == [15, 50]


def test_kat_evaluate():  # multilinear_polynomial_evaluation.rs:189-198
    assert po.evaluate(P_FQ, [0, 0, 3, 10], [5, 1]) == 50
    assert co.evaluate(FQ, co.to_limbs([0, 0, 3, 10]), [5, 1]) == 50


def test_kat_product_and_sum_poly_evaluate():  # composed_polynomial.rs:113-128, 184-207
    ev = lambda t, pt: po.evaluate(P_FQ, t, pt)  # noqa: E731
    assert ev([0, 0, 0, 3], [2, 3]) * ev([0, 0, 0, 2], [2, 3]) % P_FQ == 216
    s = ev([0, 0, 0, 3], [2, 3]) * ev([0, 0, 0, 2], [2, 3]) + ev([0, 0, 0, 4], [2, 3]) * ev([0, 0, 0, 5], [2, 3])
    assert s % P_FQ == 936


def test_kat_sum_poly_partial_evaluate():  # composed_polynomial.rs:210-256
    pe = lambda t: po.partial_evaluate(P_FQ, t, 0, 2)  # noqa: E731
    assert [pe([0, 0, 0, 3]), pe([0, 0, 0, 2])] == [[0, 6], [0, 4]]
    assert [pe([0, 0, 0, 4]), pe([0, 0, 0, 5])] == [[0, 8], [0, 10]]


def test_kat_interpolate_trims():  # univariate_polynomial_dense.rs:186-196
    assert po.interpolate(P_FQ, [0, 1, 2], [2, 4, 6]) == [2, 2]
    assert co.interpolate(FQ, [0, 1, 2], [2, 4, 6]) == [2, 2]
    assert po.interpolate(P_FQ, [0, 1, 2], [0, 0, 0]) == []
    assert co.interpolate(FQ, [0, 1, 2], [0, 0, 0]) == []


def test_kat_gkr_round_poly():  # sum_check_protocol.rs:225-245 -> evaluations (20, 68, 156)
    tabs = [[0, 3, 2, 5], [0, 6, 4, 10], [0, 1, 1, 2], [0, 2, 2, 4]]
    expect = po.interpolate(P_FQ, [0, 1, 2], [20, 68, 156])
    assert po.gkr_round_poly(P_FQ, tabs) == expect == co.interpolate(FQ, [0, 1, 2], [20, 68, 156])


def test_ref_gkr_prover_and_verifier():  # sum_check_protocol.rs:247-269
    tabs = [[0, 0, 0, 2], [0, 0, 0, 3], [0, 0, 0, 2], [0, 0, 0, 3]]
    polys, cs, _ = po.gkr_prove(FQ, 12, tabs, po.Transcript(FQ))
    ok, _, _ = po.gkr_verify(FQ, polys, cs, po.Transcript(FQ))
    assert ok
    ok2, _, _ = co.gkr_verify(FQ, polys, cs, co.Transcript())
    assert ok2


def test_ref_invalid_proof_doesnt_verify():  # sum_check_protocol.rs:207-222
    ev = [0, 3, 2, 5]
    assert po.verify(FQ, ev, [[3, 9], [1, 2]], 20) is False
    rp = np.array([co.to_limbs([3, 9]), co.to_limbs([1, 2])])
    assert co.verify(FQ, co.to_limbs(ev), rp, 20) == 0


def test_ref_valid_proving_small():
    ev = [0, 0, 0, 2, 0, 10, 0, 17]  # sum_check_benchmark.rs:11-20
    polys, cs, _ = po.prove(FQ, ev)
    assert cs == 29 and po.verify(FQ, ev, polys, cs)


def test_verify_panic_cases_c_oracle():
    ev = co.to_limbs([1, 2, 3, 4])
    polys, cs, _ = po.prove(FQ, [1, 2, 3, 4])
    rp = np.array([co.to_limbs(p) for p in polys])
    assert co.verify(FQ, ev, rp, cs) == 1
    assert co.verify(FQ, ev, rp[:1], cs) == -1  # evaluate() length mismatch panics
    assert co.verify(FQ, ev, rp[:, :1], cs) in (0, -1)  # 1-element polys: sum check first


# --- agreement of the two restatements ----------------------------------------
@pytest.mark.parametrize("field", [0, 1, 2])
def test_c_and_python_oracles_agree(field):
    ev = po.synth(field, 11, 0, 0, 64)
    assert co.from_limbs(co.synth(field, 11, 0, 0, 64)) == ev
    polys, cs, _ = po.prove(field, ev)
    rp, cc = co.prove(field, co.to_limbs(ev))
    assert cc == cs and [co.from_limbs(x) for x in rp] == polys
    tabs = [po.synth(field, 12, t, 0, 64) for t in range(4)]
    p1, _, c1 = po.gkr_prove(field, 0, tabs, po.Transcript(field))
    p2, c2 = co.gkr_prove(field, [co.to_limbs(t) for t in tabs], co.Transcript())
    assert p1 == p2 and c1 == c2
    P = po.MODULI[field]
    for bit in range(6):
        r = po.synth(field, 13, 0, bit, 1)[0]
        assert co.from_limbs(co.partial_evaluate(field, co.to_limbs(ev), bit, r)) == po.partial_evaluate(P, ev, bit, r)


def test_gkr_final_claim_is_sumpoly_at_challenges():
    f = 0
    P = po.MODULI[f]
    tabs = [po.synth(f, 21, t, 0, 32) for t in range(4)]
    polys, _, chal = po.gkr_prove(f, 0, tabs, po.Transcript(f))
    claim = (po.uni_evaluate(P, polys[0], 0) + po.uni_evaluate(P, polys[0], 1)) % P
    ok, fin, vch = po.gkr_verify(f, polys, claim, po.Transcript(f))
    e = [po.evaluate(P, t, chal) for t in tabs]
    assert ok and vch == chal and fin == (e[0] * e[1] + e[2] * e[3]) % P


# --- golden vectors -------------------------------------------------------------
def test_golden_keccak_and_transcript(golden):
    for v in golden["keccak256"]:
        assert po.keccak256(bytes.fromhex(v["msg_hex"])).hex() == v["digest"]
    for v in golden["transcript"]:
        t = co.Transcript()
        t.append(v["preimage"].encode())
        assert [t.get_random_challenge(v["field"]), t.get_random_challenge(v["field"])] == [
            h2i(x) for x in v["challenges"]
        ]


def test_golden_sumcheck_12(golden):
    for g in golden["sumcheck_prove_12"]:
        s = g["input"]
        tab = co.synth(s["field"], s["seed"], s["table"], 0, 1 << s["nvars"])
        assert hashlib.sha256(tab.astype("<u8").tobytes()).hexdigest() == s["sha256"]
        rp, cs = co.prove(s["field"], tab)
        assert cs == h2i(g["claimed_sum"])
        assert [co.from_limbs(x) for x in rp] == [[h2i(a), h2i(b)] for a, b in g["round_polys"]]


@pytest.mark.parametrize("fast", [False, True])
def test_golden_gkr_10(golden, fast):  # fast: the fused OpenMP restatement, same transcript
    for g in golden["gkr_prove_10"]:
        tabs = []
        for s in g["inputs"]:
            tab = co.synth(s["field"], s["seed"], s["table"], 0, 1 << s["nvars"])
            assert hashlib.sha256(tab.astype("<u8").tobytes()).hexdigest() == s["sha256"]
            tabs.append(tab)
        f = g["inputs"][0]["field"]
        polys, chal = co.gkr_prove(f, tabs, co.Transcript(), fast=fast)
        assert polys == [[h2i(c) for c in p] for p in g["round_polys"]]
        assert chal == [h2i(c) for c in g["challenges"]]


@pytest.mark.parametrize("fast", [False, True])
def test_golden_gkr_ref_2var(golden, fast):
    g = golden["gkr_ref_2var"]
    polys, chal = co.gkr_prove(g["field"], [co.to_limbs(t) for t in g["tables"]], co.Transcript(), fast=fast)
    assert polys == [[h2i(c) for c in p] for p in g["round_polys"]]
    assert chal == [h2i(c) for c in g["challenges"]]


def test_oracle_scale_and_binop():  # multilinear_polynomial_evaluation.rs:93-97, :113-151 (zip)
    p = po.MODULI[0]
    assert po.scale(p, [0, 1, p - 1], 3) == [0, 3, p - 3]
    assert po.binop(p, [1, 2, 3, 4], [5, 6], "add") == [6, 8]
    assert po.binop(p, [1, 2], [5, 6, 7, 8], "sub") == [p - 4, p - 4]
    assert po.binop(p, [2, 3], [4, 5], "mul") == [8, 15]


@pytest.mark.slow
def test_ref_port_pins_large_fixture():
    """tests/golden/large.json was written by the fused restatement
    (or_gkr_prove_fast). The reference-faithful port (or_gkr_prove: the
    allocation-per-round algorithm of sum_check_protocol.rs:86-166) reproduces
    the committed 23-variable fixture — round polynomials, challenges and the
    proof blob digest (pyoracle's independent blob writer) — so the full-size
    fixtures do not rest on the fast restatement alone (bench.py's cpu_baseline
    does the same at 24 variables on the GPU box)."""
    import json
    import os

    fix = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "large.json")))["bn254_fr_23_s3"]
    n, seed, field = fix["nvars"], fix["seed"], fix["field"]
    tabs = [co.synth(field, seed, t, 0, 1 << n) for t in range(4)]
    polys, chal = co.gkr_prove(field, tabs, co.Transcript())
    del tabs
    assert polys == [[h2i(c) for c in p] for p in fix["round_polys"]]
    assert chal == [h2i(c) for c in fix["challenges"]]
    c = polys[0] + [0] * (3 - len(polys[0]))
    claimed = (2 * c[0] + c[1] + c[2]) % po.MODULI[field]  # s(0) + s(1)
    assert claimed == h2i(fix["claimed_sum"])
    blob = po.proof_blob(po.BLOB_GKR, field, claimed, polys)
    assert po.keccak256(blob).hex() == fix["blob_keccak256"]


@pytest.mark.slow
def test_ref_port_equals_fast_restatement_21():
    """The two restatements agree above the golden sizes (21 variables, every
    step kind of the fast schedule)."""
    tabs = [co.synth(0, 9, t, 0, 1 << 21) for t in range(4)]
    assert co.gkr_prove(0, tabs, co.Transcript()) == co.gkr_prove(0, tabs, co.Transcript(), fast=True)
