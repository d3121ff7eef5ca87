"""GPU parity: the HIP path (through the C ABI) against the oracle, the
golden vectors and the reference's own tests. Bit-exact for every output."""
from __future__ import annotations

import os

import ctypes as C
import hashlib

import numpy as np
import pytest

import coracle as co
import pyoracle as po
from conftest import h2i

import zk_amd
from zk_amd import Field, MultilinearPoly, ProductPoly, SumPoly, Transcript
from zk_amd._lib import check, lib
from zk_amd.context import REPR_MONTGOMERY
from zk_amd.elems import as_limbs, ptr, to_ints

pytestmark = pytest.mark.gpu
FIELDS = [0, 1, 2]


def digest(a: np.ndarray) -> str:
    return hashlib.sha256(np.ascontiguousarray(a, dtype="<u8").tobytes()).hexdigest()


# --- data generation and conversion -------------------------------------------
@pytest.mark.parametrize("field", FIELDS)
def test_device_synth_matches_oracle(ctx, field):
    t = ctx.synth(field, 1000, seed=7, table=2, index0=5, stride=3)
    want = np.concatenate([co.synth(field, 7, 2, 5 + 3 * m, 1) for m in range(1000)])
    assert np.array_equal(t.download(), want)


@pytest.mark.parametrize("field", FIELDS)
def test_upload_download_roundtrip(ctx, field):
    vals = co.synth(field, 3, 0, 0, 777)
    t = ctx.upload(field, vals)
    assert np.array_equal(t.download(), vals)
    mont = t.download(REPR_MONTGOMERY)
    t2 = ctx.upload(field, mont, REPR_MONTGOMERY)
    assert np.array_equal(t2.download(), vals)


def test_non_canonical_input_rejected(ctx):
    p = po.MODULI[0]
    with pytest.raises(ValueError):
        MultilinearPoly([1, p], Field.BN254_FR, ctx).partial_evaluate(0, 3)


# --- MultilinearPoly -------------------------------------------------------------
def test_kat_partial_evaluate(ctx):  # multilinear_polynomial_evaluation.rs:174-186
    poly = MultilinearPoly([0, 0, 3, 10], Field.BN254_FQ, ctx)
    assert poly.partial_evaluate(0, 5).evaluation == [15, 50]


def test_kat_evaluate(ctx):  # multilinear_polynomial_evaluation.rs:189-198
    assert MultilinearPoly([0, 0, 3, 10], Field.BN254_FQ, ctx).evaluate([5, 1]) == 50


@pytest.mark.parametrize("field", FIELDS)
@pytest.mark.parametrize("n", [1, 2, 7, 13])
def test_partial_evaluate_every_bit(ctx, field, n):
    tab = co.synth(field, 40 + n, 0, 0, 1 << n)
    poly = MultilinearPoly(tab, field, ctx)
    for bit in range(n):
        r = po.synth(field, 41, 1, bit, 1)[0]
        assert np.array_equal(poly.partial_evaluate(bit, r).limbs, co.partial_evaluate(field, tab, bit, r)), bit


def test_fold_20var_golden(ctx, golden):  # BASELINE config 2
    g = golden["fold_20"]
    s = g["input"]
    tab = co.synth(s["field"], s["seed"], s["table"], 0, 1 << s["nvars"])
    assert digest(tab) == s["sha256"]
    out = MultilinearPoly(tab, s["field"], ctx).partial_evaluate(0, h2i(g["r"]))
    assert digest(out.limbs) == g["output_sha256"]


@pytest.mark.parametrize("field", FIELDS)
def test_device_resident_fold(ctx, field):
    n = 16
    d_in = ctx.synth(field, 1 << n, seed=9, table=0)
    d_out = ctx.alloc(field, 1 << (n - 1))
    r = po.synth(field, 9, 5, 0, 1)[0]
    check(lib().zk_dev_mle_partial_evaluate(ctx.h, field, d_in.ptr, n, 0, 0, ptr(as_limbs([r])), d_out.ptr))
    want = co.partial_evaluate(field, co.synth(field, 9, 0, 0, 1 << n), 0, r)
    assert np.array_equal(d_out.download(), want)


@pytest.mark.parametrize("field", FIELDS)
@pytest.mark.parametrize("n", [0, 1, 5, 12])
def test_evaluate(ctx, field, n):
    tab = co.synth(field, 50, 0, 0, 1 << n)
    pt = po.synth(field, 51, 0, 0, n)
    assert MultilinearPoly(tab, field, ctx).evaluate(pt) == co.evaluate(field, tab, pt)


def test_evaluate_wrong_point_length_panics_like_reference(ctx):
    with pytest.raises(ValueError):
        MultilinearPoly([1, 2, 3, 4], Field.BN254_FR, ctx).evaluate([1])


def test_sum_poly_evaluate_and_partial_evaluate(ctx):  # composed_polynomial.rs:184-256
    sp = SumPoly([
        ProductPoly([[0, 0, 0, 3], [0, 0, 0, 2]], Field.BN254_FQ, ctx),
        ProductPoly([[0, 0, 0, 4], [0, 0, 0, 5]], Field.BN254_FQ, ctx),
    ])
    assert sp.evaluate([2, 3]) == 936
    pe = sp.partial_evaluate(2)
    got = [[m.evaluation for m in pp.evaluation] for pp in pe.polys]
    assert got == [[[0, 6], [0, 4]], [[0, 8], [0, 10]]]
    assert ProductPoly([[0, 0, 0, 3], [0, 0, 0, 2]], Field.BN254_FQ, ctx).evaluate([2, 3]) == 216


# --- plain sum-check ---------------------------------------------------------------
@pytest.mark.parametrize("field", FIELDS)
def test_prove_12var_golden(ctx, golden, field):  # BASELINE config 1
    g = golden["sumcheck_prove_12"][field]
    s = g["input"]
    tab = co.synth(s["field"], s["seed"], s["table"], 0, 1 << s["nvars"])
    proof = zk_amd.prove(MultilinearPoly(tab, field, ctx))
    assert proof.claimed_sum == h2i(g["claimed_sum"])
    assert proof.proof_polynomials == [[h2i(a), h2i(b)] for a, b in g["round_polys"]]
    assert zk_amd.verify(MultilinearPoly(tab, field, ctx), proof)


@pytest.mark.parametrize("n", [0, 1, 2, 9])
def test_prove_small_vs_oracle(ctx, n):
    tab = co.synth(2, 60 + n, 0, 0, 1 << n)
    proof = zk_amd.prove(MultilinearPoly(tab, 2, ctx))
    rp, cs = co.prove(2, tab)
    assert proof.claimed_sum == cs
    assert proof.proof_polynomials == [co.from_limbs(x) for x in rp]
    assert zk_amd.verify(MultilinearPoly(tab, 2, ctx), proof)


def test_reference_valid_proving_and_verification(ctx, golden):  # sum_check_protocol.rs:194-204
    n = 20
    poly = MultilinearPoly(np.tile(np.array([10, 0, 0, 0], np.uint64), (1 << n, 1)), Field.BN254_FQ, ctx)
    proof = zk_amd.prove(poly)
    assert proof.claimed_sum == h2i(golden["sumcheck_const10_20"]["claimed_sum"])
    assert proof.proof_polynomials == [[10 << (n - 1 - k)] * 2 for k in range(n)]
    assert zk_amd.verify(poly, proof) is True


def test_reference_invalid_proof_doesnt_verify(ctx):  # sum_check_protocol.rs:207-222
    poly = MultilinearPoly([0, 3, 2, 5], Field.BN254_FQ, ctx)
    assert zk_amd.verify(poly, zk_amd.Proof([[3, 9], [1, 2]], 20)) is False


def test_verify_rejects_tampering(ctx):
    tab = co.synth(0, 70, 0, 0, 1 << 10)
    poly = MultilinearPoly(tab, 0, ctx)
    proof = zk_amd.prove(poly)
    p = po.MODULI[0]
    bad = zk_amd.Proof([list(x) for x in proof.proof_polynomials], proof.claimed_sum)
    bad.proof_polynomials[4][0] = (bad.proof_polynomials[4][0] + 1) % p
    bad.proof_polynomials[4][1] = (bad.proof_polynomials[4][1] - 1) % p  # sum still matches
    assert zk_amd.verify(poly, bad) is False
    assert zk_amd.verify(poly, zk_amd.Proof(proof.proof_polynomials, (proof.claimed_sum + 1) % p)) is False
    with pytest.raises(ValueError):  # too few rounds: evaluate() panics
        zk_amd.verify(poly, zk_amd.Proof(proof.proof_polynomials[:-1], proof.claimed_sum))


# --- GKR sum-check --------------------------------------------------------------------
def _sumpoly(tabs, field, ctx):
    return SumPoly([ProductPoly([tabs[0], tabs[1]], field, ctx), ProductPoly([tabs[2], tabs[3]], field, ctx)])


def test_kat_gkr_round_poly(ctx):  # sum_check_protocol.rs:225-245: evaluations (20, 68, 156)
    tabs = [[0, 3, 2, 5], [0, 6, 4, 10], [0, 1, 1, 2], [0, 2, 2, 4]]
    proof = zk_amd.gkr_prove(0, _sumpoly(tabs, Field.BN254_FQ, ctx), Transcript(Field.BN254_FQ))
    assert proof.proof_polynomials[0].coefficient == po.interpolate(po.MODULI[1], [0, 1, 2], [20, 68, 156])


def test_reference_gkr_prover_and_verifier(ctx, golden):  # sum_check_protocol.rs:247-269
    g = golden["gkr_ref_2var"]
    proof = zk_amd.gkr_prove(12, _sumpoly(g["tables"], Field.BN254_FQ, ctx), Transcript(Field.BN254_FQ))
    assert [p.coefficient for p in proof.proof_polynomials] == [[h2i(c) for c in p] for p in g["round_polys"]]
    assert proof.random_challenges == [h2i(c) for c in g["challenges"]]
    assert proof.claimed_sum == 12
    v = zk_amd.gkr_verify(proof.proof_polynomials, proof.claimed_sum, Transcript(Field.BN254_FQ))
    assert v.verified is True


@pytest.mark.parametrize("field", FIELDS)
def test_gkr_prove_10var_golden(ctx, golden, field):
    g = golden["gkr_prove_10"][field]
    tabs = [co.synth(s["field"], s["seed"], s["table"], 0, 1 << s["nvars"]) for s in g["inputs"]]
    t = Transcript(field)
    proof = zk_amd.gkr_prove(h2i(g["claimed_sum"]), _sumpoly(tabs, field, ctx), t)
    assert [p.coefficient for p in proof.proof_polynomials] == [[h2i(c) for c in p] for p in g["round_polys"]]
    assert proof.random_challenges == [h2i(c) for c in g["challenges"]]
    v = zk_amd.gkr_verify(proof.proof_polynomials, proof.claimed_sum, Transcript(field))
    assert v.verified and v.final_claimed_sum == h2i(g["final_claim"])


@pytest.mark.parametrize("field", FIELDS)
@pytest.mark.parametrize("n", [0, 1, 2, 3, 15])
def test_gkr_prove_vs_oracle(ctx, field, n):
    tabs = [co.synth(field, 80 + n, t, 0, 1 << n) for t in range(4)]
    t1, t2 = Transcript(field), co.Transcript()
    t1.append(b"prefix")
    t2.append(b"prefix")  # caller-owned transcript state carries in
    proof = zk_amd.gkr_prove(0, _sumpoly(tabs, field, ctx), t1)
    polys, chal = co.gkr_prove(field, tabs, t2)
    assert [p.coefficient for p in proof.proof_polynomials] == polys
    assert proof.random_challenges == chal
    assert t1.get_random_challenge() == t2.get_random_challenge(field)  # transcripts end in the same state


def test_gkr_zero_tables_trim_to_empty(ctx):
    tabs = [[0] * 8] * 4
    proof = zk_amd.gkr_prove(0, _sumpoly(tabs, 0, ctx), Transcript(0))
    assert all(p.coefficient == [] for p in proof.proof_polynomials)
    polys, chal = co.gkr_prove(0, [co.to_limbs(t) for t in tabs], co.Transcript())
    assert proof.random_challenges == chal


def test_gkr_extra_products_and_factors_ignored_like_reduce(ctx):
    # reduce() reads products 0,1 and factors 0,1 only (composed_polynomial.rs:52-54,88-99);
    # a 3rd factor raises the degree (4 interpolation points) but not the polynomial.
    f = 0
    tabs = [co.synth(f, 90, t, 0, 64) for t in range(6)]
    sp = SumPoly([ProductPoly([tabs[0], tabs[1], tabs[4]], f, ctx), ProductPoly([tabs[2], tabs[3], tabs[5]], f, ctx),
                  ProductPoly([tabs[5], tabs[4], tabs[0]], f, ctx)])
    proof = zk_amd.gkr_prove(0, sp, Transcript(f))
    polys, chal = co.gkr_prove(f, tabs[:4], co.Transcript())
    assert [p.coefficient for p in proof.proof_polynomials] == polys and proof.random_challenges == chal


@pytest.mark.parametrize("field", FIELDS)
def test_gkr_device_resident_matches_host_api(ctx, field):
    n = 14
    dev = [ctx.synth(field, 1 << n, seed=3, table=t) for t in range(4)]
    arr = (C.c_void_p * 4)(*[d.ptr.value for d in dev])
    coeffs = np.zeros((n, 3, 4), np.uint64)
    nco = np.zeros(n, np.uint8)
    ch = np.zeros((n, 4), np.uint64)
    tr = Transcript(field)
    check(lib().zk_dev_gkr_sumcheck_prove(ctx.h, field, arr, n, 0, ptr(as_limbs([0])), tr.h, ptr(coeffs), ptr(nco),
                                          ptr(ch)))
    tabs = [co.synth(field, 3, t, 0, 1 << n) for t in range(4)]
    polys, chal = co.gkr_prove(field, tabs, co.Transcript())
    assert [to_ints(coeffs[k, : nco[k]]) for k in range(n)] == polys
    assert to_ints(ch) == chal


@pytest.mark.parametrize("field", FIELDS)
def test_gkr_montgomery_repr(ctx, field):
    n = 6
    tabs = [co.synth(field, 5, t, 0, 1 << n) for t in range(4)]
    mont = [ctx.upload(field, t).download(REPR_MONTGOMERY) for t in tabs]
    arr = (C.c_void_p * 4)(*[m.ctypes.data for m in mont])
    coeffs = np.zeros((n, 3, 4), np.uint64)
    nco = np.zeros(n, np.uint8)
    ch = np.zeros((n, 4), np.uint64)
    cs = np.zeros((1, 4), np.uint64)
    tr = Transcript(field)
    check(lib().zk_gkr_sumcheck_prove(ctx.h, field, REPR_MONTGOMERY, arr, n, ptr(np.zeros((1, 4), np.uint64)), tr.h,
                                      ptr(coeffs), ptr(nco), ptr(ch), ptr(cs)))
    polys, chal = co.gkr_prove(field, tabs, co.Transcript())
    # outputs come back in Montgomery form: convert through the device
    got_ch = ctx.upload(field, ch, REPR_MONTGOMERY).to_ints()
    assert got_ch == chal
    for k in range(n):
        if nco[k]:
            assert ctx.upload(field, coeffs[k, : nco[k]], REPR_MONTGOMERY).to_ints() == polys[k]
        else:
            assert polys[k] == []


@pytest.mark.parametrize("field", [0, 2])
def test_gkr_22var_properties(ctx, field):
    """Full-size property check (oracle too slow here): the device proof
    verifies, and the verifier's final claim equals A*S + M*P evaluated at
    the challenges (computed by the device MLE evaluation)."""
    n = 22
    tabs = [co.synth(field, 22, t, 0, 1 << n) for t in range(4)]
    proof = zk_amd.gkr_prove(0, _sumpoly(tabs, field, ctx), Transcript(field))
    p = po.MODULI[field]
    c0 = proof.proof_polynomials[0]
    claim = (c0.evaluate(0) + c0.evaluate(1)) % p
    v = zk_amd.gkr_verify(proof.proof_polynomials, claim, Transcript(field))
    assert v.verified and v.random_challenges == proof.random_challenges
    e = [MultilinearPoly(t, field, ctx).evaluate(proof.random_challenges) for t in tabs]
    assert v.final_claimed_sum == (e[0] * e[1] + e[2] * e[3]) % p


def test_stats_and_timing(ctx):
    n = 12
    tabs = [co.synth(0, 1, t, 0, 1 << n) for t in range(4)]
    ctx.reset_stats()
    ctx.set_timing(True)
    zk_amd.gkr_prove(0, _sumpoly(tabs, 0, ctx), Transcript(0))
    ctx.set_timing(False)
    st = ctx.stats()
    k = st["kernels"]
    # rounds 0 and 1 in one pass over the inputs (k_gkr_d0m, ZK_D0 default), then
    # rounds (2,3) .. (10,11) two per step, each folding by two pending challenges
    # (the first straight from the inputs); these small steps run in one persistent
    # kernel (k_gkr_dtail), except the last ZK_HOST_ROUNDS (default 4) rounds:
    # the tail's last device step hands its tables to the host, which runs them
    assert k["gkr_d0"]["launches"] == 1 and k["gkr_dtail"]["launches"] == 1 and k["gkr_dround"]["launches"] == 0
    assert k["gkr_round0"]["launches"] + k["gkr_round"]["launches"] + k["gkr_round_lanes"]["launches"] == 0
    host_rounds = int(os.environ.get("ZK_HOST_ROUNDS", "4")) & ~1
    nd = (n - 2) // 2 - host_rounds // 2  # double steps on the device
    q = [1 << (n - 4 - 2 * d) for d in range(nd)]  # quads of each double step (Z = 4Q)
    assert k["gkr_dtail"]["alg_bytes"] == 2560 * sum(q)
    assert k["gkr_dtail"]["ms"] > 0 and st["host_syncs"] >= 1 + nd
    assert k["gkr_d0"]["alg_bytes"] == 128 * (1 << n)


@pytest.mark.parametrize("field", FIELDS)
def test_gkr_proof_blob_digest_matches_oracle(ctx, field):
    n = 16
    tabs = [co.synth(field, 37, t, 0, 1 << n) for t in range(4)]
    sp = SumPoly([ProductPoly([tabs[0], tabs[1]], field, ctx), ProductPoly([tabs[2], tabs[3]], field, ctx)])
    claimed = sum(int(a) * int(s) + int(m) * int(q) for a, s, m, q in zip(*[to_ints(t) for t in tabs])) % zk_amd.modulus(field)
    proof = zk_amd.gkr_prove(claimed, sp, Transcript(field), ctx)
    blob = proof.to_bytes(field)
    polys, chal = co.gkr_prove(field, tabs, co.Transcript())
    assert zk_amd.keccak256(blob) == po.keccak256(po.proof_blob(po.BLOB_GKR, field, claimed, [list(p) for p in polys]))
    v = zk_amd.gkr_verify_blob(blob, Transcript(field))
    assert v.verified and v.random_challenges == list(chal)
