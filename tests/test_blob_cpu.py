"""Proof blob: the library's serialiser / parser / blob
verifier against an independent writer of the same format in the Python
oracle (test infrastructure). Host-only entry points: no GPU needed.
"""
from __future__ import annotations

import pytest

import coracle as co
import pyoracle as po

import zk_amd
from zk_amd import GkrProof, Proof, Transcript, UnivariatePoly, blob_info, gkr_verify_blob, keccak256
from zk_amd._lib import ZK_BLOB_GKR, ZK_BLOB_SUMCHECK
from zk_amd.elems import to_ints

FIELDS = [0, 1, 2]


def _gkr_oracle(field: int, n: int, seed: int = 29):
    tabs = [co.synth(field, seed, t, 0, 1 << n) for t in range(4)]
    claimed = sum(int(a) * int(s) + int(m) * int(q) for a, s, m, q in zip(*[to_ints(t) for t in tabs]))
    polys, chal = co.gkr_prove(field, tabs, co.Transcript())
    return [list(p) for p in polys], claimed % zk_amd.modulus(field), list(chal)


def test_keccak256_public_vectors():
    assert keccak256(b"").hex() == "c5d2460186f7233c927e7db2dcc703c0e500b653ca82273b7bfad8045d85a470"
    assert keccak256(b"abc").hex() == "4e03657aea45a94fc7d47ba826c8d667c0d1e6e33a64a036ec44f58fa12d6c45"
    assert keccak256(b"x" * 1000) == po.keccak256(b"x" * 1000)


@pytest.mark.parametrize("field", FIELDS)
def test_gkr_blob_matches_independent_writer_and_verifies(field):
    polys, claimed, chal = _gkr_oracle(field, 9)
    proof = GkrProof([UnivariatePoly(p, field) for p in polys], claimed, chal)
    blob = proof.to_bytes()
    assert blob == po.proof_blob(po.BLOB_GKR, field, claimed, polys)
    assert blob_info(blob) == (ZK_BLOB_GKR, field, 9)
    back = GkrProof.from_bytes(blob)
    assert [p.coefficient for p in back.proof_polynomials] == polys and back.claimed_sum == claimed
    v = gkr_verify_blob(blob, Transcript(field))
    assert v.verified and v.random_challenges == chal
    ok, fin, ch = po.gkr_verify(field, polys, claimed, po.Transcript(field))
    assert ok and v.final_claimed_sum == fin


def test_gkr_blob_of_trimmed_and_empty_round_polys():
    polys = [[5, 7, 0][:2], [], [3]]  # trimmed lengths 2, 0, 1 are representable
    blob = GkrProof([UnivariatePoly(p) for p in polys], 12, []).to_bytes(0)
    assert blob == po.proof_blob(po.BLOB_GKR, 0, 12, polys)
    assert [p.coefficient for p in GkrProof.from_bytes(blob).proof_polynomials] == polys


@pytest.mark.parametrize("field", FIELDS)
def test_sumcheck_blob_round_trip(field):
    evals = to_ints(co.synth(field, 31, 0, 0, 1 << 6))
    polys, claimed, _ = po.prove(field, evals)
    blob = Proof(polys, claimed).to_bytes(field)
    assert blob == po.proof_blob(po.BLOB_SUMCHECK, field, claimed, polys)
    assert blob_info(blob) == (ZK_BLOB_SUMCHECK, field, 6)
    back = Proof.from_bytes(blob)
    assert back.proof_polynomials == polys and back.claimed_sum == claimed


def test_tampered_gkr_blob_does_not_verify():
    polys, claimed, _ = _gkr_oracle(0, 6)
    blob = bytearray(GkrProof([UnivariatePoly(p) for p in polys], claimed, []).to_bytes(0))
    blob[12 + 32 + 1] ^= 1  # low byte of round 0's c0
    assert not gkr_verify_blob(bytes(blob), Transcript(0)).verified


def _raises_einval(fn):  # the Python mirror raises ValueError where the C ABI returns ZK_EINVAL
    with pytest.raises(ValueError, match="ZK_EINVAL"):
        fn()


def test_malformed_blobs_rejected():
    polys, claimed, _ = _gkr_oracle(2, 4)
    good = GkrProof([UnivariatePoly(p, 2) for p in polys], claimed, []).to_bytes()
    _raises_einval(lambda: blob_info(b"ZKSQ" + good[4:]))                    # magic
    _raises_einval(lambda: blob_info(good[:4] + b"\x02" + good[5:]))        # version
    _raises_einval(lambda: blob_info(good[:5] + b"\x07" + good[6:]))        # kind
    _raises_einval(lambda: blob_info(good[:6] + b"\x03" + good[7:]))        # field
    _raises_einval(lambda: GkrProof.from_bytes(good[:-1]))                  # truncated
    _raises_einval(lambda: GkrProof.from_bytes(good + b"\x00"))             # trailing bytes
    four = bytearray(good)
    four[44] = 4                                                             # m > 3
    _raises_einval(lambda: GkrProof.from_bytes(bytes(four)))
    big = bytearray(good)
    big[12:44] = (zk_amd.modulus(2)).to_bytes(32, "little")                  # claimed_sum = p
    _raises_einval(lambda: GkrProof.from_bytes(bytes(big)))
    _raises_einval(lambda: Proof.from_bytes(good))                          # wrong kind
