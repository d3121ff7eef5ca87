"""The pairing oracle (oracle/pairing_oracle.py) pinned by the BLS12-381 group
laws and by the reference's KZG verification tests (pcs/src/kzg_pcs/kzg.rs:
402-463). CPU only; each pairing takes ~0.5 s of pure Python."""
from __future__ import annotations

import kzg_oracle as ko
import pairing_oracle as po
import pytest

R = ko.R
TAUS = [5, 2, 3]
EVALS = [0, 4, 0, 4, 0, 4, 3, 7]
POINT = [6, 4, 0]


def test_g2_generator_on_twist_and_of_order_r():
    assert po.g2_on_curve(po.G2)
    assert po.g2_mul(R - 1, po.G2) == po.g2_neg(po.G2)  # r G2 = O
    assert po.g2_add(po.g2_mul(R - 1, po.G2), po.G2) is None
    assert not po.g2_on_curve((po.G2[0], po.f2add(po.G2[1], (1, 0))))


def test_w_representation():
    w = [0, 1] + [0] * 10
    w6 = po.f12pow(w, 6)
    assert po.f12mul(w6, w6) == po.f12([-2, 0, 0, 0, 0, 0, 2, 0, 0, 0, 0, 0])  # w^12 = 2 w^6 - 2
    u = po.embed2((0, 1))
    assert po.f12mul(u, u) == po.f12([-1] + [0] * 11)  # u^2 = -1
    a = po.f12([3, 1, 4, 1, 5, 9, 2, 6, 5, 3, 5, 8])
    assert po.f12conj(po.f12conj(a)) == a


def test_pairing_non_degenerate_of_order_r_and_bilinear():
    e = po.pairing(ko.G1, po.G2)
    assert e != po.ONE12
    assert po.f12pow(e, R) == po.ONE12
    # e(2P, 3Q) = e(P, Q)^6 = e(6P, Q)
    e23 = po.pairing(ko.mul(2, ko.G1), po.g2_mul(3, po.G2))
    assert e23 == po.f12pow(e, 6)
    assert po.pairing(ko.mul(6, ko.G1), po.G2) == e23
    # e(-P, Q) = e(P, Q)^-1
    assert po.f12mul(po.pairing(ko.neg(ko.G1), po.G2), e) == po.ONE12
    assert po.pairing(None, po.G2) == po.ONE12 and po.pairing(ko.G1, None) == po.ONE12


def _setup():
    basis = ko.get_lagrange_basis(TAUS)
    commitment = ko.commit(EVALS, basis)
    v = ko.open_(EVALS, POINT)
    proof = ko.get_proof(EVALS, v, POINT, basis)
    return commitment, v, proof, po.g2_taus(TAUS)


def test_reference_verify():  # kzg.rs:402-431
    commitment, v, proof, g2t = _setup()
    assert po.verify(commitment, v, proof, POINT, g2t)


def test_reference_dont_verify_invalid_proof():  # kzg.rs:433-463
    commitment, v, _, g2t = _setup()
    assert not po.verify(commitment, v, [ko.G1, ko.G1, ko.G1], POINT, g2t)


def test_verify_panics_on_length_mismatch():  # :104-106
    commitment, v, proof, g2t = _setup()
    with pytest.raises(ValueError):
        po.verify(commitment, v, proof[:2], POINT, g2t)
