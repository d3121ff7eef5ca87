"""The KZG oracle (oracle/kzg_oracle.py) against the reference's own KZG tests
(pcs/src/kzg_pcs/kzg.rs:214-464) and the BLS12-381 group parameters. CPU only."""
from __future__ import annotations

import kzg_oracle as ko

R = ko.R
TAUS = [5, 2, 3]
EVALS = [0, 4, 0, 4, 0, 4, 3, 7]


def test_generator_on_curve_and_of_order_r():
    assert ko.on_curve(ko.G1)
    assert ko.mul(R - 1, ko.G1) == ko.neg(ko.G1)  # (r-1) G = -G, i.e. r G = O
    assert ko.add(ko.mul(R - 1, ko.G1), ko.G1) is None


def test_blow_up_poly():  # :222-231
    assert ko.blow_up_poly([0, 4], 4) == [0, 4, 0, 4]


def test_get_lagrange_basis():  # :233-255
    want = [(-8) % R, 12, 16, (-24) % R, 10, (-15) % R, (-20) % R, 30]
    assert ko.lagrange_scalars(TAUS) == want
    assert ko.get_lagrange_basis(TAUS) == [ko.mul(x, ko.G1) for x in want]


def test_evaluate_poly_with_l_basis_and_commit():  # :257-281, :316-341
    basis = ko.get_lagrange_basis(TAUS)
    assert ko.commit(EVALS, basis) == ko.mul(42, ko.G1)


def test_get_remainder_and_quotient():  # :283-314
    poly = [(-72) % R, (-68) % R, (-54) % R, (-50) % R]
    assert ko.get_remainder(poly, 4) == [0, 4]
    assert ko.get_quotient(poly)[0] == 18


def test_open_and_get_proof():  # :343-400
    basis = ko.get_lagrange_basis(TAUS)
    point = [6, 4, 0]
    v = ko.open_(EVALS, point)
    assert v == 72
    assert ko.get_proof(EVALS, v, point, basis) == [ko.mul(x, ko.G1) for x in (6, 18, 4)]
