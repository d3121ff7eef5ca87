"""CPU restatement of the reference multilinear KZG (pcs/src/kzg_pcs/kzg.rs)
over BLS12-381 G1.

TEST INFRASTRUCTURE ONLY. Literal: `get_lagrange_basis` (:183-212) multiplies
G1 by eq(taus, i) for every hypercube point, `evaluate_poly_with_l_basis_in_g1`
(:131-144) is the naive sum of scalar multiplications, `get_proof` (:59-95)
blows every quotient up to the full size and commits it against the full
basis. Python big-int arithmetic, affine points (None = the point at
infinity); small sizes only. The curve (y^2 = x^3 + 4 over Fq), the generator
and the group order r are the public BLS12-381 parameters used by
ark-bls12-381 0.5.0; the generator is checked on the curve and of order r in
tests/test_kzg_oracle.py.
"""
from __future__ import annotations

from pyoracle import MODULI, evaluate, partial_evaluate, tensor_add_mul

Q = 0x1A0111EA397FE69A4B1BA7B6434BACD764774B84F38512BF6730D2A0F6B0F6241EABFFFEB153FFFFB9FEFFFFFFFFAAAB
R = MODULI[2]  # BLS12-381 Fr
G1 = (0x17F1D3A73197D7942695638C4FA9AC0FC3688C4F9774B905A14E3A3F171BAC586C55E83FF97A1AEFFB3AF00ADB22C6BB,
      0x08B3F481E3AAA0F1A09E30ED741D8AE4FCF5E095D5D00AF600DB18CB2C04B3EDD03CC744A2888AE40CAA232946C5E7E1)
B = 4


def on_curve(P) -> bool:
    if P is None:
        return True
    x, y = P
    return (y * y - x * x * x - B) % Q == 0


def add(P, Pp):
    if P is None:
        return Pp
    if Pp is None:
        return P
    (x1, y1), (x2, y2) = P, Pp
    if x1 == x2:
        if (y1 + y2) % Q == 0:
            return None
        lam = 3 * x1 * x1 * pow(2 * y1, -1, Q) % Q
    else:
        lam = (y2 - y1) * pow(x2 - x1, -1, Q) % Q
    x3 = (lam * lam - x1 - x2) % Q
    return (x3, (lam * (x1 - x3) - y1) % Q)


def neg(P):
    return None if P is None else (P[0], (-P[1]) % Q)


def mul(k: int, P):  # G1Projective::mul_bigint
    acc = None
    k %= R
    while k:
        if k & 1:
            acc = add(acc, P)
        P = add(P, P)
        k >>= 1
    return acc


def generate_bhc(bits: int) -> list[list[int]]:  # :171-181
    return [[(i >> (bits - 1 - j)) & 1 for j in range(bits)] for i in range(1 << bits)]


def lagrange_scalars(taus: list[int]) -> list[int]:  # the scalars of get_lagrange_basis (:183-206)
    out = []
    for layer in generate_bhc(len(taus)):
        e = 1
        for i, bit in enumerate(layer):
            e = e * (taus[i] if bit else (1 - taus[i])) % R
        out.append(e)
    return out


def get_lagrange_basis(taus: list[int]) -> list:  # :183-212
    if len(taus) < 1:
        raise ValueError("Invalid num of vars for lagrange basis")
    return [mul(e, G1) for e in lagrange_scalars(taus)]


def evaluate_poly_with_l_basis_in_g1(evals: list[int], basis: list):  # :131-144
    if len(evals) != len(basis):
        raise ValueError("invalid polynomial or lagrange basis")
    acc = None
    for a, b in zip(evals, basis):
        acc = add(acc, mul(a, b))
    return acc


def blow_up_poly(poly: list[int], bigger_len: int) -> list[int]:  # :163-169
    return tensor_add_mul(R, [1] * (bigger_len // len(poly)), poly, "mul")


def get_quotient(poly: list[int]) -> list[int]:  # :150-161 (bit 0: both halves have the same length)
    e0 = partial_evaluate(R, poly, 0, 0)
    e1 = partial_evaluate(R, poly, 0, 1)
    return [(b - a) % R for a, b in zip(e0, e1)]


def get_remainder(poly: list[int], value: int) -> list[int]:  # :146-148
    return partial_evaluate(R, poly, 0, value)


def commit(evals: list[int], basis: list):  # KZG::commit (:51-53)
    return evaluate_poly_with_l_basis_in_g1(evals, basis)


def open_(evals: list[int], point: list[int]) -> int:  # KZG::open (:55-57)
    return evaluate(R, evals, point)


def get_proof(evals: list[int], opened: int, point: list[int], basis: list) -> list:  # :59-95
    n = len(evals).bit_length() - 1
    cur = [(e - opened) % R for e in evals]
    out = []
    for value in point:
        q = get_quotient(cur)
        qv = len(q).bit_length() - 1
        while qv < n:
            q = blow_up_poly(q, 2 * len(q))
            qv += 1
        out.append(evaluate_poly_with_l_basis_in_g1(q, basis))
        cur = get_remainder(cur, value)
    return out
