"""CPU restatement of the verifier half of the reference multilinear KZG
(pcs/src/kzg_pcs/kzg.rs): the G2 taus of run_trusted_setup (:35-49) and the
pairing-based KZG::verify (:97-129) over BLS12-381 (ark-bls12-381 0.5.0).

TEST INFRASTRUCTURE ONLY. Written independently of the library's tower code
(csrc/pairing.hpp) so the two check each other:
  * Fq12 is Fq[w] / (w^12 - 2 w^6 + 2) (a flat 12-coefficient polynomial), with
    Fq2 = Fq[u] / (u^2 + 1) embedded by u -> w^6 - 1 (so 1 + u = w^6);
  * lines are evaluated unscaled, y_P - (lambda / w) x_P + (lambda x_T - y_T) / w^3;
  * the final exponentiation is one plain power (q^12 - 1) / r.
Pinned by the group laws (generator on the twist and of order r, bilinearity,
non-degeneracy — tests/test_pairing_oracle.py) and by the reference's KZG tests
(test_verify, test_dont_verify_invalid_proof, kzg.rs:402-463). No GT value is
asserted anywhere in the reference, so pairing *values* are parity unpinned
beyond those properties. Pure Python big integers; a few seconds per pairing.
"""
from __future__ import annotations

from kzg_oracle import G1, Q, R
from kzg_oracle import add as g1_add
from kzg_oracle import mul as g1_mul
from kzg_oracle import neg as g1_neg

X_ABS = 0xD201000000010000  # |x|, x negative

# G2 generator (x0 + x1 u, y0 + y1 u)
G2 = ((0x024AA2B2F08F0A91260805272DC51051C6E47AD4FA403B02B4510B647AE3D1770BAC0326A805BBEFD48056C8C121BDB8,
       0x13E02B6052719F607DACD3A088274F65596BD0D09920B61AB5DA61BBDC7F5049334CF11213945D57E5AC7D055D042B7E),
      (0x0CE5D527727D6E118CC9CDC6DA2E351AADFD9BAA8CBDD3A76D429A695160D12C923AC9CC3BACA289E193548608B82801,
       0x0606C4A02EA734CC32ACD2B02BC28B99CB3E287E85A763AF267492AB572E99AB3F370D275CEC1DA1AAA9075FF05F79BE))
B2 = (4, 4)  # 4 (1 + u)


# ---- Fq2 ----
def f2add(a, b):
    return ((a[0] + b[0]) % Q, (a[1] + b[1]) % Q)


def f2sub(a, b):
    return ((a[0] - b[0]) % Q, (a[1] - b[1]) % Q)


def f2mul(a, b):
    return ((a[0] * b[0] - a[1] * b[1]) % Q, (a[0] * b[1] + a[1] * b[0]) % Q)


def f2neg(a):
    return ((-a[0]) % Q, (-a[1]) % Q)


def f2inv(a):
    n = pow((a[0] * a[0] + a[1] * a[1]) % Q, Q - 2, Q)
    return (a[0] * n % Q, (-a[1]) * n % Q)


def f2scal(a, k):
    return (a[0] * k % Q, a[1] * k % Q)


# ---- G2 on the twist, affine, None = infinity ----
def g2_on_curve(P) -> bool:
    if P is None:
        return True
    x, y = P
    return f2sub(f2mul(y, y), f2add(f2mul(f2mul(x, x), x), B2)) == (0, 0)


def g2_add(P, Pp):
    if P is None:
        return Pp
    if Pp is None:
        return P
    (x1, y1), (x2, y2) = P, Pp
    if x1 == x2:
        if f2add(y1, y2) == (0, 0):
            return None
        lam = f2mul(f2scal(f2mul(x1, x1), 3), f2inv(f2scal(y1, 2)))
    else:
        lam = f2mul(f2sub(y2, y1), f2inv(f2sub(x2, x1)))
    x3 = f2sub(f2sub(f2mul(lam, lam), x1), x2)
    return (x3, f2sub(f2mul(lam, f2sub(x1, x3)), y1))


def g2_neg(P):
    return None if P is None else (P[0], f2neg(P[1]))


def g2_mul(k: int, P):  # G2Projective::mul_bigint of a canonical Fr scalar
    acc = None
    k %= R
    while k:
        if k & 1:
            acc = g2_add(acc, P)
        P = g2_add(P, P)
        k >>= 1
    return acc


# ---- Fq12 = Fq[w] / (w^12 - 2 w^6 + 2) ----
def f12(coeffs):
    return [c % Q for c in coeffs]


ONE12 = [1] + [0] * 11


def f12mul(a, b):
    r = [0] * 23
    for i, x in enumerate(a):
        if x:
            for j, y in enumerate(b):
                r[i + j] += x * y
    for i in range(22, 11, -1):  # w^i = 2 w^(i-6) - 2 w^(i-12)
        c = r[i]
        if c:
            r[i - 6] += 2 * c
            r[i - 12] -= 2 * c
    return [c % Q for c in r[:12]]


def f12pow(a, e: int):
    r = ONE12
    for bit in bin(e)[2:]:
        r = f12mul(r, r)
        if bit == "1":
            r = f12mul(r, a)
    return r


def embed2(a):  # a0 + a1 u -> a0 + a1 (w^6 - 1)
    v = [0] * 12
    v[0] = (a[0] - a[1]) % Q
    v[6] = a[1] % Q
    return v


INV2 = pow(2, Q - 2, Q)
W_INV = f12([0, 0, 0, 0, 0, 1, 0, 0, 0, 0, 0, -INV2])  # w * (w^5 - w^11 / 2) = 1
W_INV3 = f12mul(f12mul(W_INV, W_INV), W_INV)
assert f12mul(W_INV, [0, 1] + [0] * 10) == ONE12


def line(lam, xT, yT, P):
    """y_P - y - lambda (x_P - x) at the untwisted T = (x_T / w^2, y_T / w^3),
    slope lambda / w: y_P - (lambda / w) x_P + (lambda x_T - y_T) / w^3."""
    xP, yP = P
    t1 = f12mul(embed2(f2scal(lam, xP)), W_INV)
    t3 = f12mul(embed2(f2sub(f2mul(lam, xT), yT)), W_INV3)
    out = [(t3[i] - t1[i]) % Q for i in range(12)]
    out[0] = (out[0] + yP) % Q
    return out


def miller_loop(P, Qp):
    f = ONE12
    T = Qp
    for bit in bin(X_ABS)[3:]:
        xT, yT = T
        lam = f2mul(f2scal(f2mul(xT, xT), 3), f2inv(f2scal(yT, 2)))
        f = f12mul(f12mul(f, f), line(lam, xT, yT, P))
        T = g2_add(T, T)
        if bit == "1":
            xT, yT = T
            lam = f2mul(f2sub(Qp[1], yT), f2inv(f2sub(Qp[0], xT)))
            f = f12mul(f, line(lam, xT, yT, P))
            T = g2_add(T, Qp)
    # x < 0: f_{x} = 1 / f_{|x|} up to vertical lines; the q^6-power is the inverse in GT
    return f12conj(f)


def f12conj(a):  # a^(q^6): w^6 -> -w^6 + 2 ... computed as a plain power is too slow; use the automorphism
    # Frobenius^6 fixes Fq and maps w -> -w (w^(q^6) = w * (w^2)^((q^6-1)/2) and
    # w^2 = v is a non-square in Fq6), so a(w) -> a(-w): negate the odd coefficients.
    return [c if i % 2 == 0 else (-c) % Q for i, c in enumerate(a)]


FINAL_EXP = (Q ** 12 - 1) // R
assert (Q ** 12 - 1) % R == 0


def pairing(P, Qp):
    """Bls12_381::pairing(P, Q) as a 12-coefficient polynomial in w."""
    if P is None or Qp is None:
        return ONE12
    return f12pow(miller_loop(P, Qp), FINAL_EXP)


def tower_to_w(c72: list[int]) -> list[int]:
    """The library's Fq12 (c0.c0, c0.c1, c0.c2, c1.c0, c1.c1, c1.c2; each Fq2 as
    (re, im)) -> this module's w-polynomial: c_(i,j) multiplies w^(i + 2j)."""
    out = [0] * 12
    for idx, (i, j) in enumerate([(0, 0), (0, 1), (0, 2), (1, 0), (1, 1), (1, 2)]):
        a, b = c72[2 * idx], c72[2 * idx + 1]
        k = i + 2 * j
        out[k] = (out[k] + a - b) % Q
        out[k + 6] = (out[k + 6] + b) % Q
    return out


def g2_taus(taus: list[int]) -> list:  # run_trusted_setup (:43-46)
    return [g2_mul(t, G2) for t in taus]


def verify(commitment, opened_value: int, proof: list, opening_values: list[int], g2_taus_: list) -> bool:
    """KZG::verify (:97-129), literal: two GT values compared."""
    if len(proof) != len(opening_values):
        raise ValueError("num of quotients in proof not equal to num of opening values")
    lhs = g1_add(commitment, g1_neg(g1_mul(opened_value, G1)))
    lhs_gt = pairing(lhs, G2)
    rhs_gt = ONE12
    for i, a in enumerate(opening_values):
        factor = g2_add(g2_taus_[i], g2_neg(g2_mul(a, G2)))
        rhs_gt = f12mul(rhs_gt, pairing(proof[i], factor))  # GT is written additively in ark
    return lhs_gt == rhs_gt
