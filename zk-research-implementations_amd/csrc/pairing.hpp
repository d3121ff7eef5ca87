// BLS12-381 G2 and the optimal ate pairing, for the verifier half of the
// multilinear KZG (pcs/src/kzg_pcs/kzg.rs:35-49 the G2 taus,
// :97-129 KZG::verify). Host-only: a verification is n + 1 Miller loops and one
// final exponentiation (O(n) work, like gkr_verify), the setup's G2 half is n
// scalar multiplications; nothing here is table-sized.
//
// Tower (the one ark-bls12-381 0.5.0 uses):
//   Fq2  = Fq[u]  / (u^2 + 1)
//   Fq6  = Fq2[v] / (v^3 - xi),  xi = 1 + u
//   Fq12 = Fq6[w] / (w^2 - v)
// G2 is the M-type sextic twist E': y^2 = x^3 + 4 xi over Fq2; the untwist
// (x', y') -> (x' / w^2, y' / w^3) maps it into E(Fq12): y^2 = x^3 + 4.
//
// Pairing: e(P, Q) = f_{|x|, Q}(P)^-1 ^ ((q^12 - 1) / r) with the BLS parameter
// x = -0xd201000000010000 (negative, hence the conjugation after the loop, as
// in ark's Bls12 Miller loop). The Miller loop keeps T on the twist in affine
// coordinates; every line is scaled by xi (in Fq2, killed by the final
// exponentiation) so that it lands in Fq12 as
//   xi * y_P + ((lambda x_T - y_T) v - lambda x_P v^2) w,
// and vertical lines are dropped (they lie in Fq6, killed by the (q^6 - 1)
// factor). Final exponentiation: easy part f^(q^6 - 1) = conj(f) / f, then
// the power (q^6 + 1) / r computed once with a small big-integer routine
// (r | q^4 - q^2 + 1 | q^6 + 1, asserted). The output is the reduced pairing
// value, so it is independent of the line scaling and of the loop's
// coordinate system.
#pragma once
#include <algorithm>
#include <cstdint>
#include <vector>

#include <array>

#include "ec.hpp"

namespace zk {

// ---- Fq2 ---------------------------------------------------------------------
struct Fq2 {
  Fq c0, c1;
};
inline Fq2 fq2_zero() { return {fq_zero(), fq_zero()}; }
inline Fq2 fq2_one() { return {fq_one(), fq_zero()}; }
inline bool fq2_is_zero(const Fq2& a) { return fq_is_zero(a.c0) && fq_is_zero(a.c1); }
inline bool fq2_eq(const Fq2& a, const Fq2& b) { return fq_eq(a.c0, b.c0) && fq_eq(a.c1, b.c1); }
inline Fq2 fq2_add(const Fq2& a, const Fq2& b) { return {fq_add(a.c0, b.c0), fq_add(a.c1, b.c1)}; }
inline Fq2 fq2_sub(const Fq2& a, const Fq2& b) { return {fq_sub(a.c0, b.c0), fq_sub(a.c1, b.c1)}; }
inline Fq2 fq2_neg(const Fq2& a) { return {fq_neg(a.c0), fq_neg(a.c1)}; }
inline Fq2 fq2_dbl(const Fq2& a) { return fq2_add(a, a); }
inline Fq2 fq2_conj(const Fq2& a) { return {a.c0, fq_neg(a.c1)}; }
inline Fq2 fq2_mul(const Fq2& a, const Fq2& b) {  // Karatsuba, u^2 = -1
  const Fq v0 = fq_mul(a.c0, b.c0), v1 = fq_mul(a.c1, b.c1);
  const Fq s = fq_mul(fq_add(a.c0, a.c1), fq_add(b.c0, b.c1));
  return {fq_sub(v0, v1), fq_sub(fq_sub(s, v0), v1)};
}
inline Fq2 fq2_sqr(const Fq2& a) {  // (a0 + a1)(a0 - a1) + 2 a0 a1 u
  return {fq_mul(fq_add(a.c0, a.c1), fq_sub(a.c0, a.c1)), fq_dbl(fq_mul(a.c0, a.c1))};
}
inline Fq2 fq2_mul_fq(const Fq2& a, const Fq& s) { return {fq_mul(a.c0, s), fq_mul(a.c1, s)}; }
inline Fq2 fq2_mul_xi(const Fq2& a) {  // (a0 + a1 u)(1 + u) = (a0 - a1) + (a0 + a1) u
  return {fq_sub(a.c0, a.c1), fq_add(a.c0, a.c1)};
}
inline Fq2 fq2_inv(const Fq2& a) {  // (a0 - a1 u) / (a0^2 + a1^2)
  const Fq t = fq_inv(fq_add(fq_sqr(a.c0), fq_sqr(a.c1)));
  return {fq_mul(a.c0, t), fq_neg(fq_mul(a.c1, t))};
}

// ---- Fq6 ---------------------------------------------------------------------
struct Fq6 {
  Fq2 c0, c1, c2;
};
inline Fq6 fq6_zero() { return {fq2_zero(), fq2_zero(), fq2_zero()}; }
inline Fq6 fq6_one() { return {fq2_one(), fq2_zero(), fq2_zero()}; }
inline bool fq6_eq(const Fq6& a, const Fq6& b) { return fq2_eq(a.c0, b.c0) && fq2_eq(a.c1, b.c1) && fq2_eq(a.c2, b.c2); }
inline Fq6 fq6_add(const Fq6& a, const Fq6& b) { return {fq2_add(a.c0, b.c0), fq2_add(a.c1, b.c1), fq2_add(a.c2, b.c2)}; }
inline Fq6 fq6_sub(const Fq6& a, const Fq6& b) { return {fq2_sub(a.c0, b.c0), fq2_sub(a.c1, b.c1), fq2_sub(a.c2, b.c2)}; }
inline Fq6 fq6_neg(const Fq6& a) { return {fq2_neg(a.c0), fq2_neg(a.c1), fq2_neg(a.c2)}; }
inline Fq6 fq6_mul(const Fq6& a, const Fq6& b) {  // schoolbook, v^3 = xi
  const Fq2 a0b0 = fq2_mul(a.c0, b.c0), a1b1 = fq2_mul(a.c1, b.c1), a2b2 = fq2_mul(a.c2, b.c2);
  const Fq2 a1b2 = fq2_mul(a.c1, b.c2), a2b1 = fq2_mul(a.c2, b.c1);
  const Fq2 a0b1 = fq2_mul(a.c0, b.c1), a1b0 = fq2_mul(a.c1, b.c0);
  const Fq2 a0b2 = fq2_mul(a.c0, b.c2), a2b0 = fq2_mul(a.c2, b.c0);
  return {fq2_add(a0b0, fq2_mul_xi(fq2_add(a1b2, a2b1))), fq2_add(fq2_add(a0b1, a1b0), fq2_mul_xi(a2b2)),
          fq2_add(fq2_add(a0b2, a1b1), a2b0)};
}
inline Fq6 fq6_mul_v(const Fq6& a) { return {fq2_mul_xi(a.c2), a.c0, a.c1}; }  // a * v
inline Fq6 fq6_inv(const Fq6& a) {
  const Fq2 t0 = fq2_sub(fq2_sqr(a.c0), fq2_mul_xi(fq2_mul(a.c1, a.c2)));
  const Fq2 t1 = fq2_sub(fq2_mul_xi(fq2_sqr(a.c2)), fq2_mul(a.c0, a.c1));
  const Fq2 t2 = fq2_sub(fq2_sqr(a.c1), fq2_mul(a.c0, a.c2));
  const Fq2 n = fq2_add(fq2_mul(a.c0, t0), fq2_mul_xi(fq2_add(fq2_mul(a.c2, t1), fq2_mul(a.c1, t2))));
  const Fq2 ni = fq2_inv(n);
  return {fq2_mul(t0, ni), fq2_mul(t1, ni), fq2_mul(t2, ni)};
}

// ---- Fq12 --------------------------------------------------------------------
struct Fq12 {
  Fq6 c0, c1;
};
inline Fq12 fq12_one() { return {fq6_one(), fq6_zero()}; }
inline bool fq12_eq(const Fq12& a, const Fq12& b) { return fq6_eq(a.c0, b.c0) && fq6_eq(a.c1, b.c1); }
inline bool fq12_is_one(const Fq12& a) { return fq12_eq(a, fq12_one()); }
inline Fq12 fq12_mul(const Fq12& a, const Fq12& b) {  // Karatsuba over w^2 = v
  const Fq6 t0 = fq6_mul(a.c0, b.c0), t1 = fq6_mul(a.c1, b.c1);
  const Fq6 s = fq6_mul(fq6_add(a.c0, a.c1), fq6_add(b.c0, b.c1));
  return {fq6_add(t0, fq6_mul_v(t1)), fq6_sub(fq6_sub(s, t0), t1)};
}
inline Fq12 fq12_sqr(const Fq12& a) {  // complex squaring: (a0 + a1 w)^2 = (a0^2 + v a1^2) + 2 a0 a1 w, 2 Fq6 products
  const Fq6 ab = fq6_mul(a.c0, a.c1);
  const Fq6 t = fq6_mul(fq6_add(a.c0, a.c1), fq6_add(a.c0, fq6_mul_v(a.c1)));  // a0^2 + v a1^2 + (1 + v) a0 a1
  return {fq6_sub(fq6_sub(t, ab), fq6_mul_v(ab)), fq6_add(ab, ab)};
}
inline Fq12 fq12_conj(const Fq12& a) { return {a.c0, fq6_neg(a.c1)}; }  // a^(q^6)
inline Fq12 fq12_inv(const Fq12& a) {  // (c0 - c1 w) / (c0^2 - v c1^2)
  const Fq6 t = fq6_inv(fq6_sub(fq6_mul(a.c0, a.c0), fq6_mul_v(fq6_mul(a.c1, a.c1))));
  return {fq6_mul(a.c0, t), fq6_neg(fq6_mul(a.c1, t))};
}
// a^e, e as little-endian u32 limbs (MSB-first square and multiply)
inline Fq12 fq12_pow(const Fq12& a, const std::vector<uint32_t>& e) {
  Fq12 r = fq12_one();
  bool started = false;
  for (size_t i = e.size(); i-- > 0;)
    for (int b = 31; b >= 0; --b) {
      if (started) r = fq12_sqr(r);
      if ((e[i] >> b) & 1u) {
        r = started ? fq12_mul(r, a) : a;
        started = true;
      }
    }
  return r;
}

// ---- small unsigned big integers (u32 limbs, LE) for the exponent -------------
namespace bigu {
using Big = std::vector<uint32_t>;
inline void trim(Big& a) {
  while (!a.empty() && a.back() == 0) a.pop_back();
}
inline Big mul(const Big& a, const Big& b) {
  Big r(a.size() + b.size(), 0);
  for (size_t i = 0; i < a.size(); ++i) {
    uint64_t c = 0;
    for (size_t j = 0; j < b.size(); ++j) {
      const uint64_t t = (uint64_t)a[i] * b[j] + r[i + j] + c;
      r[i + j] = (uint32_t)t;
      c = t >> 32;
    }
    for (size_t k = i + b.size(); c; ++k) {
      const uint64_t t = (uint64_t)r[k] + c;
      r[k] = (uint32_t)t;
      c = t >> 32;
    }
  }
  trim(r);
  return r;
}
inline void add_small(Big& a, uint32_t s) {
  uint64_t c = s;
  for (size_t i = 0; c; ++i) {
    if (i == a.size()) a.push_back(0);
    const uint64_t t = (uint64_t)a[i] + c;
    a[i] = (uint32_t)t;
    c = t >> 32;
  }
}
inline int cmp(const Big& a, const Big& b) {
  const size_t n = std::max(a.size(), b.size());
  for (size_t i = n; i-- > 0;) {
    const uint32_t x = i < a.size() ? a[i] : 0, y = i < b.size() ? b[i] : 0;
    if (x != y) return x < y ? -1 : 1;
  }
  return 0;
}
inline void sub_in(Big& a, const Big& b) {  // a -= b, a >= b
  int64_t br = 0;
  for (size_t i = 0; i < a.size(); ++i) {
    int64_t t = (int64_t)a[i] - (i < b.size() ? b[i] : 0) - br;
    br = t < 0;
    a[i] = (uint32_t)(t + (br << 32));
  }
  trim(a);
}
// bit-serial long division: returns quotient, rem gets the remainder
inline Big divmod(const Big& a, const Big& d, Big& rem) {
  Big q(a.size(), 0);
  rem.clear();
  for (size_t i = a.size() * 32; i-- > 0;) {
    // rem = 2 rem + bit
    uint32_t c = (a[i / 32] >> (i % 32)) & 1u;
    for (auto& w : rem) {
      const uint32_t nc = w >> 31;
      w = (w << 1) | c;
      c = nc;
    }
    if (c) rem.push_back(c);
    if (cmp(rem, d) >= 0) {
      sub_in(rem, d);
      q[i / 32] |= 1u << (i % 32);
    }
  }
  trim(q);
  trim(rem);
  return q;
}
}  // namespace bigu

// (q^4 - q^2 + 1) / r, computed once (the hard part; (q^6 + 1) = (q^2 + 1)(q^4 - q^2 + 1))
inline const std::vector<uint32_t>& final_exp_hard() {
  static const std::vector<uint32_t> e = [] {
    bigu::Big q(Bls12_381Fq::P, Bls12_381Fq::P + 12);
    const bigu::Big q2 = bigu::mul(q, q);
    bigu::Big q4 = bigu::mul(q2, q2);
    bigu::add_small(q4, 1);
    bigu::sub_in(q4, q2);  // q^4 - q^2 + 1
    bigu::Big r(8);
    for (int i = 0; i < 8; ++i) r[i] = Bls12_381Fr::P[i];
    bigu::trim(r);
    bigu::Big rem;
    bigu::Big out = bigu::divmod(q4, r, rem);
    if (!rem.empty()) out.clear();  // r must divide q^4 - q^2 + 1; an empty exponent makes every check fail
    return out;
  }();
  return e;
}

// Frobenius a -> a^q. In the w-power basis of Fq12 (w^2 = v, w^6 = xi), a =
// sum_k c_k w^k with c_0..c_5 = a00, a10, a01, a11, a02, a12, and
// (c w^k)^q = conj(c) w^k xi^(k (q - 1) / 6): conjugate each Fq2 coefficient
// and scale it by gamma_k = xi^(k (q - 1) / 6) (q = 1 mod 6), computed once.
inline Fq2 fq2_pow(const Fq2& a, const std::vector<uint32_t>& e) {
  Fq2 r = fq2_one();
  for (size_t i = e.size(); i-- > 0;)
    for (int b = 31; b >= 0; --b) {
      r = fq2_sqr(r);
      if ((e[i] >> b) & 1u) r = fq2_mul(r, a);
    }
  return r;
}
inline const std::array<Fq2, 6>& frob_gamma() {
  static const std::array<Fq2, 6> g = [] {
    bigu::Big q(Bls12_381Fq::P, Bls12_381Fq::P + 12);
    bigu::Big one{1};
    bigu::sub_in(q, one);  // q - 1
    bigu::Big six{6}, rem;
    const bigu::Big e = bigu::divmod(q, six, rem);  // (q - 1) / 6, exact
    const Fq2 xi = {fq_one(), fq_one()};             // 1 + u
    const Fq2 g1 = fq2_pow(xi, e);
    std::array<Fq2, 6> out;
    out[0] = fq2_one();
    for (int k = 1; k < 6; ++k) out[k] = fq2_mul(out[k - 1], g1);
    return out;
  }();
  return g;
}
inline Fq12 fq12_frobenius(const Fq12& a) {
  const std::array<Fq2, 6>& g = frob_gamma();
  Fq12 r;
  r.c0.c0 = fq2_mul(fq2_conj(a.c0.c0), g[0]);
  r.c1.c0 = fq2_mul(fq2_conj(a.c1.c0), g[1]);
  r.c0.c1 = fq2_mul(fq2_conj(a.c0.c1), g[2]);
  r.c1.c1 = fq2_mul(fq2_conj(a.c1.c1), g[3]);
  r.c0.c2 = fq2_mul(fq2_conj(a.c0.c2), g[4]);
  r.c1.c2 = fq2_mul(fq2_conj(a.c1.c2), g[5]);
  return r;
}
// a^e with fixed 4-bit windows (e LE u32 limbs)
inline Fq12 fq12_pow_w4(const Fq12& a, const std::vector<uint32_t>& e) {
  Fq12 tab[16];
  tab[0] = fq12_one();
  tab[1] = a;
  for (int i = 2; i < 16; ++i) tab[i] = fq12_mul(tab[i - 1], a);
  Fq12 r = fq12_one();
  bool started = false;
  for (size_t i = e.size(); i-- > 0;)
    for (int sh = 28; sh >= 0; sh -= 4) {
      const uint32_t d = (e[i] >> sh) & 15u;
      if (started)
        for (int k = 0; k < 4; ++k) r = fq12_sqr(r);
      if (d) {
        r = started ? fq12_mul(r, tab[d]) : tab[d];
        started = true;
      }
    }
  return r;
}

// f^((q^12 - 1) / r) = f^((q^6 - 1)(q^2 + 1) (q^4 - q^2 + 1) / r): the easy part
// by a conjugation, an inversion and two Frobenius maps, the hard part by a
// windowed power (round 6; the same value as the generic (q^6 + 1) / r power
// it replaces, pinned by the oracle's pairing values in the CPU tests)
inline Fq12 final_exponentiation(const Fq12& f) {
  const Fq12 e1 = fq12_mul(fq12_conj(f), fq12_inv(f));          // f^(q^6 - 1)
  const Fq12 e2 = fq12_mul(fq12_frobenius(fq12_frobenius(e1)), e1);  // ^(q^2 + 1)
  return fq12_pow_w4(e2, final_exp_hard());
}

// ---- G2 (the twist, over Fq2) -------------------------------------------------
struct G2A {
  Fq2 x, y;
  bool inf;
};
struct G2J {
  Fq2 X, Y, Z;
};
inline G2J g2_inf() { return {fq2_zero(), fq2_one(), fq2_zero()}; }
inline bool g2_is_inf(const G2J& p) { return fq2_is_zero(p.Z); }
inline G2J g2_from_affine(const G2A& a) { return a.inf ? g2_inf() : G2J{a.x, a.y, fq2_one()}; }
inline Fq2 g2_b() {  // 4 xi = 4 + 4u
  Fq four = fq_zero();
  four.v[0] = 4;
  const Fq f = fq_to_mont(four);
  return {f, f};
}
inline bool g2_on_curve(const G2A& a) {
  if (a.inf) return true;
  return fq2_eq(fq2_sqr(a.y), fq2_add(fq2_mul(fq2_sqr(a.x), a.x), g2_b()));
}
inline G2J g2_dbl(const G2J& p) {  // dbl-2009-l (a = 0)
  if (g2_is_inf(p)) return p;
  const Fq2 A = fq2_sqr(p.X), B = fq2_sqr(p.Y), C = fq2_sqr(B);
  const Fq2 D = fq2_dbl(fq2_sub(fq2_sub(fq2_sqr(fq2_add(p.X, B)), A), C));
  const Fq2 E = fq2_add(fq2_dbl(A), A), F = fq2_sqr(E);
  G2J r;
  r.X = fq2_sub(F, fq2_dbl(D));
  r.Y = fq2_sub(fq2_mul(E, fq2_sub(D, r.X)), fq2_dbl(fq2_dbl(fq2_dbl(C))));
  r.Z = fq2_dbl(fq2_mul(p.Y, p.Z));
  return r;
}
inline G2J g2_add(const G2J& p, const G2J& q) {  // add-2007-bl with the exceptional cases
  if (g2_is_inf(p)) return q;
  if (g2_is_inf(q)) return p;
  const Fq2 Z1Z1 = fq2_sqr(p.Z), Z2Z2 = fq2_sqr(q.Z);
  const Fq2 U1 = fq2_mul(p.X, Z2Z2), U2 = fq2_mul(q.X, Z1Z1);
  const Fq2 S1 = fq2_mul(p.Y, fq2_mul(q.Z, Z2Z2)), S2 = fq2_mul(q.Y, fq2_mul(p.Z, Z1Z1));
  const Fq2 H = fq2_sub(U2, U1), rr = fq2_dbl(fq2_sub(S2, S1));
  if (fq2_is_zero(H)) return fq2_is_zero(rr) ? g2_dbl(p) : g2_inf();
  const Fq2 I = fq2_sqr(fq2_dbl(H)), J = fq2_mul(H, I), V = fq2_mul(U1, I);
  G2J r;
  r.X = fq2_sub(fq2_sub(fq2_sqr(rr), J), fq2_dbl(V));
  r.Y = fq2_sub(fq2_mul(rr, fq2_sub(V, r.X)), fq2_dbl(fq2_mul(S1, J)));
  r.Z = fq2_mul(fq2_sub(fq2_sub(fq2_sqr(fq2_add(p.Z, q.Z)), Z1Z1), Z2Z2), H);
  return r;
}
inline G2J g2_neg(const G2J& p) { return {p.X, fq2_neg(p.Y), p.Z}; }
inline G2A g2_to_affine(const G2J& p) {
  if (g2_is_inf(p)) return {fq2_zero(), fq2_zero(), true};
  const Fq2 zi = fq2_inv(p.Z), zi2 = fq2_sqr(zi);
  return {fq2_mul(p.X, zi2), fq2_mul(p.Y, fq2_mul(zi2, zi)), false};
}
// k * p, k a canonical little-endian 256-bit integer (G2Projective::mul_bigint)
inline G2J g2_mul(const G2J& p, const uint32_t k[8]) {
  G2J r = g2_inf();
  for (int i = 7; i >= 0; --i)
    for (int b = 31; b >= 0; --b) {
      r = g2_dbl(r);
      if ((k[i] >> b) & 1u) r = g2_add(r, p);
    }
  return r;
}
inline G1J g1_neg(const G1J& p) { return {p.X, fq_neg(p.Y), p.Z}; }
inline G1J g1_mul(const G1J& p, const uint32_t k[8]) {  // G1Projective::mul_bigint
  G1J r = g1_inf();
  for (int i = 7; i >= 0; --i)
    for (int b = 31; b >= 0; --b) {
      r = g1_dbl(r);
      if ((k[i] >> b) & 1u) r = g1_add(r, p);
    }
  return r;
}

// The BLS12-381 G2 generator (ark-bls12-381 0.5.0), canonical limbs, x = x0 + x1 u
constexpr uint32_t kG2GenX0[12] = {0xc121bdb8u, 0xd48056c8u, 0xa805bbefu, 0x0bac0326u, 0x7ae3d177u, 0xb4510b64u,
                                   0xfa403b02u, 0xc6e47ad4u, 0x2dc51051u, 0x26080527u, 0xf08f0a91u, 0x024aa2b2u};
constexpr uint32_t kG2GenX1[12] = {0x5d042b7eu, 0xe5ac7d05u, 0x13945d57u, 0x334cf112u, 0xdc7f5049u, 0xb5da61bbu,
                                   0x9920b61au, 0x596bd0d0u, 0x88274f65u, 0x7dacd3a0u, 0x52719f60u, 0x13e02b60u};
constexpr uint32_t kG2GenY0[12] = {0x08b82801u, 0xe1935486u, 0x3baca289u, 0x923ac9ccu, 0x5160d12cu, 0x6d429a69u,
                                   0x8cbdd3a7u, 0xadfd9baau, 0xda2e351au, 0x8cc9cdc6u, 0x727d6e11u, 0x0ce5d527u};
constexpr uint32_t kG2GenY1[12] = {0xf05f79beu, 0xaaa9075fu, 0x5cec1da1u, 0x3f370d27u, 0x572e99abu, 0x267492abu,
                                   0x85a763afu, 0xcb3e287eu, 0x2bc28b99u, 0x32acd2b0u, 0x2ea734ccu, 0x0606c4a0u};

inline Fq fq_from_canon_limbs(const uint32_t* c) {
  Fq x;
  for (int i = 0; i < 12; ++i) x.v[i] = c[i];
  return fq_to_mont(x);
}
inline G2A g2_generator() {
  return {{fq_from_canon_limbs(kG2GenX0), fq_from_canon_limbs(kG2GenX1)},
          {fq_from_canon_limbs(kG2GenY0), fq_from_canon_limbs(kG2GenY1)},
          false};
}

// ---- Miller loop -------------------------------------------------------------
constexpr uint64_t kBlsX = 0xd201000000010000ull;  // |x|; x is negative

// xi * (line through T with slope lambda, evaluated at P), see the header
inline Fq12 line_eval(const Fq2& lambda, const Fq2& xT, const Fq2& yT, const Fq& xP, const Fq& yP) {
  Fq12 l;
  l.c0 = {{yP, yP}, fq2_zero(), fq2_zero()};  // xi * y_P = y_P + y_P u
  l.c1 = {fq2_zero(), fq2_sub(fq2_mul(lambda, xT), yT), fq2_neg(fq2_mul_fq(lambda, xP))};
  return l;
}

// f_{x, Q}(P) (conjugated for the negative x); P, Q affine Montgomery, not infinity
inline Fq12 miller_loop(const G1A& P, const G2A& Q) {
  Fq12 f = fq12_one();
  Fq2 xT = Q.x, yT = Q.y;
  for (int i = 62; i >= 0; --i) {
    f = fq12_sqr(f);
    // tangent at T
    const Fq2 x2 = fq2_sqr(xT);
    Fq2 lam = fq2_mul(fq2_add(fq2_dbl(x2), x2), fq2_inv(fq2_dbl(yT)));
    f = fq12_mul(f, line_eval(lam, xT, yT, P.x, P.y));
    Fq2 x3 = fq2_sub(fq2_sqr(lam), fq2_dbl(xT));
    yT = fq2_sub(fq2_mul(lam, fq2_sub(xT, x3)), yT);
    xT = x3;
    if ((kBlsX >> i) & 1u) {
      // chord through T and Q (T = kQ with 2 <= k < |x| < r, so T != +-Q)
      lam = fq2_mul(fq2_sub(Q.y, yT), fq2_inv(fq2_sub(Q.x, xT)));
      f = fq12_mul(f, line_eval(lam, xT, yT, P.x, P.y));
      x3 = fq2_sub(fq2_sub(fq2_sqr(lam), xT), Q.x);
      yT = fq2_sub(fq2_mul(lam, fq2_sub(xT, x3)), yT);
      xT = x3;
    }
  }
  return fq12_conj(f);
}

// prod_i e(P_i, Q_i): the product of Miller loops, one final exponentiation.
// Pairs with a point at infinity contribute 1.
inline Fq12 multi_pairing(const std::vector<G1A>& P, const std::vector<G2A>& Q) {
  Fq12 f = fq12_one();
  for (size_t i = 0; i < P.size(); ++i) {
    if (g1a_is_inf(P[i]) || Q[i].inf) continue;
    f = fq12_mul(f, miller_loop(P[i], Q[i]));
  }
  return final_exponentiation(f);
}

}  // namespace zk
