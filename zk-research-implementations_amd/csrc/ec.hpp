// BLS12-381 G1 for the multilinear KZG commitment (SURVEY.md 8(f3);
// pcs/src/kzg_pcs/kzg.rs). Host and device code (ZK_HD).
//
// Base field Fq: 381-bit prime, 12 x 32-bit little-endian limbs, Montgomery
// form with R = 2^384 (ark-ff 0.5.0's Fp384 uses 6 x u64, same R). CIOS
// multiplication as in field.hpp, 12 rows: 288 v_mad_u64_u32. Every operation
// returns a fully reduced value (p < 2^381, so sums never overflow 384 bits).
//
// Curve y^2 = x^3 + 4 (a = 0). Points in Jacobian coordinates (X:Y:Z),
// x = X/Z^2, y = Y/Z^3, Z = 0 the point at infinity; bases in affine form,
// (0, 0) marking infinity (not on the curve). Formulas from the Explicit-
// Formulas Database for a = 0: dbl-2009-l, madd-2007-bl, add-2007-bl, with
// the exceptional cases (P = Q, P = -Q, infinity) handled explicitly, so the
// group element — and hence the canonical affine output — is exact.
#pragma once
#include <string.h>

#include "field.hpp"

namespace zk {

struct Bls12_381Fq {
  static constexpr uint32_t P[12] = {0xffffaaabu, 0xb9feffffu, 0xb153ffffu, 0x1eabfffeu, 0xf6b0f624u, 0x6730d2a0u,
                                     0xf38512bfu, 0x64774b84u, 0x434bacd7u, 0x4b1ba7b6u, 0x397fe69au, 0x1a0111eau};
  static constexpr uint32_t PINV = 0xfffcfffdu;  // -p^-1 mod 2^32
  static constexpr uint32_t R1[12] = {0x0002fffdu, 0x76090000u, 0xc40c0002u, 0xebf4000bu, 0x53c758bau, 0x5f489857u,
                                      0x70525745u, 0x77ce5853u, 0xa256ec6du, 0x5c071a97u, 0xfa80e493u, 0x15f65ec3u};
  static constexpr uint32_t R2[12] = {0x1c341746u, 0xf4df1f34u, 0x09d104f1u, 0x0a76e6a6u, 0x4c95b6d5u, 0x8de5476cu,
                                      0x939d83c0u, 0x67eb88a9u, 0xb519952du, 0x9a793e85u, 0x92cae3aau, 0x11988fe5u};
};

struct Fq {
  uint32_t v[12];
};

ZK_HD Fq fq_zero() {
  Fq r;
#pragma unroll
  for (int i = 0; i < 12; ++i) r.v[i] = 0;
  return r;
}
ZK_HD Fq fq_one() {
  Fq r;
#pragma unroll
  for (int i = 0; i < 12; ++i) r.v[i] = Bls12_381Fq::R1[i];
  return r;
}
ZK_HD bool fq_is_zero(const Fq& a) {
  uint32_t acc = 0;
#pragma unroll
  for (int i = 0; i < 12; ++i) acc |= a.v[i];
  return acc == 0;
}
ZK_HD bool fq_eq(const Fq& a, const Fq& b) {
  uint32_t acc = 0;
#pragma unroll
  for (int i = 0; i < 12; ++i) acc |= a.v[i] ^ b.v[i];
  return acc == 0;
}
ZK_HD Fq fq_reduce_once(const Fq& x) {
  Fq t;
  uint32_t b = 0;
#pragma unroll
  for (int i = 0; i < 12; ++i) t.v[i] = subb32(x.v[i], Bls12_381Fq::P[i], b, &b);
  Fq r;
#pragma unroll
  for (int i = 0; i < 12; ++i) r.v[i] = b ? x.v[i] : t.v[i];
  return r;
}
ZK_HD bool fq_is_canonical(const Fq& x) {
  uint32_t b = 0;
#pragma unroll
  for (int i = 0; i < 12; ++i) (void)subb32(x.v[i], Bls12_381Fq::P[i], b, &b);
  return b != 0;
}
ZK_HD Fq fq_add(const Fq& a, const Fq& b) {
  Fq s;
  uint32_t c = 0;
#pragma unroll
  for (int i = 0; i < 12; ++i) s.v[i] = addc32(a.v[i], b.v[i], c, &c);
  return fq_reduce_once(s);
}
ZK_HD Fq fq_sub(const Fq& a, const Fq& b) {
  Fq d;
  uint32_t bw = 0;
#pragma unroll
  for (int i = 0; i < 12; ++i) d.v[i] = subb32(a.v[i], b.v[i], bw, &bw);
  const uint32_t mask = 0u - bw;
  uint32_t c = 0;
  Fq r;
#pragma unroll
  for (int i = 0; i < 12; ++i) r.v[i] = addc32(d.v[i], Bls12_381Fq::P[i] & mask, c, &c);
  return r;
}
ZK_HD Fq fq_dbl(const Fq& a) { return fq_add(a, a); }
ZK_HD Fq fq_neg(const Fq& a) { return fq_sub(fq_zero(), a); }

#if !defined(__HIP_DEVICE_COMPILE__)
// Host: the same product on 6 x 64-bit limbs (unsigned __int128 rows, CIOS),
// ~4x fewer instructions than the 32-bit rows below — the host's G1/G2 work
// (the MSMs' window Horners, the setup's G2 taus, point normalisation, the
// pairings) is chains of these. Same value: the fully reduced a b 2^-384 mod p.
namespace fqh {
using u128 = unsigned __int128;
constexpr uint64_t P(int i) { return (uint64_t)Bls12_381Fq::P[2 * i] | ((uint64_t)Bls12_381Fq::P[2 * i + 1] << 32); }
constexpr uint64_t pinv() {  // -p^-1 mod 2^64 (Newton)
  uint64_t x = 1;
  for (int i = 0; i < 7; ++i) x *= 2 - P(0) * x;
  return (uint64_t)0 - x;
}
inline Fq mul(const Fq& a, const Fq& b) {
  uint64_t A[6], B[6], t[7] = {0, 0, 0, 0, 0, 0, 0};
  memcpy(A, a.v, 48);
  memcpy(B, b.v, 48);
  for (int i = 0; i < 6; ++i) {
    uint64_t c = 0;
    for (int j = 0; j < 6; ++j) {
      const u128 x = (u128)A[j] * B[i] + t[j] + c;
      t[j] = (uint64_t)x;
      c = (uint64_t)(x >> 64);
    }
    const uint64_t t6 = t[6] + c;  // (t < 2p < 2^382 between rows: no overflow)
    const uint64_t m = t[0] * pinv();
    u128 x = (u128)m * P(0) + t[0];
    c = (uint64_t)(x >> 64);
    for (int j = 1; j < 6; ++j) {
      x = (u128)m * P(j) + t[j] + c;
      t[j - 1] = (uint64_t)x;
      c = (uint64_t)(x >> 64);
    }
    x = (u128)t6 + c;
    t[5] = (uint64_t)x;
    t[6] = (uint64_t)(x >> 64);
  }
  Fq r;
  memcpy(r.v, t, 48);
  return fq_reduce_once(r);  // (t < 2p)
}
}  // namespace fqh
#endif

// CIOS Montgomery product a*b*2^-384 mod p (invariant t < 2p < 2^384 between rows)
ZK_HD Fq fq_mul(const Fq& a, const Fq& b) {
#if !defined(__HIP_DEVICE_COMPILE__)
  return fqh::mul(a, b);
#endif
  uint32_t t[12];
#pragma unroll
  for (int j = 0; j < 12; ++j) t[j] = 0;
#pragma unroll
  for (int i = 0; i < 12; ++i) {
    const uint32_t bi = b.v[i];
    uint64_t Pr[12];
#pragma unroll
    for (int j = 0; j < 12; ++j) Pr[j] = mad64(a.v[j], bi, t[j]);
    uint32_t u[13];
    uint32_t c = 0;
    u[0] = (uint32_t)Pr[0];
#pragma unroll
    for (int j = 1; j < 12; ++j) u[j] = addc32((uint32_t)Pr[j], (uint32_t)(Pr[j - 1] >> 32), c, &c);
    u[12] = (uint32_t)(Pr[11] >> 32) + c;
    const uint32_t m = u[0] * Bls12_381Fq::PINV;
    uint64_t Qr[12];
#pragma unroll
    for (int j = 0; j < 12; ++j) Qr[j] = mad64(m, Bls12_381Fq::P[j], u[j]);
    c = 0;
#pragma unroll
    for (int j = 1; j < 12; ++j) t[j - 1] = addc32((uint32_t)Qr[j], (uint32_t)(Qr[j - 1] >> 32), c, &c);
    t[11] = u[12] + (uint32_t)(Qr[11] >> 32) + c;
  }
  Fq r;
#pragma unroll
  for (int j = 0; j < 12; ++j) r.v[j] = t[j];
  return fq_reduce_once(r);
}
ZK_HD Fq fq_sqr(const Fq& a) { return fq_mul(a, a); }
ZK_HD Fq fq_to_mont(const Fq& canon) {
  Fq r2;
#pragma unroll
  for (int i = 0; i < 12; ++i) r2.v[i] = Bls12_381Fq::R2[i];
  return fq_mul(canon, r2);
}
ZK_HD Fq fq_from_mont(const Fq& m) {
  Fq one = fq_zero();
  one.v[0] = 1;
  return fq_mul(m, one);
}
// a^(p-2) (Fermat), a != 0; left-to-right over the bits of p - 2
ZK_HD Fq fq_inv(const Fq& a) {
  uint32_t e[12];
  uint32_t b = 0;
  e[0] = subb32(Bls12_381Fq::P[0], 2u, 0u, &b);
  for (int i = 1; i < 12; ++i) e[i] = subb32(Bls12_381Fq::P[i], 0u, b, &b);
  Fq r = fq_one();
  for (int i = 11; i >= 0; --i)
    for (int k = 31; k >= 0; --k) {
      r = fq_sqr(r);
      if ((e[i] >> k) & 1u) r = fq_mul(r, a);
    }
  return r;
}

// ---- G1 ----------------------------------------------------------------------
struct G1J {
  Fq X, Y, Z;
};
struct G1A {
  Fq x, y;  // (0, 0): infinity
};

ZK_HD G1J g1_inf() { return {fq_zero(), fq_one(), fq_zero()}; }
ZK_HD bool g1_is_inf(const G1J& p) { return fq_is_zero(p.Z); }
ZK_HD bool g1a_is_inf(const G1A& p) { return fq_is_zero(p.x) && fq_is_zero(p.y); }
ZK_HD G1J g1_from_affine(const G1A& a) { return g1a_is_inf(a) ? g1_inf() : G1J{a.x, a.y, fq_one()}; }

ZK_HD G1J g1_dbl(const G1J& p) {  // dbl-2009-l
  if (g1_is_inf(p)) return p;
  const Fq A = fq_sqr(p.X), Bq = fq_sqr(p.Y), C = fq_sqr(Bq);
  const Fq D = fq_dbl(fq_sub(fq_sub(fq_sqr(fq_add(p.X, Bq)), A), C));
  const Fq E = fq_add(fq_dbl(A), A), F = fq_sqr(E);
  G1J r;
  r.X = fq_sub(F, fq_dbl(D));
  const Fq C8 = fq_dbl(fq_dbl(fq_dbl(C)));
  r.Y = fq_sub(fq_mul(E, fq_sub(D, r.X)), C8);
  r.Z = fq_dbl(fq_mul(p.Y, p.Z));
  return r;
}

ZK_HD G1J g1_add_mixed(const G1J& p, const G1A& q) {  // madd-2007-bl
  if (g1a_is_inf(q)) return p;
  if (g1_is_inf(p)) return G1J{q.x, q.y, fq_one()};
  const Fq Z1Z1 = fq_sqr(p.Z);
  const Fq U2 = fq_mul(q.x, Z1Z1), S2 = fq_mul(q.y, fq_mul(p.Z, Z1Z1));
  const Fq H = fq_sub(U2, p.X), rr = fq_dbl(fq_sub(S2, p.Y));
  if (fq_is_zero(H)) return fq_is_zero(rr) ? g1_dbl(p) : g1_inf();
  const Fq HH = fq_sqr(H), I = fq_dbl(fq_dbl(HH)), J = fq_mul(H, I), V = fq_mul(p.X, I);
  G1J r;
  r.X = fq_sub(fq_sub(fq_sqr(rr), J), fq_dbl(V));
  r.Y = fq_sub(fq_mul(rr, fq_sub(V, r.X)), fq_dbl(fq_mul(p.Y, J)));
  r.Z = fq_sub(fq_sub(fq_sqr(fq_add(p.Z, H)), Z1Z1), HH);
  return r;
}

ZK_HD G1J g1_add(const G1J& p, const G1J& q) {  // add-2007-bl
  if (g1_is_inf(p)) return q;
  if (g1_is_inf(q)) return p;
  const Fq Z1Z1 = fq_sqr(p.Z), Z2Z2 = fq_sqr(q.Z);
  const Fq U1 = fq_mul(p.X, Z2Z2), U2 = fq_mul(q.X, Z1Z1);
  const Fq S1 = fq_mul(p.Y, fq_mul(q.Z, Z2Z2)), S2 = fq_mul(q.Y, fq_mul(p.Z, Z1Z1));
  const Fq H = fq_sub(U2, U1), rr = fq_dbl(fq_sub(S2, S1));
  if (fq_is_zero(H)) return fq_is_zero(rr) ? g1_dbl(p) : g1_inf();
  const Fq I = fq_sqr(fq_dbl(H)), J = fq_mul(H, I), V = fq_mul(U1, I);
  G1J r;
  r.X = fq_sub(fq_sub(fq_sqr(rr), J), fq_dbl(V));
  r.Y = fq_sub(fq_mul(rr, fq_sub(V, r.X)), fq_dbl(fq_mul(S1, J)));
  r.Z = fq_mul(fq_sub(fq_sub(fq_sqr(fq_add(p.Z, q.Z)), Z1Z1), Z2Z2), H);
  return r;
}

// XYZZ accumulators (round 4): (X, Y, ZZ, ZZZ) is the affine point (X/ZZ,
// Y/ZZZ) with ZZ^3 = ZZZ^2; ZZ = 0 is infinity. Adding an affine point costs
// 8 multiplications + 2 squarings (madd-2008-s) against 7 + 4 for Jacobian
// madd-2007-bl, and a run of additions converts to Jacobian once (3 + 4).
struct G1XYZZ {
  Fq X, Y, ZZ, ZZZ;
};
ZK_HD G1XYZZ g1x_inf() { return {fq_zero(), fq_zero(), fq_zero(), fq_zero()}; }
ZK_HD G1XYZZ g1x_dbl(const G1XYZZ& p) {  // dbl-2008-s-1 (a = 0)
  if (fq_is_zero(p.ZZ)) return p;
  const Fq U = fq_dbl(p.Y), V = fq_sqr(U), W = fq_mul(U, V), S = fq_mul(p.X, V);
  const Fq X2 = fq_sqr(p.X), M = fq_add(fq_dbl(X2), X2);
  G1XYZZ r;
  r.X = fq_sub(fq_sqr(M), fq_dbl(S));
  r.Y = fq_sub(fq_mul(M, fq_sub(S, r.X)), fq_mul(W, p.Y));
  r.ZZ = fq_mul(V, p.ZZ);
  r.ZZZ = fq_mul(W, p.ZZZ);
  return r;
}
ZK_HD G1XYZZ g1x_add_mixed(const G1XYZZ& p, const G1A& q) {  // madd-2008-s
  if (g1a_is_inf(q)) return p;
  if (fq_is_zero(p.ZZ)) return {q.x, q.y, fq_one(), fq_one()};
  const Fq P = fq_sub(fq_mul(q.x, p.ZZ), p.X), R = fq_sub(fq_mul(q.y, p.ZZZ), p.Y);
  if (fq_is_zero(P)) return fq_is_zero(R) ? g1x_dbl(p) : g1x_inf();
  const Fq PP = fq_sqr(P), PPP = fq_mul(P, PP), Q = fq_mul(p.X, PP);
  G1XYZZ r;
  r.X = fq_sub(fq_sub(fq_sqr(R), PPP), fq_dbl(Q));
  r.Y = fq_sub(fq_mul(R, fq_sub(Q, r.X)), fq_mul(p.Y, PPP));
  r.ZZ = fq_mul(p.ZZ, PP);
  r.ZZZ = fq_mul(p.ZZZ, PPP);
  return r;
}
ZK_HD G1XYZZ g1x_add(const G1XYZZ& p, const G1XYZZ& q) {  // add-2008-s
  if (fq_is_zero(q.ZZ)) return p;
  if (fq_is_zero(p.ZZ)) return q;
  const Fq U1 = fq_mul(p.X, q.ZZ), U2 = fq_mul(q.X, p.ZZ);
  const Fq S1 = fq_mul(p.Y, q.ZZZ), S2 = fq_mul(q.Y, p.ZZZ);
  const Fq P = fq_sub(U2, U1), R = fq_sub(S2, S1);
  if (fq_is_zero(P)) return fq_is_zero(R) ? g1x_dbl(p) : g1x_inf();
  const Fq PP = fq_sqr(P), PPP = fq_mul(P, PP), Q = fq_mul(U1, PP);
  G1XYZZ r;
  r.X = fq_sub(fq_sub(fq_sqr(R), PPP), fq_dbl(Q));
  r.Y = fq_sub(fq_mul(R, fq_sub(Q, r.X)), fq_mul(S1, PPP));
  r.ZZ = fq_mul(fq_mul(p.ZZ, q.ZZ), PP);
  r.ZZZ = fq_mul(fq_mul(p.ZZZ, q.ZZZ), PPP);
  return r;
}
// Jacobian with Z' = ZZ ZZZ (= Z^5 for Z^2 = ZZ): X' = X ZZ^4, Y' = Y ZZZ^4
ZK_HD G1J g1x_to_jac(const G1XYZZ& p) {
  if (fq_is_zero(p.ZZ)) return g1_inf();
  const Fq a = fq_sqr(p.ZZ), b = fq_sqr(p.ZZZ);
  return {fq_mul(p.X, fq_sqr(a)), fq_mul(p.Y, fq_sqr(b)), fq_mul(p.ZZ, p.ZZZ)};
}

ZK_HD G1A g1_to_affine(const G1J& p) {
  if (g1_is_inf(p)) return {fq_zero(), fq_zero()};
  const Fq zi = fq_inv(p.Z), zi2 = fq_sqr(zi);
  return {fq_mul(p.X, zi2), fq_mul(p.Y, fq_mul(zi2, zi))};
}
// affine with a known Z^-1 (batch normalisation)
ZK_HD G1A g1_to_affine_zi(const G1J& p, const Fq& zi) {
  if (g1_is_inf(p)) return {fq_zero(), fq_zero()};
  const Fq zi2 = fq_sqr(zi);
  return {fq_mul(p.X, zi2), fq_mul(p.Y, fq_mul(zi2, zi))};
}

// k * p for a small scalar k (double-and-add, MSB first)
ZK_HD G1J g1_mul_small(const G1J& p, uint32_t k) {
  G1J r = g1_inf();
  for (int b = 31; b >= 0; --b) {
    r = g1_dbl(r);
    if ((k >> b) & 1u) r = g1_add(r, p);
  }
  return r;
}

// The BLS12-381 G1 generator (ark-bls12-381 0.5.0), canonical limbs
constexpr uint32_t kG1GenX[12] = {0xdb22c6bbu, 0xfb3af00au, 0xf97a1aefu, 0x6c55e83fu, 0x171bac58u, 0xa14e3a3fu,
                                  0x9774b905u, 0xc3688c4fu, 0x4fa9ac0fu, 0x2695638cu, 0x3197d794u, 0x17f1d3a7u};
constexpr uint32_t kG1GenY[12] = {0x46c5e7e1u, 0x0caa2329u, 0xa2888ae4u, 0xd03cc744u, 0x2c04b3edu, 0x00db18cbu,
                                  0xd5d00af6u, 0xfcf5e095u, 0x741d8ae4u, 0xa09e30edu, 0xe3aaa0f1u, 0x08b3f481u};

}  // namespace zk
