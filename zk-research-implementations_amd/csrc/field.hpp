// Prime-field arithmetic shared by the host C++ and the gfx950 kernels.
//
// Element = 8 x 32-bit little-endian limbs in Montgomery form with R = 2^256,
// i.e. the same 32-byte image as ark-ff 0.5.0's `Fp<MontBackend<_, 4>, 4>`
// (4 x u64 LE limbs, Montgomery, R = 2^256), so a Rust caller's `Vec<F>`
// memory is usable as-is (Cargo.lock:89-92 pins ark-ff 0.5.0; the field
// operations it replaces are every `+ - *` in
// multilinear_polynomial_evaluation.rs:52-110, composed_polynomial.rs:52-99,
// sum_check_protocol.rs:25-166 and univariate_polynomial_dense.rs:20-74).
//
// Multiplication is word-serial Montgomery (CIOS) built on gfx950's
// v_mad_u64_u32 (32x32+64 -> 64) and v_add_co/v_addc_co carry chains; every
// operation returns a fully reduced value in [0, p), so canonical results
// are bit-identical to ark-ff regardless of the internal schedule.
#pragma once
#include <stdint.h>

#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#define ZK_HD __host__ __device__ __forceinline__
#else
#define ZK_HD static inline
#endif

namespace zk {

enum FieldId : int { BN254_FR = 0, BN254_FQ = 1, BLS12_381_FR = 2 };

// Public curve constants (ark-bn254 0.5.0 / ark-bls12-381 0.5.0, Cargo.lock:45-60).
struct Bn254Fr {
  static constexpr int id = BN254_FR;
  static constexpr uint32_t P[8] = {0xf0000001u, 0x43e1f593u, 0x79b97091u, 0x2833e848u,
                                    0x8181585du, 0xb85045b6u, 0xe131a029u, 0x30644e72u};
  static constexpr uint32_t PINV = 0xefffffffu;  // -p^-1 mod 2^32
  static constexpr uint32_t R1[8] = {0x4ffffffbu, 0xac96341cu, 0x9f60cd29u, 0x36fc7695u,
                                     0x7879462eu, 0x666ea36fu, 0x9a07df2fu, 0x0e0a77c1u};
  static constexpr uint32_t R2[8] = {0xae216da7u, 0x1bb8e645u, 0xe35c59e3u, 0x53fe3ab1u,
                                     0x53bb8085u, 0x8c49833du, 0x7f4e44a5u, 0x0216d0b1u};
  static constexpr uint32_t INV2[8] = {0x1ffffffeu, 0x783c14d8u, 0x0c8d1eddu, 0xaf982f6fu,
                                       0xfcfd4f45u, 0x8f5f7492u, 0x3d9cbfacu, 0x1f37631au};
};
struct Bn254Fq {
  static constexpr int id = BN254_FQ;
  static constexpr uint32_t P[8] = {0xd87cfd47u, 0x3c208c16u, 0x6871ca8du, 0x97816a91u,
                                    0x8181585du, 0xb85045b6u, 0xe131a029u, 0x30644e72u};
  static constexpr uint32_t PINV = 0xe4866389u;
  static constexpr uint32_t R1[8] = {0xc58f0d9du, 0xd35d438du, 0xf5c70b3du, 0x0a78eb28u,
                                     0x7879462cu, 0x666ea36fu, 0x9a07df2fu, 0x0e0a77c1u};
  static constexpr uint32_t R2[8] = {0x538afa89u, 0xf32cfc5bu, 0xd44501fbu, 0xb5e71911u,
                                     0x0a417ff6u, 0x47ab1effu, 0xcab8351fu, 0x06d89f71u};
  static constexpr uint32_t INV2[8] = {0x4f060572u, 0x87bee7d2u, 0x2f1c6ae5u, 0xd0fd2addu,
                                       0xfcfd4f44u, 0x8f5f7492u, 0x3d9cbfacu, 0x1f37631au};
};
struct Bls12_381Fr {
  static constexpr int id = BLS12_381_FR;
  static constexpr uint32_t P[8] = {0x00000001u, 0xffffffffu, 0xfffe5bfeu, 0x53bda402u,
                                    0x09a1d805u, 0x3339d808u, 0x299d7d48u, 0x73eda753u};
  static constexpr uint32_t PINV = 0xffffffffu;
  static constexpr uint32_t R1[8] = {0xfffffffeu, 0x00000001u, 0x00034802u, 0x5884b7fau,
                                     0xecbc4ff5u, 0x998c4fefu, 0xacc5056fu, 0x1824b159u};
  static constexpr uint32_t R2[8] = {0xf3f29c6du, 0xc999e990u, 0x87925c23u, 0x2b6cedcbu,
                                     0x7254398fu, 0x05d31496u, 0x9f59ff11u, 0x0748d9d9u};
  static constexpr uint32_t INV2[8] = {0xffffffffu, 0x00000000u, 0x0001a401u, 0xac425bfdu,
                                       0xf65e27fau, 0xccc627f7u, 0xd66282b7u, 0x0c1258acu};
};

struct Fe {
  uint32_t v[8];
};

// ---- carry primitives ------------------------------------------------------
ZK_HD uint32_t addc32(uint32_t a, uint32_t b, uint32_t cin, uint32_t* cout) {
#if defined(__clang__)
  unsigned int c;
  uint32_t r = __builtin_addc(a, b, cin, &c);
  *cout = c;
  return r;
#else
  uint64_t s = (uint64_t)a + b + cin;
  *cout = (uint32_t)(s >> 32);
  return (uint32_t)s;
#endif
}
ZK_HD uint32_t subb32(uint32_t a, uint32_t b, uint32_t bin, uint32_t* bout) {
#if defined(__clang__)
  unsigned int c;
  uint32_t r = __builtin_subc(a, b, bin, &c);
  *bout = c;
  return r;
#else
  uint64_t d = (uint64_t)a - b - bin;
  *bout = (uint32_t)(d >> 63);
  return (uint32_t)d;
#endif
}
// 32x32 + 32 -> 64 (maps to one v_mad_u64_u32 with a zero-extended addend)
ZK_HD uint64_t mad64(uint32_t a, uint32_t b, uint32_t c) { return (uint64_t)a * b + c; }

// ---- field operations ------------------------------------------------------
template <class F>
ZK_HD Fe fe_zero() {
  Fe r;
#pragma unroll
  for (int i = 0; i < 8; ++i) r.v[i] = 0;
  return r;
}
template <class F>
ZK_HD Fe fe_one() {  // Montgomery image of 1 = R mod p
  Fe r;
#pragma unroll
  for (int i = 0; i < 8; ++i) r.v[i] = F::R1[i];
  return r;
}
template <class F>
ZK_HD Fe fe_inv2() {
  Fe r;
#pragma unroll
  for (int i = 0; i < 8; ++i) r.v[i] = F::INV2[i];
  return r;
}

// r = x - p if x >= p else x   (x < 2p, x < 2^256)
template <class F>
ZK_HD Fe fe_reduce_once(const Fe& x) {
  Fe t;
  uint32_t b = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) t.v[i] = subb32(x.v[i], F::P[i], b, &b);
  Fe r;
#pragma unroll
  for (int i = 0; i < 8; ++i) r.v[i] = b ? x.v[i] : t.v[i];
  return r;
}

template <class F>
ZK_HD Fe fe_add(const Fe& a, const Fe& b) {
  // p < 2^255, so a + b < 2^256: no carry out of the top limb.
  Fe s;
  uint32_t c = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) s.v[i] = addc32(a.v[i], b.v[i], c, &c);
  return fe_reduce_once<F>(s);
}

template <class F>
ZK_HD Fe fe_sub(const Fe& a, const Fe& b) {
  Fe d;
  uint32_t bw = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) d.v[i] = subb32(a.v[i], b.v[i], bw, &bw);
  // if borrow: d += p (mask form keeps the wave uniform)
  const uint32_t mask = 0u - bw;
  uint32_t c = 0;
  Fe r;
#pragma unroll
  for (int i = 0; i < 8; ++i) r.v[i] = addc32(d.v[i], F::P[i] & mask, c, &c);
  return r;
}

template <class F>
ZK_HD Fe fe_dbl(const Fe& a) {
  return fe_add<F>(a, a);
}

// Montgomery product a*b*R^-1 mod p, CIOS over 32-bit words.
// Row A: u = t + a*b_i (8 mads on zero-extended t_j, then one carry chain
// folding hi(P_{j-1}) into lo(P_j)). Row B: u += m*p, shift one word down.
// Invariant t < 2p < 2^256 between rows (p < 2^255).
template <class F>
ZK_HD Fe fe_mul(const Fe& a, const Fe& b) {
  uint32_t t[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) t[j] = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const uint32_t bi = b.v[i];
    uint64_t P[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) P[j] = mad64(a.v[j], bi, t[j]);
    uint32_t u[9];
    uint32_t c = 0;
    u[0] = (uint32_t)P[0];
#pragma unroll
    for (int j = 1; j < 8; ++j) u[j] = addc32((uint32_t)P[j], (uint32_t)(P[j - 1] >> 32), c, &c);
    u[8] = (uint32_t)(P[7] >> 32) + c;
    const uint32_t m = u[0] * F::PINV;
    uint64_t Q[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) Q[j] = mad64(m, F::P[j], u[j]);
    c = 0;
#pragma unroll
    for (int j = 1; j < 8; ++j) t[j - 1] = addc32((uint32_t)Q[j], (uint32_t)(Q[j - 1] >> 32), c, &c);
    t[7] = u[8] + (uint32_t)(Q[7] >> 32) + c;
  }
  Fe r;
#pragma unroll
  for (int j = 0; j < 8; ++j) r.v[j] = t[j];
  return fe_reduce_once<F>(r);
}

// ---- unreduced products (lazy reduction) ------------------------------------
// Sums of products of Montgomery images are accumulated as 544-bit integers
// (17 words) and reduced once: REDC is linear, so
// REDC(sum a_i b_i) = sum REDC(a_i b_i) mod p. Saves the 72 reduction mads of
// every accumulated product (one full fe_mul is 136).
struct Wide {
  uint32_t w[17];
};
template <class F>
ZK_HD Wide wide_zero() {
  Wide r;
#pragma unroll
  for (int i = 0; i < 17; ++i) r.w[i] = 0;
  return r;
}
// acc += a * b  (512-bit product by rows of v_mad_u64_u32 + one carry chain each)
template <class F>
ZK_HD void wide_mac(Wide& acc, const Fe& a, const Fe& b) {
  uint32_t t[16];
  {
    uint64_t P[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) P[j] = (uint64_t)a.v[j] * b.v[0];
    uint32_t c = 0;
    t[0] = (uint32_t)P[0];
#pragma unroll
    for (int j = 1; j < 8; ++j) t[j] = addc32((uint32_t)P[j], (uint32_t)(P[j - 1] >> 32), c, &c);
    t[8] = (uint32_t)(P[7] >> 32) + c;
  }
#pragma unroll
  for (int i = 1; i < 8; ++i) {
    uint64_t P[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) P[j] = mad64(a.v[j], b.v[i], t[i + j]);
    uint32_t c = 0;
    t[i] = (uint32_t)P[0];
#pragma unroll
    for (int j = 1; j < 8; ++j) t[i + j] = addc32((uint32_t)P[j], (uint32_t)(P[j - 1] >> 32), c, &c);
    t[i + 8] = (uint32_t)(P[7] >> 32) + c;  // the partial product fits i+9 words
  }
  uint32_t c = 0;
#pragma unroll
  for (int k = 0; k < 16; ++k) acc.w[k] = addc32(acc.w[k], t[k], c, &c);
  acc.w[16] += c;
}
template <class F>
ZK_HD void wide_add(Wide& acc, const Wide& x) {
  uint32_t c = 0;
#pragma unroll
  for (int k = 0; k < 17; ++k) acc.w[k] = addc32(acc.w[k], x.w[k], c, &c);
}
// REDC of a 544-bit value: V * 2^-256 mod p, fully reduced
template <class F>
ZK_HD Fe wide_redc(const Wide& V) {
  uint32_t t[18];
#pragma unroll
  for (int k = 0; k < 17; ++k) t[k] = V.w[k];
  t[17] = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const uint32_t m = t[i] * F::PINV;
    uint64_t Q[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) Q[j] = mad64(m, F::P[j], t[i + j]);
    uint32_t c = 0;
#pragma unroll
    for (int j = 1; j < 8; ++j) t[i + j] = addc32((uint32_t)Q[j], (uint32_t)(Q[j - 1] >> 32), c, &c);
    t[i + 8] = addc32(t[i + 8], (uint32_t)(Q[7] >> 32), c, &c);
#pragma unroll
    for (int q = i + 9; q < 18; ++q) t[q] = addc32(t[q], 0u, c, &c);
  }
  // T = t[8..17] < 2^288 + p:  T mod p = (lo256 mod p) + hi * 2^256 mod p
  Fe lo;
#pragma unroll
  for (int k = 0; k < 8; ++k) lo.v[k] = t[8 + k];
#pragma unroll
  for (int k = 0; k < 5; ++k) lo = fe_reduce_once<F>(lo);
  Fe hi = fe_zero<F>();
  hi.v[0] = t[16];
  hi.v[1] = t[17];
  Fe r2;
#pragma unroll
  for (int k = 0; k < 8; ++k) r2.v[k] = F::R2[k];
  return fe_add<F>(lo, fe_mul<F>(hi, r2));  // hi * R mod p
}

// Fold by two challenges at once (two successive partial_evaluate(0, .) calls,
// multilinear_polynomial_evaluation.rs:52-63): for the four table entries
// x_ab (a = first folded variable, b = second)
//   Z = x00 + ra (x10 - x00) + rb (x01 - x00) + ra rb (x11 - x10 - x01 + x00)
// The three products are summed unreduced and reduced by ONE REDC: 3 x 64 +
// 64 mads instead of 3 chained Montgomery multiplies (3 x 128). rab = ra*rb.
// The sum W < 3 p^2 < 2^512 (p < 2^255), so REDC(W) < W / 2^256 + p < 3p and
// fits 9 words; two conditional subtractions bring it into [0, p).
template <class F>
ZK_HD Fe redc3p(const Wide& W) {
  uint32_t t[17];
#pragma unroll
  for (int k = 0; k < 17; ++k) t[k] = W.w[k];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const uint32_t m = t[i] * F::PINV;
    uint64_t Q[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) Q[j] = mad64(m, F::P[j], t[i + j]);
    uint32_t c = 0;
#pragma unroll
    for (int j = 1; j < 8; ++j) t[i + j] = addc32((uint32_t)Q[j], (uint32_t)(Q[j - 1] >> 32), c, &c);
    t[i + 8] = addc32(t[i + 8], (uint32_t)(Q[7] >> 32), c, &c);
#pragma unroll
    for (int q = i + 9; q < 17; ++q) t[q] = addc32(t[q], 0u, c, &c);
  }
  // V = t[8..16] < 3p: subtract p while V >= p (at most twice)
#pragma unroll
  for (int pass = 0; pass < 2; ++pass) {
    uint32_t d[9], b = 0;
#pragma unroll
    for (int k = 0; k < 8; ++k) d[k] = subb32(t[8 + k], F::P[k], b, &b);
    d[8] = subb32(t[16], 0u, b, &b);
#pragma unroll
    for (int k = 0; k < 9; ++k) t[8 + k] = b ? t[8 + k] : d[k];
  }
  Fe r;
#pragma unroll
  for (int k = 0; k < 8; ++k) r.v[k] = t[8 + k];
  return r;
}
template <class F>
ZK_HD Fe fold2(const Fe& x00, const Fe& x01, const Fe& x10, const Fe& x11, const Fe& ra, const Fe& rb,
               const Fe& rab) {
  const Fe d1 = fe_sub<F>(x10, x00);
  const Fe d2 = fe_sub<F>(x01, x00);
  const Fe d3 = fe_sub<F>(fe_sub<F>(x11, x01), d1);
  Wide w = wide_zero<F>();
  wide_mac<F>(w, ra, d1);
  wide_mac<F>(w, rb, d2);
  wide_mac<F>(w, rab, d3);
  return fe_add<F>(x00, redc3p<F>(w));
}

// Limb sums -> field element. w[i] (i < L <= 17) are sums of 32-bit words at
// weight 2^(32 i) (each < 2^62), i.e. the integer T = sum_i w[i] 2^(32 i) < 2^624.
// Split T = C0 + C1 R + C2 R^2 (R = 2^256).
//   product sums (sums of a*b over Montgomery images, T ~ R^2 x):  T R^-1 = C0 R^-1 + C1 + C2 R
//   element sums (sums of Montgomery images, T ~ R x):            T      = C0 + C1 R          (C2 = 0)
template <class F>
ZK_HD Fe limbs_to_fe(const uint64_t* w, int L, bool product) {
  uint32_t t[24];
  uint64_t carry = 0;
  for (int i = 0; i < 24; ++i) {
    const uint64_t s = (i < L ? w[i] : 0) + carry;
    t[i] = (uint32_t)s;
    carry = s >> 32;
  }
  Fe ch[3];
  for (int c = 0; c < 3; ++c) {
    for (int k = 0; k < 8; ++k) ch[c].v[k] = t[8 * c + k];
    for (int k = 0; k < 5; ++k) ch[c] = fe_reduce_once<F>(ch[c]);  // 2^256 < 6p
  }
  Fe r2, one = fe_zero<F>();
  for (int k = 0; k < 8; ++k) r2.v[k] = F::R2[k];
  one.v[0] = 1;
  if (product) return fe_add<F>(fe_add<F>(fe_mul<F>(ch[0], one), ch[1]), fe_mul<F>(ch[2], r2));
  return fe_add<F>(ch[0], fe_mul<F>(ch[1], r2));
}

template <class F>
ZK_HD Fe fe_to_mont(const Fe& canon) {  // canon < p
  Fe r2;
#pragma unroll
  for (int i = 0; i < 8; ++i) r2.v[i] = F::R2[i];
  return fe_mul<F>(canon, r2);
}
template <class F>
ZK_HD Fe fe_from_mont(const Fe& m) {
  Fe one = fe_zero<F>();
  one.v[0] = 1;
  return fe_mul<F>(m, one);
}

template <class F>
ZK_HD bool fe_is_zero(const Fe& a) {
  uint32_t acc = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) acc |= a.v[i];
  return acc == 0;
}
template <class F>
ZK_HD bool fe_eq(const Fe& a, const Fe& b) {
  uint32_t acc = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) acc |= a.v[i] ^ b.v[i];
  return acc == 0;
}
// canonical < p ?
template <class F>
ZK_HD bool fe_is_canonical(const Fe& x) {
  uint32_t b = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) (void)subb32(x.v[i], F::P[i], b, &b);
  return b != 0;
}

// 2^e mod p as a plain (non-Montgomery) integer, at compile time (e doublings)
template <class F>
constexpr Fe pow2_mod_p(int e) {
  Fe x{};
  x.v[0] = 1;
  for (int i = 0; i < e; ++i) {
    uint32_t y[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    uint32_t c = 0;
    for (int k = 0; k < 8; ++k) {
      const uint64_t s = ((uint64_t)x.v[k] << 1) | c;
      y[k] = (uint32_t)s;
      c = (uint32_t)(s >> 32);
    }
    bool ge = true;  // y >= p (y < 2p < 2^256)
    for (int k = 7; k >= 0; --k)
      if (y[k] != F::P[k]) {
        ge = y[k] > F::P[k];
        break;
      }
    if (ge) {
      uint32_t b = 0;
      for (int k = 0; k < 8; ++k) {
        const uint64_t d = (uint64_t)y[k] - F::P[k] - b;
        y[k] = (uint32_t)d;
        b = (uint32_t)(d >> 63);
      }
    }
    for (int k = 0; k < 8; ++k) x.v[k] = y[k];
  }
  return x;
}

}  // namespace zk
