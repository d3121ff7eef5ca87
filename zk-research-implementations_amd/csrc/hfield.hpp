// Host-only field arithmetic on 4 x 64-bit limbs (unsigned __int128 products)
// for the per-round hand-off: the same values as the 8 x 32-bit ZK_HD
// templates of field.hpp (Montgomery form, R = 2^256, every result fully
// reduced), at about a quarter of the instructions. Fe's 8 LE u32 limbs are
// the same bytes as 4 LE u64 limbs.
#pragma once
#include <stdint.h>
#include <string.h>

#include "field.hpp"

namespace zk {
namespace h64 {
using u128 = unsigned __int128;
struct V {
  uint64_t l[4];
};
inline V of(const Fe& x) {
  V r;
  memcpy(r.l, x.v, 32);
  return r;
}
inline Fe fe(const V& x) {
  Fe r;
  memcpy(r.v, x.l, 32);
  return r;
}
template <class F>
constexpr uint64_t P(int i) {
  return (uint64_t)F::P[2 * i] | ((uint64_t)F::P[2 * i + 1] << 32);
}
template <class F>
constexpr uint64_t pinv() {  // -p^-1 mod 2^64 (Newton)
  uint64_t x = 1;
  for (int i = 0; i < 7; ++i) x *= 2 - P<F>(0) * x;
  return (uint64_t)0 - x;
}
// x - p if x >= p (x < 2^256 + carry bit `hi`), branch-free
template <class F>
inline V sub_p_if_ge(const V& x, uint64_t hi = 0) {
  V d;
  unsigned long b = 0;
  for (int i = 0; i < 4; ++i) d.l[i] = __builtin_subcl(x.l[i], P<F>(i), b, &b);
  const uint64_t keep = (uint64_t)0 - (uint64_t)(b & (hi ^ 1));  // all ones: x < p, keep x
  V r;
  for (int i = 0; i < 4; ++i) r.l[i] = (x.l[i] & keep) | (d.l[i] & ~keep);
  return r;
}
template <class F>
inline V add(const V& a, const V& b) {  // p < 2^255: no carry out
  V s;
  unsigned long c = 0;
  for (int i = 0; i < 4; ++i) s.l[i] = __builtin_addcl(a.l[i], b.l[i], c, &c);
  return sub_p_if_ge<F>(s);
}
template <class F>
inline V sub(const V& a, const V& b) {
  V d;
  unsigned long bw = 0;
  for (int i = 0; i < 4; ++i) d.l[i] = __builtin_subcl(a.l[i], b.l[i], bw, &bw);
  const uint64_t mask = (uint64_t)0 - (uint64_t)bw;
  unsigned long c = 0;
  for (int i = 0; i < 4; ++i) d.l[i] = __builtin_addcl(d.l[i], P<F>(i) & mask, c, &c);
  return d;
}
// Montgomery product a b R^-1 mod p (CIOS, 4 x 64)
template <class F>
inline V mul(const V& a, const V& b) {
  uint64_t t[6] = {0, 0, 0, 0, 0, 0};
  for (int i = 0; i < 4; ++i) {
    uint64_t C = 0;
    for (int j = 0; j < 4; ++j) {
      const u128 s = (u128)a.l[j] * b.l[i] + t[j] + C;
      t[j] = (uint64_t)s;
      C = (uint64_t)(s >> 64);
    }
    u128 s = (u128)t[4] + C;
    t[4] = (uint64_t)s;
    t[5] = (uint64_t)(s >> 64);
    const uint64_t m = t[0] * pinv<F>();
    s = (u128)m * P<F>(0) + t[0];
    C = (uint64_t)(s >> 64);
    for (int j = 1; j < 4; ++j) {
      s = (u128)m * P<F>(j) + t[j] + C;
      t[j - 1] = (uint64_t)s;
      C = (uint64_t)(s >> 64);
    }
    s = (u128)t[4] + C;
    t[3] = (uint64_t)s;
    t[4] = t[5] + (uint64_t)(s >> 64);
  }
  V r;
  for (int j = 0; j < 4; ++j) r.l[j] = t[j];
  return sub_p_if_ge<F>(r, t[4]);
}
template <class F>
inline V reduce(V x) {  // any 256-bit x -> x mod p (2^256 < 6p)
  for (int k = 0; k < 5; ++k) x = sub_p_if_ge<F>(x);
  return x;
}
// Montgomery reduction of a 512-bit T = (lo, hi) with hi < p: T R^-1 mod p
// (T < p R, so the result before the final subtraction is < 2p)
template <class F>
inline V redc512(const uint64_t (&x)[8]) {
  uint64_t t[9];
  for (int i = 0; i < 8; ++i) t[i] = x[i];
  t[8] = 0;
  for (int i = 0; i < 4; ++i) {
    const uint64_t m = t[i] * pinv<F>();
    uint64_t c = 0;
    for (int j = 0; j < 4; ++j) {
      const u128 s = (u128)m * P<F>(j) + t[i + j] + c;
      t[i + j] = (uint64_t)s;
      c = (uint64_t)(s >> 64);
    }
    for (int k = i + 4; k < 9 && c; ++k) {
      const u128 s = (u128)t[k] + c;
      t[k] = (uint64_t)s;
      c = (uint64_t)(s >> 64);
    }
  }
  V r = {{t[4], t[5], t[6], t[7]}};
  return sub_p_if_ge<F>(r, t[8]);
}
template <class F>
inline bool lt_p(const uint64_t* x) {  // x[0..3] < p
  unsigned long b = 0;
  for (int i = 0; i < 4; ++i) (void)__builtin_subcl(x[i], P<F>(i), b, &b);
  return b != 0;
}
// acc (9 limbs) += a b (512-bit product, no reduction)
inline void mac_wide(uint64_t (&acc)[9], const V& a, const V& b) {
  uint64_t pr[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  for (int i = 0; i < 4; ++i) {
    uint64_t c = 0;
    for (int j = 0; j < 4; ++j) {
      const u128 s = (u128)a.l[j] * b.l[i] + pr[i + j] + c;
      pr[i + j] = (uint64_t)s;
      c = (uint64_t)(s >> 64);
    }
    pr[i + 4] = c;
  }
  unsigned long c = 0;
  for (int k = 0; k < 8; ++k) acc[k] = __builtin_addcl(acc[k], pr[k], c, &c);
  acc[8] += c;
}
template <class F>
inline V r2() {
  V r;
  for (int i = 0; i < 4; ++i) r.l[i] = (uint64_t)F::R2[2 * i] | ((uint64_t)F::R2[2 * i + 1] << 32);
  return r;
}
}  // namespace h64

// Host versions of the field.hpp operations used per round (same results).
template <class F>
inline Fe hfe_mul(const Fe& a, const Fe& b) {
  return h64::fe(h64::mul<F>(h64::of(a), h64::of(b)));
}
template <class F>
inline Fe hfe_add(const Fe& a, const Fe& b) {
  return h64::fe(h64::add<F>(h64::of(a), h64::of(b)));
}
template <class F>
inline Fe hfe_sub(const Fe& a, const Fe& b) {
  return h64::fe(h64::sub<F>(h64::of(a), h64::of(b)));
}
// x / 2 mod p (x < p; Montgomery-linear: the image of x/2 is half the image of x)
template <class F>
inline Fe hfe_half(const Fe& x) {
  h64::V v = h64::of(x);
  const uint64_t odd = (uint64_t)0 - (v.l[0] & 1);
  unsigned long c = 0;
  for (int i = 0; i < 4; ++i) v.l[i] = __builtin_addcl(v.l[i], h64::P<F>(i) & odd, c, &c);  // < 2p < 2^256
  for (int i = 0; i < 3; ++i) v.l[i] = (v.l[i] >> 1) | (v.l[i + 1] << 63);
  v.l[3] >>= 1;
  return h64::fe(v);
}
template <class F>
inline Fe hfe_from_mont(const Fe& m) {
  h64::V one = {{1, 0, 0, 0}};
  return h64::fe(h64::mul<F>(h64::of(m), one));
}
template <class F>
inline Fe hfe_to_mont(const Fe& canon_any) {  // any 256-bit value, reduced mod p first
  return h64::fe(h64::mul<F>(h64::reduce<F>(h64::of(canon_any)), h64::r2<F>()));
}
// limbs_to_fe (field.hpp) on 64-bit limbs
template <class F>
inline Fe hlimbs_to_fe(const uint64_t* w, int L, bool product) {
  if (product && L <= 9) {  // the matrix-core steps' 9 limb sums: T < 2^320 < p R, one REDC
    using u128 = unsigned __int128;
    uint64_t t8[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    u128 acc = 0;
    for (int k = 0; k < 5; ++k) {
      acc += (u128)(2 * k < L ? w[2 * k] : 0) + ((u128)(2 * k + 1 < L ? w[2 * k + 1] : 0) << 32);
      t8[k] = (uint64_t)acc;
      acc >>= 64;
    }
    t8[5] = (uint64_t)acc;
    return h64::fe(h64::redc512<F>(t8));
  }
  // T = sum_i w[i] 2^(32 i): add the even words and the odd words shifted by
  // 32 into 64-bit limbs with carries
  uint64_t t[13] = {0};
  unsigned long c = 0;
  for (int k = 0; k < 12; ++k) {  // limb k gets w[2k] + (w[2k+1] << 32) + (w[2k-1] >> 32) + carry
    const uint64_t e = 2 * k < L ? w[2 * k] : 0;
    const uint64_t o = 2 * k + 1 < L ? w[2 * k + 1] : 0;
    const uint64_t prev_hi = 2 * k - 1 >= 0 && 2 * k - 1 < L ? (w[2 * k - 1] >> 32) : 0;
    unsigned long c1 = 0, c2 = 0;
    uint64_t s = __builtin_addcl(e, o << 32, 0, &c1);
    s = __builtin_addcl(s, prev_hi, 0, &c2);
    t[k] = __builtin_addcl(s, c, 0, &c);
    c += c1 + c2;
  }
  h64::V ch[3];
  for (int k = 0; k < 4; ++k) {
    ch[0].l[k] = t[k];
    ch[1].l[k] = t[4 + k];
    ch[2].l[k] = t[8 + k];
  }
  if (product && (t[8] | t[9] | t[10] | t[11]) == 0 && h64::lt_p<F>(t + 4)) {  // T < p R: one 512-bit REDC
    const uint64_t (&lo8)[8] = *reinterpret_cast<const uint64_t(*)[8]>(t);
    return h64::fe(h64::redc512<F>(lo8));
  }
  h64::V one = {{1, 0, 0, 0}};
  if (product)  // REDC(C0) + (C1 mod p) + C2 R   (mul(x, 1) is exact for any x < 2^256)
    return h64::fe(h64::add<F>(h64::add<F>(h64::mul<F>(ch[0], one), h64::reduce<F>(ch[1])),
                               h64::mul<F>(h64::reduce<F>(ch[2]), h64::r2<F>())));
  return h64::fe(h64::add<F>(h64::reduce<F>(ch[0]), h64::mul<F>(h64::reduce<F>(ch[1]), h64::r2<F>())));
}
// sum of products of Montgomery images accumulated by mac_wide -> Montgomery image of the field sum
template <class F>
inline Fe wide_to_fe(const uint64_t (&acc)[9]) {
  if (acc[8] == 0 && h64::lt_p<F>(acc + 4))  // < p R: one REDC (a few products of values < p)
    return h64::fe(h64::redc512<F>(*reinterpret_cast<const uint64_t(*)[8]>(acc)));
  uint64_t w[18];
  for (int k = 0; k < 9; ++k) {
    w[2 * k] = (uint32_t)acc[k];
    w[2 * k + 1] = acc[k] >> 32;
  }
  return hlimbs_to_fe<F>(w, 18, true);
}
}  // namespace zk
