// Device-resident Fiat-Shamir step.
//
// After challenge k-1 the transcript sponge is always "fresh state + the
// 32-byte digest d_{k-1} buffered" (get_random_challenge = finalize_reset,
// then append(d): fiat_shamir_transcript.rs:28-37). Round k then appends at
// most three 32-byte coefficients (GKR, trimmed) or exactly two (plain
// sum-check) and draws r_k: 32 + <=96 bytes < the 136-byte Keccak rate, so
// the whole step is ONE Keccak-f[1600] of (d_{k-1} || coeffs || pad) from the
// zero state. The round kernel's last block runs it on wave 0 and writes an
// FsRec; the next round kernel reads r_k from that record, so rounds 1..n-1
// are enqueued back to back with no host round trip.
//
// Same arithmetic as the host path (zk_sumcheck.hip finish_round / challenge):
//   e1 = s_{k-1}(r_{k-1}) - e0      (GKR rounds k >= 1)
//   c0 = e0, c2 = (e0 - 2 e1 + e2)/2, c1 = e1 - e0 - c2   (interpolate, :48-74)
//   trim trailing zero coefficients (univariate_polynomial_dense.rs:14-18)
//   r_k = from_le_bytes_mod_order(d_k); claim_k = s_k(r_k) (Horner)
#pragma once
#include "field.hpp"

namespace zk {

enum FsMode : uint32_t { FS_GKR = 0, FS_PLAIN = 1 };

struct alignas(256) FsRec {
  Fe r;                // challenge r_k (Montgomery)
  Fe claim;            // GKR: s_k(r_k) (Montgomery); plain: unused
  uint32_t digest[8];  // d_k: the Keccak digest r_k was read from
  Fe coeff[3];         // GKR: s_k coefficients, plain: (s0, s1); Montgomery, zero past ncoeff
  uint32_t ncoeff;
};

// ---------------------------------------------------------------------------
// Keccak-f[1600] across a wave: lane l < 25 holds state word l = x + 5y.
// Per round two LDS exchanges: theta reads the two neighbouring columns'
// parities (10 words), rho rotates in-lane, pi+chi read the three B words the
// lane's row needs (3 words). LDS ops of one wave complete in order, so no
// barrier is needed; the wavefront fence only stops compiler reordering.
// ---------------------------------------------------------------------------
namespace kdetail {
constexpr int kRho[25] = {0, 1, 62, 28, 27, 36, 44, 6, 55, 20, 3, 10, 43, 25, 39, 41, 45, 15, 21, 8, 18, 2, 61, 56, 14};
constexpr uint64_t pack_rho(int first, int n) {
  uint64_t k = 0;
  for (int i = 0; i < n; ++i) k |= (uint64_t)((64 - kRho[first + i]) & 63) << (6 * i);
  return k;
}
constexpr uint64_t kRotR0 = pack_rho(0, 10), kRotR1 = pack_rho(10, 10), kRotR2 = pack_rho(20, 5);
constexpr uint64_t kRC[24] = {
    0x0000000000000001ull, 0x0000000000008082ull, 0x800000000000808aull, 0x8000000080008000ull,
    0x000000000000808bull, 0x0000000080000001ull, 0x8000000080008081ull, 0x8000000000008009ull,
    0x000000000000008aull, 0x0000000000000088ull, 0x0000000080008009ull, 0x000000008000000aull,
    0x000000008000808bull, 0x800000000000008bull, 0x8000000000008089ull, 0x8000000000008003ull,
    0x8000000000008002ull, 0x8000000000000080ull, 0x000000000000800aull, 0x800000008000000aull,
    0x8000000080008081ull, 0x8000000000008080ull, 0x0000000080000001ull, 0x8000000080008008ull};
}  // namespace kdetail

struct U2 {
  uint32_t lo, hi;
};
__device__ __forceinline__ U2 u2(uint64_t x) { return {(uint32_t)x, (uint32_t)(x >> 32)}; }
__device__ __forceinline__ uint64_t u64(U2 x) { return (uint64_t)x.lo | ((uint64_t)x.hi << 32); }
__device__ __forceinline__ U2 u2xor(U2 a, U2 b) { return {a.lo ^ b.lo, a.hi ^ b.hi}; }
// rotate right by u in [0, 63]: optional word swap + two funnel shifts
__device__ __forceinline__ U2 rotr_var(U2 x, uint32_t u) {
  const bool sw = u & 32u;
  const uint32_t lo = sw ? x.hi : x.lo, hi = sw ? x.lo : x.hi, s = u & 31u;
  return {__builtin_amdgcn_alignbit(hi, lo, s), __builtin_amdgcn_alignbit(lo, hi, s)};
}
__device__ __forceinline__ U2 rotl1(U2 x) {
  return {__builtin_amdgcn_alignbit(x.lo, x.hi, 31), __builtin_amdgcn_alignbit(x.hi, x.lo, 31)};
}

// `a` = this lane's state word (lanes >= 25: ignored, returns 0).
// sa, sb: 32-word LDS scratch each.
__device__ __forceinline__ uint64_t keccak_f_lanes(uint64_t a_in, uint32_t lane, uint64_t* sa, uint64_t* sb) {
  if (lane >= 25) return 0;
  const uint32_t x = lane % 5u, y = lane / 5u;
  const uint32_t xm = (x + 4u) % 5u, xp = (x + 1u) % 5u;
  const uint64_t rk = lane < 10 ? kdetail::kRotR0 : lane < 20 ? kdetail::kRotR1 : kdetail::kRotR2;
  const uint32_t rotr = (uint32_t)(rk >> (6 * (lane < 10 ? lane : lane < 20 ? lane - 10 : lane - 20))) & 63u;
  // B(X, Y) = rho(A(xs, ys)) with ys = X, xs = 3 (Y - 3X) mod 5 (pi inverted)
  auto src = [](uint32_t X, uint32_t Y) { return (3u * (Y + 15u - 3u * X)) % 5u + 5u * X; };
  const uint32_t s0 = src(x, y), s1 = src(xp, y), s2 = src((x + 2u) % 5u, y);
  U2 a = u2(a_in);
#pragma unroll
  for (int round = 0; round < 24; ++round) {
    sa[lane] = u64(a);
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    U2 cm = u2(sa[xm] ^ sa[xm + 5] ^ sa[xm + 10] ^ sa[xm + 15] ^ sa[xm + 20]);
    U2 cp = u2(sa[xp] ^ sa[xp + 5] ^ sa[xp + 10] ^ sa[xp + 15] ^ sa[xp + 20]);
    a = u2xor(a, u2xor(cm, rotl1(cp)));          // theta
    a = rotr_var(a, rotr);                        // rho
    sb[lane] = u64(a);
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    const uint64_t b0 = sb[s0], b1 = sb[s1], b2 = sb[s2];  // pi
    uint64_t na = b0 ^ (~b1 & b2);                // chi
    if (lane == 0) na ^= kdetail::kRC[round];     // iota
    a = u2(na);
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  }
  return u64(a);
}

template <class F>
__device__ __forceinline__ Fe fe_half(const Fe& x) {  // x / 2 mod p (x < p); Montgomery-linear
  const uint32_t odd = 0u - (x.v[0] & 1u);
  uint32_t t[8], c = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) t[i] = addc32(x.v[i], F::P[i] & odd, c, &c);  // < 2p < 2^256
  Fe r;
#pragma unroll
  for (int i = 0; i < 7; ++i) r.v[i] = __builtin_amdgcn_alignbit(t[i + 1], t[i], 1);
  r.v[7] = t[7] >> 1;
  return r;
}

__device__ __forceinline__ Fe ld_fe_u(const Fe* p) {  // wave-uniform 32-B load
  Fe x;
#pragma unroll
  for (int i = 0; i < 8; ++i) x.v[i] = p->v[i];
  return x;
}

// One Fiat-Shamir step on wave 0 (all 64 lanes call it with the same e[]).
// GKR: e[] = (e0, e2) of round k (e1 derived from prev->claim) or, when
// has_e1, (e0, e1, e2). Plain: e[] = (s0, s1). Writes *out (lane 0).
template <class F>
__device__ __forceinline__ void fs_step_wave(uint32_t mode, const Fe* e, bool has_e1, const FsRec* __restrict__ prev,
                                             FsRec* __restrict__ out, uint64_t* lds /* >= 96 words */) {
  const uint32_t lane = threadIdx.x & 63u;
  Fe c[3];
  uint32_t m;
  if (mode == FS_GKR) {
    const Fe e0 = e[0];
    const Fe e1 = has_e1 ? e[1] : fe_sub<F>(ld_fe_u(&prev->claim), e0);
    const Fe e2 = has_e1 ? e[2] : e[1];
    c[0] = e0;
    c[2] = fe_half<F>(fe_sub<F>(fe_add<F>(e0, e2), fe_dbl<F>(e1)));
    c[1] = fe_sub<F>(fe_sub<F>(e1, e0), c[2]);
    m = !fe_is_zero<F>(c[2]) ? 3u : !fe_is_zero<F>(c[1]) ? 2u : !fe_is_zero<F>(c[0]) ? 1u : 0u;
  } else {
    c[0] = e[0];
    c[1] = e[1];
    c[2] = fe_zero<F>();
    m = 2;
  }
  // canonical bytes of the absorbed coefficients: lane i converts c_i
  uint64_t* blk = lds + 64;  // 17-word message block
  if (lane < 3) {
    Fe x = c[0];
    if (lane == 1) x = c[1];
    if (lane == 2) x = c[2];
    const Fe cc = fe_from_mont<F>(x);
#pragma unroll
    for (int j = 0; j < 4; ++j) blk[4 + 4 * lane + j] = lane < m ? ((uint64_t)cc.v[2 * j] | ((uint64_t)cc.v[2 * j + 1] << 32)) : 0;
  }
  if (lane < 4) blk[lane] = (uint64_t)prev->digest[2 * lane] | ((uint64_t)prev->digest[2 * lane + 1] << 32);
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  uint64_t w = 0;
  if (lane < 16) w = blk[lane];  // words 4m+4.. are zero (lanes < 3 zeroed unused coefficients)
  if (lane == 4 + 4 * m) w ^= 0x01ull;                 // pad10*1, first byte
  if (lane == 16) w ^= 0x80ull << 56;                  // last byte of the 136-byte block
  const uint64_t st = keccak_f_lanes(w, lane, lds, lds + 32);
  if (lane < 4) blk[lane] = st;
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  Fe d;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const uint64_t v = blk[j];
    d.v[2 * j] = (uint32_t)v;
    d.v[2 * j + 1] = (uint32_t)(v >> 32);
  }
  Fe r = d;
#pragma unroll
  for (int i = 0; i < 5; ++i) r = fe_reduce_once<F>(r);  // 2^256 < 6p
  const Fe rm = fe_to_mont<F>(r);
  Fe claim = fe_zero<F>();
  if (mode == FS_GKR) claim = fe_add<F>(c[0], fe_mul<F>(rm, fe_add<F>(c[1], fe_mul<F>(rm, c[2]))));
  if (lane == 0) {
    out->r = rm;
    out->claim = claim;
#pragma unroll
    for (int i = 0; i < 8; ++i) out->digest[i] = d.v[i];
#pragma unroll
    for (int i = 0; i < 3; ++i) out->coeff[i] = (uint32_t)i < m ? c[i] : fe_zero<F>();
    out->ncoeff = m;
  }
}

}  // namespace zk
