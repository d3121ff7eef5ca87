// Device-resident Fiat-Shamir for the persistent double-step tail
// (ZK_DEVICE_FS=1, k_gkr_dtail<F, true>).
//
// The reference draws one challenge per round from its Keccak transcript
// (fiat_shamir_transcript.rs:23-29, sum_check_protocol.rs:96-108). After
// challenge k-1 the sponge is always "zero state + the 32-byte digest d_{k-1}
// buffered" (get_random_challenge = finalize_reset, then append(d):
// :28-37), and round k appends at most three 32-byte coefficients (GKR,
// trimmed), so 32 + <= 96 bytes < the 136-byte rate: the whole round is ONE
// Keccak-f[1600] of (d_{k-1} || LE32(c_0..c_{m-1}) || pad) from the zero
// state, and r_k = LE(d_k) mod p. A double step (two rounds, kernels.hpp
// k_gkr_dtail) therefore needs, after its eight product sums are in the last
// block's LDS: the sums reduced, round m's interpolation + Keccak, the claim
// s_m(r_m) and the Lagrange weights at r_m, round m+1's two values, its
// interpolation + Keccak, s_{m+1}(r_{m+1}) and r_m r_{m+1} — the arithmetic of
// host.hpp finish_round / two_rounds, value for value. Wave 0 of the block that
// counts in last runs it; independent products sit on different lanes of one
// instruction stream (no divergent branches), the Keccak permutation is spread
// over 25 lanes with two LDS exchanges per round.
#pragma once
#include "field.hpp"

namespace zk {

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

// Keccak-f[1600] across a wave (same permutation as keccak.hpp Keccak256::permute):
// lane l < 25 holds state word l = x + 5y. Per round two LDS exchanges: theta
// reads the two neighbouring columns' parities, rho rotates in-lane, pi + chi
// read the three B words the lane's row needs. LDS operations of one wave
// complete in order, so no barrier is needed; the wavefront fence only stops
// compiler reordering. `a` = this lane's state word (lanes >= 25: ignored,
// returns 0); sa, sb: 32-word LDS scratch each.
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
    a = u2xor(a, u2xor(cm, rotl1(cp)));  // theta
    a = rotr_var(a, rotr);               // rho
    sb[lane] = u64(a);
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    const uint64_t b0 = sb[s0], b1 = sb[s1], b2 = sb[s2];  // pi
    uint64_t na = b0 ^ (~b1 & b2);                           // chi
    if (lane == 0) na ^= kdetail::kRC[round];                // iota
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

// The relay words of a device-FS step (RPost, kernels.hpp): 0-23 (ra, rb, ra rb)
// as block_get_rs reads them, 24-31 the digest d the next round re-absorbs,
// 32-39 the claim s(r) of the last round; every word tagged (tag << 32 | value).
constexpr int kFsWords = 40;

// What one device double step hands the host (pinned, written with system-scope
// stores, `tag` last after the others drained): the two rounds' trimmed
// coefficients and challenges, which the host absorbs / draws again into its own
// transcript and compares (host.hpp replay_device_fs).
struct alignas(64) FsLog {
  uint32_t c[2][3][8];  // round coefficients (Montgomery images; zero past m)
  uint32_t r[2][8];     // challenges (Montgomery images)
  uint32_t m[2];        // trimmed coefficient counts
  uint32_t tag;         // the step's relay tag, written last
};

struct DfsScratch {
  uint64_t sa[32], sb[32], blk[20];
  Fe d[8];  // the step's eight product sums, reduced
  Fe v[8];  // per-lane results exchanged between stages
};

__device__ __forceinline__ Fe fe_ld_u(const Fe* p) {  // wave-uniform read of an LDS element
  Fe x;
#pragma unroll
  for (int i = 0; i < 8; ++i) x.v[i] = p->v[i];
  return x;
}
__device__ __forceinline__ Fe fe_sel(bool c, const Fe& a, const Fe& b) {
  Fe r;
#pragma unroll
  for (int i = 0; i < 8; ++i) r.v[i] = c ? a.v[i] : b.v[i];
  return r;
}
__device__ __forceinline__ void wave_sync_lds() { __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront"); }

// One round's Fiat-Shamir on wave 0 (every lane passes the same e0, e1, e2 and
// dig = d_{k-1}): interpolation through (0, e0), (1, e1), (2, e2)
// (univariate_polynomial_dense.rs:48-74, trailing zeros trimmed :14-18),
// append(fq_vec_to_bytes(c)) (:32-37), get_random_challenge. On return dig =
// d_k, r = r_k (Montgomery), c = the coefficients (Montgomery, zero past m).
template <class F>
__device__ __forceinline__ void dfs_round(const Fe& e0, const Fe& e1, const Fe& e2, uint32_t (&dig)[8], Fe& r,
                                          Fe (&c)[3], uint32_t& m, DfsScratch& s) {
  const uint32_t lane = threadIdx.x & 63u;
  c[0] = e0;
  c[2] = fe_half<F>(fe_sub<F>(fe_add<F>(e0, e2), fe_dbl<F>(e1)));
  c[1] = fe_sub<F>(fe_sub<F>(e1, e0), c[2]);
  m = !fe_is_zero<F>(c[2]) ? 3u : !fe_is_zero<F>(c[1]) ? 2u : !fe_is_zero<F>(c[0]) ? 1u : 0u;
  // the 136-byte block: words 0-3 the digest, 4 + 4i .. the canonical bytes of c_i
  {
    const Fe cc = fe_from_mont<F>(fe_sel(lane == 0, c[0], fe_sel(lane == 1, c[1], c[2])));  // lane i: c_i
    if (lane < 3) {
#pragma unroll
      for (int j = 0; j < 4; ++j)
        s.blk[4 + 4 * lane + j] = lane < m ? ((uint64_t)cc.v[2 * j] | ((uint64_t)cc.v[2 * j + 1] << 32)) : 0;
    }
#pragma unroll
    for (int j = 0; j < 4; ++j)  // (static indices: a lane-indexed register array would live in scratch)
      if (lane == (uint32_t)j) s.blk[j] = (uint64_t)dig[2 * j] | ((uint64_t)dig[2 * j + 1] << 32);
  }
  wave_sync_lds();
  uint64_t w = lane < 16 ? s.blk[lane] : 0;  // words past 4 + 4m are zero (lanes < 3 zeroed unused coefficients)
  if (lane == 4 + 4 * m) w ^= 0x01ull;       // pad10*1: first byte after the message
  if (lane == 16) w ^= 0x80ull << 56;        // last byte of the rate
  const uint64_t st = keccak_f_lanes(w, lane, s.sa, s.sb);
  if (lane < 4) s.blk[lane] = st;
  wave_sync_lds();
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const uint64_t v = s.blk[j];
    dig[2 * j] = (uint32_t)v;
    dig[2 * j + 1] = (uint32_t)(v >> 32);
  }
  Fe x;
#pragma unroll
  for (int i = 0; i < 8; ++i) x.v[i] = dig[i];
#pragma unroll
  for (int i = 0; i < 5; ++i) x = fe_reduce_once<F>(x);  // from_le_bytes_mod_order: 2^256 < 6p
  r = fe_to_mont<F>(x);
  wave_sync_lds();  // s.blk is rewritten by the next round
}

// A double step's two rounds on wave 0 of the last block (host.hpp two_rounds):
// tot = the 8 x 17 limb sums (categories 0 V00, 1 V22, 2 V01, 3 V02, 4 V10,
// 5 V20, 6 V21, 7 V12), claim = s_{m-1}(r_{m-1}), dig = d_{m-1}. Returns
// (r_m, r_{m+1}, r_m r_{m+1}) in rr, s_{m+1}(r_{m+1}) in claim, d_{m+1} in dig;
// lane 0 fills *log (not its tag).
// limbs_to_fe (field.hpp) of 17 product-sum limbs, fully unrolled (registers only)
template <class F>
__device__ __forceinline__ Fe limbs17_to_fe(const uint64_t* w) {
  uint32_t t[24];
  uint64_t carry = 0;
#pragma unroll
  for (int i = 0; i < 24; ++i) {
    const uint64_t x = (i < 17 ? w[i] : 0) + carry;
    t[i] = (uint32_t)x;
    carry = x >> 32;
  }
  Fe ch[3];
#pragma unroll
  for (int c = 0; c < 3; ++c) {
#pragma unroll
    for (int k = 0; k < 8; ++k) ch[c].v[k] = t[8 * c + k];
#pragma unroll
    for (int k = 0; k < 5; ++k) ch[c] = fe_reduce_once<F>(ch[c]);  // 2^256 < 6p
  }
  Fe r2, one = fe_zero<F>();
#pragma unroll
  for (int k = 0; k < 8; ++k) r2.v[k] = F::R2[k];
  one.v[0] = 1;
  return fe_add<F>(fe_add<F>(fe_mul<F>(ch[0], one), ch[1]), fe_mul<F>(ch[2], r2));
}

template <class F>
__device__ __forceinline__ void dfs_double(const uint64_t* tot, Fe& claim, uint32_t (&dig)[8], Fe (&rr)[3], FsLog* log,
                                        DfsScratch& s) {
  const uint32_t lane = threadIdx.x & 63u;
  {
    const Fe x = limbs17_to_fe<F>(tot + 17 * (lane & 7));
    if (lane < 8) s.d[lane] = x;
  }
  wave_sync_lds();
  Fe d[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) d[i] = fe_ld_u(&s.d[i]);
  wave_sync_lds();
  const Fe one = fe_one<F>(), two = fe_add<F>(one, one);
  // round m: e0 = V00 + V01, e1 = s_{m-1}(r_{m-1}) - e0, e2 = V20 + V21
  Fe c1[3], r1;
  uint32_t m1;
  {
    const Fe e0 = fe_add<F>(d[0], d[2]);
    dfs_round<F>(e0, fe_sub<F>(claim, e0), fe_add<F>(d[5], d[6]), dig, r1, c1, m1, s);
  }
  // claim s_m(r_m) = c0 + r (c1 + r c2) on lane 0; lanes 1-3 the Lagrange numerators
  // (r-1)(r-2), r(r-2), r(r-1) — one product per lane per stage
  const Fe rm1 = fe_sub<F>(r1, one), rm2 = fe_sub<F>(r1, two);
  {
    const Fe a = fe_sel(lane == 0, r1, fe_sel(lane == 1, rm1, r1));
    const Fe b = fe_sel(lane == 0, c1[2], fe_sel(lane == 3, rm1, rm2));
    Fe v = fe_mul<F>(a, b);
    v = fe_sel(lane == 0, fe_add<F>(v, c1[1]), v);
    const Fe v2 = fe_mul<F>(fe_sel(lane == 0, r1, one), v);  // lane 0: r (c1 + r c2); others: v (times R/R)
    if (lane < 4) s.v[lane] = v2;
  }
  wave_sync_lds();
  const Fe claim1 = fe_add<F>(c1[0], fe_ld_u(&s.v[0]));
  const Fe L0 = fe_half<F>(fe_ld_u(&s.v[1])), L1 = fe_sub<F>(fe_zero<F>(), fe_ld_u(&s.v[2])),
           L2 = fe_half<F>(fe_ld_u(&s.v[3]));
  wave_sync_lds();
  // round m+1's values at r_m: e0' through (V00, V10, V20), e2' through (V02, V12, V22) (lanes 0, 1)
  {
    Wide w = wide_zero<F>();
    wide_mac<F>(w, L0, fe_sel(lane == 0, d[0], d[3]));
    wide_mac<F>(w, L1, fe_sel(lane == 0, d[4], d[7]));
    wide_mac<F>(w, L2, fe_sel(lane == 0, d[5], d[1]));
    const Fe v = wide_redc<F>(w);
    if (lane < 2) s.v[lane] = v;
  }
  wave_sync_lds();
  const Fe f0 = fe_ld_u(&s.v[0]), f2 = fe_ld_u(&s.v[1]);
  wave_sync_lds();
  Fe c2[3], r2;
  uint32_t m2;
  dfs_round<F>(f0, fe_sub<F>(claim1, f0), f2, dig, r2, c2, m2, s);
  // lane 0: s_{m+1}(r_{m+1}) (Horner, two stages); lane 1: r_m r_{m+1}
  {
    Fe v = fe_mul<F>(r2, fe_sel(lane == 0, c2[2], r1));
    v = fe_sel(lane == 0, fe_add<F>(v, c2[1]), v);
    const Fe v2 = fe_mul<F>(fe_sel(lane == 0, r2, one), v);
    if (lane < 2) s.v[lane] = v2;
  }
  wave_sync_lds();
  claim = fe_add<F>(c2[0], fe_ld_u(&s.v[0]));
  rr[0] = r1;
  rr[1] = r2;
  rr[2] = fe_ld_u(&s.v[1]);
  wave_sync_lds();
  if (lane == 0 && log) {
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        __hip_atomic_store(&log->c[0][i][k], c1[i].v[k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        __hip_atomic_store(&log->c[1][i][k], c2[i].v[k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      }
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      __hip_atomic_store(&log->r[0][k], r1.v[k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      __hip_atomic_store(&log->r[1][k], r2.v[k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
    __hip_atomic_store(&log->m[0], m1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __hip_atomic_store(&log->m[1], m2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

}  // namespace zk
