// Round sums on the matrix cores (gfx950 v_mfma_i32_32x32x32_i8).
//
// A round's product sums are dot products over the hypercube,
//   sum_j X_j * Y_j   (X, Y = the tables of one product at one grid point;
//                      sum_check_protocol.rs:152-166 via composed_polynomial.rs:88-99),
// and written in 8-bit digits x_j = sum_k x_jk 2^(8k) they are an integer
// matrix product:
//   sum_j X_j Y_j = sum_{k,l} 2^(8(k+l)) C[k][l],   C[k][l] = sum_j x_jk y_jl,
// i.e. C = x^T y, a 32 x 32 (digit positions) x J (hypercube points)
// contraction that the int8 MFMA computes EXACTLY in int32. The field
// multiplications of the sums thus leave the VALU (whose 256-bit multiply
// bound the previous kernels) for the matrix cores, which have
// ~500x the throughput needed, and the kernel becomes bound by HBM.
//
// Signed digits. The MFMA multiplies signed int8, so a value x is written as
// 32 digits in [-128, 127]: with K = 0x8080...80, byte k of (x + K) xor 0x80,
// read as int8, is digit k of x whenever -K <= x < 2^256 - K (two's-complement
// x; for every field x in [0, p) qualifies since p < 0.498 * 2^256, and for
// BN254 so does the lazy 2 hi - lo in (-p, 2p)). Products of such
// representatives are congruent mod p to the field products, so the sums
// stay exact integers congruent to the reference's field sums.
//
// Operand images. A wave writes the digit images of 32 values per table
// into LDS (one 32-byte row per value) and reads them back with
// ds_read_b64_tr_b8 (gfx950's transposed LDS read), which hands lane i of a
// 16-lane group column i of an 8 x 16-byte block: exactly the MFMA operand
// layout (A[row = digit][k = point], B[k = point][col = digit]); operand
// maps and the transposed read measured on the box (tools/microbench_mfma.hip).
#pragma once
#include <type_traits>
#include "kernels.hpp"

namespace zk {

typedef int i32x2 __attribute__((ext_vector_type(2)));
typedef int i32x4 __attribute__((ext_vector_type(4)));
typedef int i32x16 __attribute__((ext_vector_type(16)));
typedef __attribute__((address_space(3))) i32x2 lds_i32x2;

// digits of x in place: byte k of the result, as int8, is digit k of x
__device__ __forceinline__ void to_digits(Fe& x) {
  uint32_t c = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) x.v[i] = addc32(x.v[i], 0x80808080u, c, &c) ^ 0x80808080u;
}

// 2 hi - lo as a two's-complement 256-bit integer (no reduction; the caller
// keeps |result| < 2^255)
__device__ __forceinline__ Fe lazy2(const Fe& lo, const Fe& hi) {
  Fe r;
  uint32_t c = 0, b = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) r.v[i] = addc32(hi.v[i], hi.v[i], c, &c);
#pragma unroll
  for (int i = 0; i < 8; ++i) r.v[i] = subb32(r.v[i], lo.v[i], b, &b);
  return r;
}
// lazy (-p, 2p) extended points have valid digits: 2p < 2^256 - K
template <class F>
constexpr bool kLazyDigits = (uint64_t)F::P[7] * 2 + 2 < 0x7F7F7F7Full;

// one 32 x 32 x 32 step: acc += digits(A image)^T * digits(B image) over the
// 32 rows (points) of two [32][32]-byte LDS images
__device__ __forceinline__ i32x4 tr_frag(const uint8_t* img) {
  const uint32_t l = threadIdx.x & 63, g = l >> 4, i16 = l & 15;
  const uint32_t q = i16 >> 1, p = i16 & 1;
  // lane 2q+p of 16-lane group g supplies row (16(g>>1) + 8t + q), bytes 16(g&1) + 8p .. +7
  const uint8_t* base = img + (16 * (g >> 1) + q) * 32 + 16 * (g & 1) + 8 * p;
  const i32x2 r0 = __builtin_amdgcn_ds_read_tr8_b64_v2i32((lds_i32x2*)(base));
  const i32x2 r1 = __builtin_amdgcn_ds_read_tr8_b64_v2i32((lds_i32x2*)(base + 8 * 32));
  i32x4 f;
  f[0] = r0[0];
  f[1] = r0[1];
  f[2] = r1[0];
  f[3] = r1[1];
  return f;
}

__device__ __forceinline__ void st_row(uint8_t* row, const Fe& x) {
  uint4* d = reinterpret_cast<uint4*>(row);
  d[0] = make_uint4(x.v[0], x.v[1], x.v[2], x.v[3]);
  d[1] = make_uint4(x.v[4], x.v[5], x.v[6], x.v[7]);
}

// ---------------------------------------------------------------------------
// k_gkr_d0m: rounds 0 and 1 from the input tables in one pass (the step of
// the removed VALU k_gkr_d0r: nine categories, limb-sum output) with the products on
// the matrix cores. Wave w of a block serves product pp = w & 1 (0: A*S,
// 1: M*P) over its own sequence of chunks of 32 quads (waves 0-1 and 2-3
// take alternate chunks), so every input byte is loaded once. Per chunk lane
// l < 32 holds the four corners of X for quad l, lane l >= 32 those of Y;
// the lanes form the nine grid-point values in two phases of at most five
// (the corners and (0,2); then (2,0) (2,1) (1,2) (2,2)), write their digit
// images and run one MFMA per point (K = the 32 quads) into nine int32
// tiles. The next chunk's corners are loaded before this one is processed.
// Epilogue: the tiles' anti-diagonal sums (digit position k + l) per
// category in LDS (int64), then per category the signed integer
//   G = sum_d T_d 2^(8d) + M,  M = p 2^275 > |G| (a multiple of p: G stays
// congruent), normalised to 17 non-negative 32-bit words — the unreduced
// 17-word product sum of the VALU kernels — and grid_finish.
// Bounds: |C| <= 2^19 per chunk, so a wave takes at most kD0MChunksMax
// chunks (int32 tiles); |G| < 2 * 2^16 * 2^510 < M < 2^530 for a block.
// ---------------------------------------------------------------------------
constexpr uint32_t kD0MChunksMax = 2048;  // chunks of 32 quads per wave (int32 tile bound: 1 MFMA per chunk)
static_assert(1ull * (1u << 19) * kD0MChunksMax <= (1ull << 30), "d0m tile bound");
constexpr int kD0MPts = 5;                // point images per phase
struct D0MScratch {
  uint8_t img[4][kD0MPts][2][32][32];   // per wave: point, table (X, Y), 32 rows of 32 bytes
  unsigned long long T[kD0Cats][64];    // anti-diagonal sums per category (int64)
  uint64_t tot[kSlotU64];
  uint64_t pp[kBlock];
  uint32_t am_last;
};

// write the digit images of NP values and accumulate one MFMA per value
template <int NP>
__device__ __forceinline__ void d0m_phase(Fe (&v)[kD0MPts], uint8_t (*img)[2][32][32], i32x16* acc) {
  const uint32_t l = threadIdx.x & 63, half = l >> 5, ql = l & 31;
#pragma unroll
  for (int i = 0; i < NP; ++i) {
    to_digits(v[i]);
    st_row(&img[i][half][ql][0], v[i]);
  }
  asm volatile("" ::: "memory");  // a wave's LDS ops run in order: the reads below see the rows
#pragma unroll
  for (int i = 0; i < NP; ++i) {
    const i32x4 fa = tr_frag(&img[i][0][0][0]), fb = tr_frag(&img[i][1][0][0]);
    acc[i] = __builtin_amdgcn_mfma_i32_32x32x32_i8(fa, fb, acc[i], 0, 0, 0);
  }
  asm volatile("" ::: "memory");  // the next rows are written after these reads
}

template <class F>
__device__ __forceinline__ void d0m_load(const Fe* __restrict__ T, uint64_t Q, uint64_t j, Fe (&c)[4]) {
  if (j < Q) {
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      ZK_DCHECK(j + k * Q < 4 * Q);
      c[k] = ld_fe(T, j + k * Q);
    }
  } else {  // past the end: zero points (every lane stays active for the transposed reads)
#pragma unroll
    for (int k = 0; k < 4; ++k) c[k] = fe_zero<F>();
  }
}

// M = p * 2^275 as 17 words
template <class F>
__device__ __forceinline__ uint32_t d0m_offset_word(int w) {
  // p << 19 occupies words 8..16 (bit 275 = word 8, bit 19)
  if (w < 8) return 0;
  const int i = w - 8;  // word i of p << 19
  const uint32_t lo = i < 8 ? F::P[i] << 19 : 0;
  const uint32_t hi = i >= 1 ? F::P[i - 1] >> 13 : 0;
  return lo | hi;
}

template <class F>
__global__ __launch_bounds__(kBlock, 2) void k_gkr_d0m(const Fe* __restrict__ A, const Fe* __restrict__ S,
                                                      const Fe* __restrict__ M, const Fe* __restrict__ P, uint64_t Q,
                                                      RoundSink sink) {
  if (blockIdx.x == 0) ZK_SINK_STAMP(sink, 0);
  __shared__ D0MScratch sc;
  const uint32_t t = threadIdx.x, w = t >> 6, l = t & 63, pp = w & 1;
  for (uint32_t i = t; i < kD0Cats * 64; i += kBlock) (&sc.T[0][0])[i] = 0;
  // tiles in category order: 0 V00, 1 V22, 2 V01, 3 V02, 4 V10, 5 V20, 6 V21, 7 V12, 8 V11
  i32x16 acc[kD0Cats];
#pragma unroll
  for (int i = 0; i < kD0Cats; ++i)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[i][r] = 0;
  const Fe* __restrict__ T = (l >> 5) ? (pp ? P : S) : (pp ? M : A);
  const uint64_t nch = (Q + 31) / 32, stride = (uint64_t)gridDim.x * 2;
  uint64_t ch = (uint64_t)blockIdx.x * 2 + (w >> 1);
  Fe nx[4];
  d0m_load<F>(T, Q, ch * 32 + (l & 31), nx);
  for (; ch < nch; ch += stride) {
    Fe c[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) c[k] = nx[k];  // corners (0,0) (0,1) (1,0) (1,1)
    if (ch + stride < nch) d0m_load<F>(T, Q, (ch + stride) * 32 + (l & 31), nx);
    Fe v[kD0MPts];
    v[0] = c[0];
    v[1] = c[1];
    v[2] = c[2];
    v[3] = c[3];
    v[4] = kLazyDigits<F> ? lazy2(c[0], c[1]) : at2<F>(c[0], c[1]);  // (0,2)
    {
      i32x16 a5[5] = {acc[0], acc[2], acc[4], acc[8], acc[3]};
      d0m_phase<5>(v, sc.img[w], a5);
      acc[0] = a5[0]; acc[2] = a5[1]; acc[4] = a5[2]; acc[8] = a5[3]; acc[3] = a5[4];
    }
    v[0] = at2<F>(c[0], c[2]);                                          // (2,0), reduced
    v[1] = at2<F>(c[1], c[3]);                                          // (2,1), reduced
    v[2] = kLazyDigits<F> ? lazy2(c[2], c[3]) : at2<F>(c[2], c[3]);      // (1,2)
    v[3] = kLazyDigits<F> ? lazy2(v[0], v[1]) : at2<F>(v[0], v[1]);      // (2,2) from reduced (2,0), (2,1)
    {
      i32x16 a4[4] = {acc[5], acc[6], acc[7], acc[1]};
      d0m_phase<4>(v, sc.img[w], a4);
      acc[5] = a4[0]; acc[6] = a4[1]; acc[7] = a4[2]; acc[1] = a4[3];
    }
  }
  __syncthreads();  // T zeroed
  const uint32_t col = l & 31, h = l >> 5;
#pragma unroll
  for (int i = 0; i < kD0Cats; ++i) {
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const uint32_t row = (r & 3) + 8 * (r >> 2) + 4 * h;
      atomicAdd(&sc.T[i][row + col], (unsigned long long)(long long)acc[i][r]);
    }
  }
  __syncthreads();
  if (t < (uint32_t)kD0Cats) {  // G + M -> 17 words, signed byte-wise carry
    int64_t carry = 0;
    uint32_t word = 0;
    for (int d = 0; d < 68; ++d) {
      const int wd = d >> 2, sh = 8 * (d & 3);
      int64_t s = carry + (d < 63 ? (int64_t)sc.T[t][d] : 0);
      s += (int64_t)((d0m_offset_word<F>(wd) >> sh) & 0xffu);
      word |= (uint32_t)(s & 0xff) << sh;
      carry = s >> 8;
      if ((d & 3) == 3) {
        sc.tot[t * 17 + wd] = word;
        word = 0;
      }
    }
  }
  __syncthreads();
  grid_finish<kD0Limbs>(sc, sink);
}


// ---------------------------------------------------------------------------
// Double steps on the matrix cores: k_gkr_dm (two pending challenges).
//
// The step of k_gkr_dround<F, 2> (kernels.hpp): fold the level-(i-2) tables
// by (ra, rb) at once, write level i, and sum the eight grid-point products
// of rounds i and i+1 over level i's quads. Both halves are contractions:
//
// Fold. Z = x00 + ra d1 + rb d2 + rab d3 (fold2, field.hpp) with
// d1 = x10 - x00, d2 = x01 - x00, d3 = x11 - x01 - d1. With the step
// constants w_c[k] = r_c 2^(8k + 64) mod p (c = ra, rb, rab; k = 0..31) and
// the signed digits delta_{c,k} of d_c,
//   Y = sum_{c,k} delta_{c,k} w_c[k] == (ra d1 + rb d2 + rab d3) 2^64 (mod p),
// and digit position pos of Y is sum_{c,k} w_c[k]_pos delta_{c,k}: an
// MFMA with A = the constants' digits (rows pos, k = (c, k)) and B = the
// differences' digits (k = (c, k), columns = 32 elements), K = 96. Column e
// of the int32 result is element e's 32 position sums (|.| < 2^21), split
// over lanes e and e + 32 (even / odd 32-bit words); the lanes assemble
// signed 64-bit word sums, trade halves with v_permlane32_swap, propagate
// carries, run two 32-bit REDC steps (the 2^64) and add x00: Z fully
// reduced. The 3 x 96 constants' digit rows are built once per block.
//
// Products. As k_gkr_d0m: lane l holds the four folded corners of quad
// j0 + l of its wave's table (wave w: table w = A, S, M, P), forms the
// eight grid-point values (categories of kernels.hpp: 0 V00, 1 V22, 2 V01,
// 3 V02, 4 V10, 5 V20, 6 V21, 7 V12) and writes their digit rows into a
// block image [category][table][64 quads]; after a barrier wave w runs the
// products of pair w & 1 (A*S or M*P) for categories 4 (w >> 1) .. +3, two
// K = 32 MFMAs each. Epilogue and limb sums as k_gkr_d0m (8 categories).
// ---------------------------------------------------------------------------
#define ZK_P2D8(F, b) pow2_mod_p<F>(b), pow2_mod_p<F>(b + 8), pow2_mod_p<F>(b + 16), pow2_mod_p<F>(b + 24)
#define ZK_P2D_INIT(F)                                                                                             \
  {ZK_P2D8(F, 64), ZK_P2D8(F, 96), ZK_P2D8(F, 128), ZK_P2D8(F, 160), ZK_P2D8(F, 192), ZK_P2D8(F, 224),             \
   ZK_P2D8(F, 256), ZK_P2D8(F, 288)}
static __constant__ Fe kP2DBn254Fr[32] = ZK_P2D_INIT(Bn254Fr);
static __constant__ Fe kP2DBn254Fq[32] = ZK_P2D_INIT(Bn254Fq);
static __constant__ Fe kP2DBls12_381Fr[32] = ZK_P2D_INIT(Bls12_381Fr);
template <class F>
__device__ __forceinline__ Fe p2dig(uint32_t k) {  // 2^(8k + 64) mod p
  if constexpr (F::id == BN254_FR) return kP2DBn254Fr[k];
  else if constexpr (F::id == BN254_FQ) return kP2DBn254Fq[k];
  else return kP2DBls12_381Fr[k];
}

// the partner lane's value (lane l <-> l ^ 32; v_permlane32_swap, tools/microbench_mfma.hip)
__device__ __forceinline__ uint32_t xchg32(uint32_t x) {
  const auto r = __builtin_amdgcn_permlane32_swap(x, x, false, false);
  return (threadIdx.x & 32) ? r[0] : r[1];
}
__device__ __forceinline__ Fe sub256(const Fe& a, const Fe& b) {  // two's complement a - b
  Fe r;
  uint32_t bw = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) r.v[i] = subb32(a.v[i], b.v[i], bw, &bw);
  return r;
}
// signed 64-bit sum of four int32 byte-position sums at byte offsets 0, 8, 16, 24
__device__ __forceinline__ int64_t word_of(int a0, int a1, int a2, int a3) {
  return (int64_t)a0 + ((int64_t)a1 << 8) + ((int64_t)a2 << 16) + ((int64_t)a3 << 24);
}
// The two B fragments of a fold MFMA pair straight from one v_permlane32_swap
// per register pair (no selects): with vdst = word q (bytes 4q..) and vsrc =
// word 4 + q of the lane's element, the swapped vdst holds [word q of elements
// 0..31 | word 4 + q of elements 0..31] (acc0's columns), the swapped vsrc
// [word q of elements 32..63 | word 4 + q of elements 32..63] (acc1's).
__device__ __forceinline__ void fold_operands(const Fe& x, i32x4& b0, i32x4& b1) {
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const auto r = __builtin_amdgcn_permlane32_swap(x.v[q], x.v[4 + q], false, false);
    b0[q] = (int)r[0];
    b1[q] = (int)r[1];
  }
}
// Lane-contiguous non-temporal input loads (round 6, ZK_LC_LOADS). A wave's
// 64 lanes load the 1 KiB of 32 consecutive elements e0 .. e0 + 31 as whole
// 128-B lines: lane l takes bytes 16 (l >> 5) .. +15 of element e0 + (l & 31).
// That is a fold MFMA's B operand as it stands ([digits 0-15 of elements
// 0-31 | digits 16-31 of the same], fold_operands), and a digit-image row half
// for the round-sum images. Measured memory-only (tools/microbench_wmix.hip
// pfnt / gldsnt): the element-per-lane shape (two 16-B loads per lane, each
// instruction touching half of every line) streams 2 GiB at 6.3 TB/s with the
// default policy and 5.6 with nt; whole lines per instruction with nt, 7.1 TB/s
// (the first fold pass's read/write mix: 481 -> 445 us).
__device__ __forceinline__ u32x4 ld_half_nt(const Fe* __restrict__ X, uint64_t e0) {
  const uint32_t l = threadIdx.x & 63;
  return __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(X) + 2 * (e0 + (l & 31)) + (l >> 5));
}

// digits (to_digits) of N values held as ld_half_nt halves, in place: every lane
// adds its half of K = 0x8080...80; the carry out of an element's low half
// (lane l < 32) enters its high half (lane l + 32) through one v_permlane32_swap
// for all N; then the xor. Same bytes as to_digits on the whole element.
template <int N>
__device__ __forceinline__ void to_digits_halves(u32x4 (&h)[N]) {
  static_assert(N <= 32, "one carry bit per value in a 32-bit word");
  uint32_t cm = 0;
#pragma unroll
  for (int i = 0; i < N; ++i) {
    uint32_t c = 0;
#pragma unroll
    for (int j = 0; j < 4; ++j) h[i][j] = addc32(h[i][j], 0x80808080u, c, &c);
    cm |= c << i;
  }
  // the low half's carries, in the high half's lane (the swap runs with every lane
  // active: inside the select's branch the low lanes would be masked off)
  const uint32_t pc = xchg32(cm);
  const uint32_t cin = (threadIdx.x & 32) ? pc : 0u;
#pragma unroll
  for (int i = 0; i < N; ++i) {
    uint32_t c = (cin >> i) & 1u;
#pragma unroll
    for (int j = 0; j < 4; ++j) h[i][j] = addc32(h[i][j], 0u, c, &c) ^ 0x80808080u;
  }
}
__device__ __forceinline__ i32x4 as_i32x4(const u32x4& v) {
  i32x4 r;
  r[0] = (int)v[0];
  r[1] = (int)v[1];
  r[2] = (int)v[2];
  r[3] = (int)v[3];
  return r;
}

// The result words after a fold MFMA pair: lane (e, h) holds words 2g + h of
// both columns (acc0: element e, acc1: element 32 + e); one swap per 32-bit
// half gives every lane words 2g and 2g + 1 of its own element.
__device__ __forceinline__ void fold_words(const i32x16& acc0, const i32x16& acc1, int64_t (&W)[8]) {
#pragma unroll
  for (int g = 0; g < 4; ++g) {
    const uint64_t w0 = (uint64_t)word_of(acc0[4 * g], acc0[4 * g + 1], acc0[4 * g + 2], acc0[4 * g + 3]);
    const uint64_t w1 = (uint64_t)word_of(acc1[4 * g], acc1[4 * g + 1], acc1[4 * g + 2], acc1[4 * g + 3]);
    const auto lo = __builtin_amdgcn_permlane32_swap((uint32_t)w0, (uint32_t)w1, false, false);
    const auto hi = __builtin_amdgcn_permlane32_swap((uint32_t)(w0 >> 32), (uint32_t)(w1 >> 32), false, false);
    W[2 * g] = (int64_t)(((uint64_t)hi[0] << 32) | lo[0]);
    W[2 * g + 1] = (int64_t)(((uint64_t)hi[1] << 32) | lo[1]);
  }
}

// Z = x00 + Y 2^-64 (mod p), Y = sum_i W[i] 2^(32 i) (signed words, |Y| < 2^271)
template <class F>
__device__ __forceinline__ Fe dm_finish(const int64_t (&W)[8], const Fe& x00) {
  uint32_t y[8];
  int64_t c = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int64_t v = W[i] + c;
    y[i] = (uint32_t)v;
    c = v >> 32;
  }
  int64_t top = c;  // Y = y + top 2^256
#pragma unroll
  for (int st = 0; st < 2; ++st) {  // REDC by 2^32: (Y + m p) / 2^32, exact
    const uint32_t m = y[0] * F::PINV;
    uint64_t a = (uint64_t)m * F::P[0] + y[0];
    uint32_t cc = (uint32_t)(a >> 32);
#pragma unroll
    for (int j = 1; j < 8; ++j) {
      a = (uint64_t)m * F::P[j] + y[j] + cc;
      y[j - 1] = (uint32_t)a;
      cc = (uint32_t)(a >> 32);
    }
    const int64_t tt = top + cc;
    y[7] = (uint32_t)tt;
    top = tt >> 32;
  }
  // V = y + top 2^256 in (-2^208, p + 2^208); x00 + V + p in (0, 3p + 2^208): two conditional subtractions
  Fe s;
  uint32_t c1 = 0, c2 = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) s.v[i] = addc32(y[i], x00.v[i], c1, &c1);
#pragma unroll
  for (int i = 0; i < 8; ++i) s.v[i] = addc32(s.v[i], F::P[i], c2, &c2);
  int32_t hi = (int32_t)top + (int32_t)c1 + (int32_t)c2;  // 0 or 1
#pragma unroll
  for (int pass = 0; pass < 2; ++pass) {
    Fe t;
    uint32_t b = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const uint32_t q = pass == 0 ? ((F::P[i] << 1) | (i ? F::P[i - 1] >> 31 : 0u)) : F::P[i];
      t.v[i] = subb32(s.v[i], q, b, &b);
    }
    const int32_t th = hi - (int32_t)b;
    const bool take = th >= 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) s.v[i] = take ? t.v[i] : s.v[i];
    hi = take ? th : hi;
  }
  return s;
}

// fold element i of one table (level-(i-2) inputs at i, i + h4, i + 2 h4, i + 3 h4) by
// (ra, rb, rab); every lane folds its own element, wf[c] = the A fragments of the constants
__device__ __forceinline__ void dm_load(const Fe* __restrict__ X, uint64_t i, uint64_t h4, Fe (&x)[4]) {
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    ZK_DCHECK(i + k * h4 < 4 * h4);
    x[k] = ld_fe(X, i + k * h4);  // x00, x01, x10, x11
  }
}
template <class F>
__device__ __forceinline__ Fe dm_fold(const Fe (&x)[4], const i32x4 (&wf)[3]) {
  const Fe &x00 = x[0], &x01 = x[1], &x10 = x[2], &x11 = x[3];
  Fe d[3];
  if constexpr (kLazyDigits<F>) {  // signed differences, |d1|, |d2| < p, |d3| < 2p
    d[0] = sub256(x10, x00);
    d[1] = sub256(x01, x00);
    d[2] = sub256(sub256(x11, x01), d[0]);
  } else {
    d[0] = fe_sub<F>(x10, x00);
    d[1] = fe_sub<F>(x01, x00);
    d[2] = fe_sub<F>(fe_sub<F>(x11, x01), d[0]);
  }
  i32x16 acc0, acc1;  // columns: elements j0 .. j0+31 (acc0), j0+32 .. j0+63 (acc1)
#pragma unroll
  for (int r = 0; r < 16; ++r) acc0[r] = acc1[r] = 0;
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    to_digits(d[c]);
    // B fragment of lane (e, h): digits 16h .. 16h+15 of element e (acc0) / 32 + e (acc1);
    // lane e owns element e, lane e + 32 element 32 + e (fold_operands)
    i32x4 b0, b1;
    fold_operands(d[c], b0, b1);
    acc0 = __builtin_amdgcn_mfma_i32_32x32x32_i8(wf[c], b0, acc0, 0, 0, 0);
    acc1 = __builtin_amdgcn_mfma_i32_32x32x32_i8(wf[c], b1, acc1, 0, 0, 0);
  }
  int64_t W[8];
  fold_words(acc0, acc1, W);
  return dm_finish<F>(W, x00);
}

constexpr uint32_t kDMQuads = 64;        // quads per chunk (one per lane)
constexpr uint32_t kDMChunksMax = 1024;  // chunks per block (int32 product tiles: 2 MFMAs, 2^20 per chunk)
static_assert(2ull * (1u << 19) * kDMChunksMax <= (1ull << 30), "dm tile bound");
struct DMScratch {
  uint8_t img[kDCats][4][kDMQuads][32];  // 64 KB: category, table, quad, digit row
  uint8_t wimg[3][32][32];                // digit rows of the fold constants (c, k)
  unsigned long long T[kDCats][64];
  uint64_t tot[kSlotU64];
  uint64_t pp[kBlock];
  uint32_t am_last;
};

template <class F>
__device__ __forceinline__ void dm_row(uint8_t (&row)[32], Fe x) {
  to_digits(x);
  st_row(row, x);
}

// G + M -> 17 words for category t (threads < ncat), as k_gkr_d0m
template <class F>
__device__ __forceinline__ void diag_to_words(const unsigned long long (&T)[64], uint64_t* out) {
  // word w of G: S_w = sum_{i<4} T[4w+i] 2^(8i) (|T| < 2^37: |S_w| < 2^62), then one
  // signed carry chain over the 17 words (fully unrolled: the LDS reads issue up front)
  int64_t S[17];
#pragma unroll
  for (int w = 0; w < 17; ++w) {
    int64_t v = 0;
#pragma unroll
    for (int i = 0; i < 4; ++i)
      if (4 * w + i < 63) v += (int64_t)T[4 * w + i] * ((int64_t)1 << (8 * i));
    S[w] = v;
  }
  int64_t carry = 0;
#pragma unroll
  for (int w = 0; w < 17; ++w) {
    const int64_t v = S[w] + (int64_t)d0m_offset_word<F>(w) + carry;
    out[w] = (uint32_t)v;
    carry = v >> 32;
  }
}

// The eight grid-point values of the quad whose folded corners z[0..3] this
// lane holds (wave w = table w) -> digit rows; barrier; wave w then runs the
// products of pair w & 1 for categories 4 (w >> 1) .. +3 (two K = 32 MFMAs
// each, K = the 64 quads of the chunk); barrier (the image is reused).
template <class F>
__device__ __forceinline__ void dm_products(const Fe (&z)[4], DMScratch& sc, i32x16 (&acc)[4]) {
  const uint32_t w = threadIdx.x >> 6, l = threadIdx.x & 63, pp = w & 1, cg = w >> 1;
  const Fe v20 = at2<F>(z[0], z[2]), v21 = at2<F>(z[1], z[3]);  // reduced
  dm_row<F>(sc.img[0][w][l], z[0]);
  dm_row<F>(sc.img[2][w][l], z[1]);
  dm_row<F>(sc.img[4][w][l], z[2]);
  dm_row<F>(sc.img[3][w][l], kLazyDigits<F> ? lazy2(z[0], z[1]) : at2<F>(z[0], z[1]));
  dm_row<F>(sc.img[7][w][l], kLazyDigits<F> ? lazy2(z[2], z[3]) : at2<F>(z[2], z[3]));
  dm_row<F>(sc.img[5][w][l], v20);
  dm_row<F>(sc.img[6][w][l], v21);
  dm_row<F>(sc.img[1][w][l], kLazyDigits<F> ? lazy2(v20, v21) : at2<F>(v20, v21));
  __syncthreads();
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const uint32_t cat = 4 * cg + i;
#pragma unroll
    for (int half = 0; half < 2; ++half) {
      const i32x4 fa = tr_frag(&sc.img[cat][2 * pp][32 * half][0]);
      const i32x4 fb = tr_frag(&sc.img[cat][2 * pp + 1][32 * half][0]);
      acc[i] = __builtin_amdgcn_mfma_i32_32x32x32_i8(fa, fb, acc[i], 0, 0, 0);
    }
  }
  __syncthreads();
}
template <class F, int NT>
__device__ __forceinline__ void tiles_to_words(const unsigned long long (&T)[NT][64], uint64_t (&W)[NT][17]);

// tiles -> anti-diagonal sums -> 17 words per category -> grid limb sums
template <class F>
__device__ __forceinline__ void dm_epilogue(const i32x16 (&acc)[4], DMScratch& sc, const RoundSink& sink) {
  const uint32_t t = threadIdx.x;
  const uint32_t l = t & 63, cg = t >> 7, col = l & 31, h = l >> 5;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const uint32_t row = (r & 3) + 8 * (r >> 2) + 4 * h;
      atomicAdd(&sc.T[4 * cg + i][row + col], (unsigned long long)(long long)acc[i][r]);
    }
  }
  __syncthreads();
  tiles_to_words<F, kDCats>(sc.T, *reinterpret_cast<uint64_t(*)[kDCats][17]>(sc.tot));
  __syncthreads();
  grid_finish<kDLimbs>(sc, sink);
}

template <class F>
__global__ __launch_bounds__(kBlock, 2) void k_gkr_dm(const Fe* __restrict__ A, const Fe* __restrict__ S,
                                                     const Fe* __restrict__ M, const Fe* __restrict__ P,
                                                     Fe* __restrict__ A2, Fe* __restrict__ S2, Fe* __restrict__ M2,
                                                     Fe* __restrict__ P2, uint64_t Q, DIn din, RoundSink sink) {
  Fe ra, rb, rab;
  if (blockIdx.x == 0) ZK_SINK_STAMP(sink, 0);
  block_get_rs(din, ra, rb, rab, gridDim.x > 1);
  if (blockIdx.x == 0) ZK_SINK_STAMP(sink, 1);
  __shared__ DMScratch sc;
  const uint32_t t = threadIdx.x, w = t >> 6, l = t & 63;
  if (t < 96) {
    const uint32_t c = t >> 5, k = t & 31;
    dm_row<F>(sc.wimg[c][k], fe_mul<F>(c == 0 ? ra : (c == 1 ? rb : rab), p2dig<F>(k)));
  }
  for (uint32_t i = t; i < kDCats * 64; i += kBlock) (&sc.T[0][0])[i] = 0;
  __syncthreads();
  i32x4 wf[3];
#pragma unroll
  for (int c = 0; c < 3; ++c) wf[c] = tr_frag(&sc.wimg[c][0][0]);
  const Fe* __restrict__ X = w == 0 ? A : (w == 1 ? S : (w == 2 ? M : P));
  Fe* __restrict__ X2 = w == 0 ? A2 : (w == 1 ? S2 : (w == 2 ? M2 : P2));
  i32x16 acc[4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[i][r] = 0;
  const uint64_t nch = Q / kDMQuads, h4 = 4 * Q;
  Fe in[4];  // inputs of the next fold, loaded one fold ahead
  if ((uint64_t)blockIdx.x < nch) dm_load(X, (uint64_t)blockIdx.x * kDMQuads + l, h4, in);
  for (uint64_t ch = blockIdx.x; ch < nch; ch += gridDim.x) {
    const uint64_t j = ch * kDMQuads + l;
    Fe z[4];  // corners V(a, b) = Z[j + (2a + b) Q]
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      Fe cur[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) cur[q] = in[q];
      if (k < 3)
        dm_load(X, j + (k + 1) * Q, h4, in);
      else if (ch + gridDim.x < nch)
        dm_load(X, (ch + gridDim.x) * kDMQuads + l, h4, in);
      z[k] = dm_fold<F>(cur, wf);
      ZK_DCHECK(j + k * Q < 4 * Q);
      st_fold(X2, j + k * Q, z[k]);
    }
    dm_products<F>(z, sc, acc);
  }
  if (blockIdx.x == 0) ZK_SINK_STAMP(sink, 3);  // block 0 leaves its main loop
  ZK_BLOCK_STAMP(sink, 0);
  dm_epilogue<F>(acc, sc, sink);
}


// ---------------------------------------------------------------------------
// Rounds 0, 1 and 2 in one pass over the inputs (k_gkr_d0t, even schedules
// start here: the first fold pass then writes 1/8 of the tables instead of
// 1/4). An octant j < O holds the corners X_u = X[j + u O], u = 4a + 2b + c
// (a = variable 0, the MSB). Along one variable X(t) Y(t) = (1-t)^2 X0 Y0 +
// t(1-t) (X0 Y1 + X1 Y0) + t^2 X1 Y1, so the three rounds need, per axis, the
// three "moments" 0 (X0 Y0), 1 (X1 Y1), s (X0 Y1 + X1 Y0): 27 moment tiles
// T(alpha, beta, gamma) = sum_j sum of the 2^(#s) corner products X_u Y_v
// they stand for — 64 corner-pair products per octant and product, all on
// corner digits (no extended points, no VALU arithmetic beyond the digits).
// The host (three_rounds) evaluates any grid point from the tiles with the
// weights (1-t)^2, t^2, t(1-t). Block b serves product b & 1 (A*S or M*P);
// per chunk of 32 octants wave w loads corners 2w and 2w+1 of both tables
// (lanes 0-31 X, 32-63 Y) and writes their digit rows into a double-buffered
// image [corner][table][32][32]; after one barrier wave w = 2 aX + aY runs the
// 16 products X_u Y_v with u in aX's half (variable 0 = aX) and v in aY's:
// their tiles share the variable-0 moment (aX == aY ? aX : s), so a wave
// holds 9 tiles (b, c moments) and reads 8 fragments per chunk. The two s
// waves add into the same tiles. Output: per tile the block's sum + p 2^275
// as 17 words,
// reduced mod p in the block (3 Montgomery multiplies): 27 x 8 limb sums.
// ---------------------------------------------------------------------------
constexpr int kD0TCats = 27;
constexpr int kD0TLimbs = kD0TCats * 9;  // 243 limb sums (9 words per category, congruent mod p)
// chunks per block: the busiest tile slot of a wave takes 4 of its 16 MFMAs
// per chunk (4 x 2^19 = 2^21), so 512 chunks keep |slot| <= 2^30
constexpr uint32_t kD0TChunksMax = 512;
static_assert(4ull * (1u << 19) * kD0TChunksMax <= (1ull << 30), "d0t tile bound");
// moment digit of one axis: corners (x, y) -> 0, 1 or 2 (= s)
__host__ __device__ constexpr int moment_digit(int x, int y) { return x == y ? x : 2; }

// A block's 17-word sum x (non-negative, normalised) -> 9 limb sums of a value
// congruent to it mod p: words 0..7 plus sum_{w >= 8} x_w (2^(32 w) mod p),
// each 32 x 32-bit product split over two columns (column sums < 2^37). The
// host's hlimbs_to_fe takes any limb sums; 27 x 9 = 243 fit one slot.
#define ZK_P2W_INIT(F)                                                                                          \
  {pow2_mod_p<F>(256), pow2_mod_p<F>(288), pow2_mod_p<F>(320), pow2_mod_p<F>(352), pow2_mod_p<F>(384),             \
   pow2_mod_p<F>(416), pow2_mod_p<F>(448), pow2_mod_p<F>(480), pow2_mod_p<F>(512)}
static __constant__ Fe kP2WBn254Fr[9] = ZK_P2W_INIT(Bn254Fr);
static __constant__ Fe kP2WBn254Fq[9] = ZK_P2W_INIT(Bn254Fq);
static __constant__ Fe kP2WBls12_381Fr[9] = ZK_P2W_INIT(Bls12_381Fr);
template <class F>
__device__ __forceinline__ Fe p2w(uint32_t k) {  // 2^(32 (8 + k)) mod p
  if constexpr (F::id == BN254_FR) return kP2WBn254Fr[k];
  else if constexpr (F::id == BN254_FQ) return kP2WBn254Fq[k];
  else return kP2WBls12_381Fr[k];
}
template <class F>
__device__ __forceinline__ uint32_t p2w_word(uint32_t k, uint32_t j) {  // word j of 2^(32 (8 + k)) mod p (dynamic j)
  if constexpr (F::id == BN254_FR) return kP2WBn254Fr[k].v[j];
  else if constexpr (F::id == BN254_FQ) return kP2WBn254Fq[k].v[j];
  else return kP2WBls12_381Fr[k].v[j];
}
template <class F>
__device__ __forceinline__ void words17_to_limbs9(const uint64_t* x, uint64_t* out) {
  uint64_t col[9];
#pragma unroll
  for (int j = 0; j < 8; ++j) col[j] = x[j];
  col[8] = 0;
#pragma unroll
  for (int w = 8; w < 17; ++w) {
    const Fe k = p2w<F>(w - 8);
    const uint32_t xw = (uint32_t)x[w];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const uint64_t pr = (uint64_t)xw * k.v[j];
      col[j] += (uint32_t)pr;
      col[j + 1] += pr >> 32;
    }
  }
#pragma unroll
  for (int j = 0; j < 9; ++j) out[j] = col[j];
}

// Block-parallel epilogue of NT tiles (the per-tile serial chains of
// diag_to_words / words17_to_limbs9 took ~1.5 us each on one wave):
// (tile, word) items build S_w, NT threads run the 17-step carries in place,
// (tile, limb) items fold the high words (2 products per high word each).
template <class F, int NT>
__device__ __forceinline__ void tiles_to_words(const unsigned long long (&T)[NT][64], uint64_t (&W)[NT][17]) {
  for (uint32_t it = threadIdx.x; it < (uint32_t)NT * 17; it += kBlock) {
    const uint32_t tile = it / 17, w = it % 17;
    int64_t v = 0;
#pragma unroll
    for (uint32_t i = 0; i < 4; ++i)
      if (4 * w + i < 63) v += (int64_t)T[tile][4 * w + i] * ((int64_t)1 << (8 * i));
    W[tile][w] = (uint64_t)v;
  }
  __syncthreads();
  if (threadIdx.x < (uint32_t)NT) {
    int64_t carry = 0;
#pragma unroll
    for (int w = 0; w < 17; ++w) {
      const int64_t v = (int64_t)W[threadIdx.x][w] + (int64_t)d0m_offset_word<F>(w) + carry;
      W[threadIdx.x][w] = (uint32_t)v;
      carry = v >> 32;
    }
  }
  __syncthreads();
}
template <class F>
__device__ __forceinline__ void stage_p2w(uint32_t (&K)[9][8]) {  // threads < 72; read after a barrier
  if (threadIdx.x < 72) K[threadIdx.x >> 3][threadIdx.x & 7] = p2w_word<F>(threadIdx.x >> 3, threadIdx.x & 7);
}
template <class F, int NT>
__device__ __forceinline__ void words_to_limbs9(const uint64_t (&W)[NT][17], const uint32_t (&K)[9][8], uint64_t* tot) {
  for (uint32_t it = threadIdx.x; it < (uint32_t)NT * 9; it += kBlock) {
    const uint32_t tile = it / 9, j = it % 9;
    uint64_t col = j < 8 ? W[tile][j] : 0;
#pragma unroll
    for (int w = 8; w < 17; ++w) {
      const uint32_t xw = (uint32_t)W[tile][w];
      if (j < 8) col += (uint32_t)((uint64_t)xw * K[w - 8][j]);
      if (j > 0) col += ((uint64_t)xw * K[w - 8][j - 1]) >> 32;
    }
    tot[it] = col;
  }
}

struct D0TScratch {
  uint8_t img[2][8][2][32][32];  // buffer, corner, table (X, Y), octant, digit row (32 KiB)
  unsigned long long T[kD0TCats][64];
  uint64_t w17[kD0TCats][17];
  uint64_t tot[kSlotU64];
  uint64_t pp[kBlock];
  uint32_t am_last;
  uint32_t p2w[9][8];  // 2^(32 (8 + k)) mod p, staged at kernel start for words_to_limbs9
};

// wave w = 2 aX + aY: products X_u Y_v, u = 4 aX + ux, v = 4 aY + vy; tile slot 3 d_b + d_c
__device__ __forceinline__ void d0t_mfmas(const uint8_t (*img)[2][32][32], i32x16 (&acc)[9]) {
  const uint32_t w = threadIdx.x >> 6, aX = w >> 1, aY = w & 1;
  i32x4 fa[4], fb[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    fa[k] = tr_frag(&img[4 * aX + k][0][0][0]);
    fb[k] = tr_frag(&img[4 * aY + k][1][0][0]);
  }
#pragma unroll
  for (int ux = 0; ux < 4; ++ux)
#pragma unroll
    for (int vy = 0; vy < 4; ++vy) {
      const int slot = 3 * moment_digit(ux >> 1, vy >> 1) + moment_digit(ux & 1, vy & 1);
      acc[slot] = __builtin_amdgcn_mfma_i32_32x32x32_i8(fa[ux], fb[vy], acc[slot], 0, 0, 0);
    }
}
__device__ __forceinline__ void d0t_flush(const i32x16 (&acc)[9], unsigned long long (&T)[kD0TCats][64]) {
  const uint32_t w = threadIdx.x >> 6, l = threadIdx.x & 63, col = l & 31, h = l >> 5;
  const uint32_t da = (uint32_t)moment_digit((int)(w >> 1), (int)(w & 1));
#pragma unroll
  for (int i = 0; i < 9; ++i) {
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const uint32_t row = (r & 3) + 8 * (r >> 2) + 4 * h;
      atomicAdd(&T[9 * da + i][row + col], (unsigned long long)(long long)acc[i][r]);
    }
  }
}

// order 2: the groups themselves in the order t33_group_perm, so that the
// first k_gkr_t33 (reverse order) writes its LAST outputs as whole input sets
// of the second k_gkr_t33's first chunks (64-octant both; ZK_MALL_ORDER=2)
__device__ __forceinline__ uint64_t t33_group_perm(uint64_t j, uint64_t n3) {  // n3 = first-t33 chunks (8 | n3)
  return (j >> 3) + (n3 >> 3) * (j & 7);
}
// order 1 (host.hpp, ZK_MALL_ORDER): logical chunk q is physical chunk
// 2 g + (r & 1) + (r >> 1) nch / 8 with g = q / 16, r = q % 16 — the 16 chunks
// of group g are exactly the inputs of the next step's (64-octant k_gkr_t33)
// chunk g, so the pass's LAST reads are whole t33 chunks, which the next step
// (order 1: chunks in reverse) reads FIRST, while the 256 MB Infinity Cache may
// still hold them. Any order gives the same sums (exact integer tiles).
// LC (ZK_LC_LOADS): the corners load as whole lines with the non-temporal
// policy (ld_half_nt: lane l holds half l >> 5 of octant l & 31's corner, for
// both tables), ZK_D0T_AHEAD chunks ahead (2 measured 1.001-1.021 against
// 0.993-1.009 ms per proof for 1, profiles/r6_d0t_ahead_ab.txt), and each lane
// writes its half digit row.
// (Measured and removed: the last 1/8 of the chunks read with the default
// policy, so the Infinity Cache would keep them for the first k_gkr_t33 —
// profiles/r6_lc_mall_tail_ab.txt.)
#ifndef ZK_D0T_AHEAD
#define ZK_D0T_AHEAD 1
#endif
template <class F, bool LC = false>
__global__ __launch_bounds__(kBlock, 2) void k_gkr_d0t(const Fe* __restrict__ A, const Fe* __restrict__ S,
                                                      const Fe* __restrict__ M, const Fe* __restrict__ P, uint64_t O,
                                                      uint32_t order, RoundSink sink) {
  if (blockIdx.x == 0) ZK_SINK_STAMP(sink, 0);
  __shared__ D0TScratch sc;
  const uint32_t t = threadIdx.x, w = t >> 6, l = t & 63, half = l >> 5, ql = l & 31;
  for (uint32_t i = t; i < kD0TCats * 64; i += kBlock) (&sc.T[0][0])[i] = 0;
  stage_p2w<F>(sc.p2w);
  i32x16 acc[9];
#pragma unroll
  for (int i = 0; i < 9; ++i)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[i][r] = 0;
  const uint32_t pp = blockIdx.x & 1;
  const Fe* __restrict__ T = half ? (pp ? P : S) : (pp ? M : A);
  const uint64_t nch = O / 32, nb = gridDim.x >> 1;
  auto phys = [&](uint64_t q) -> uint64_t {
    if (!order) return q;
    uint64_t g = q >> 4;
    const uint64_t r = q & 15;
    if (order == 2) g = t33_group_perm(g, nch >> 4);
    return 2 * g + (r & 1) + (r >> 1) * (nch >> 3);
  };
  uint64_t ch = blockIdx.x >> 1;
  Fe cn[2];
  // (LC) hn[a][i]: corner 2w + (i >> 1) of table i & 1 (X, Y), this lane's half, a chunks ahead
  u32x4 hn[ZK_D0T_AHEAD][4];
  const Fe* __restrict__ TX = pp ? M : A;
  const Fe* __restrict__ TY = pp ? P : S;
  auto load_lc = [&](uint64_t q, u32x4 (&h)[4]) {  // logical chunk q (past the end: chunk 0, every block the same lines)
    const uint64_t pc = phys(q < nch ? q : 0);
    ZK_DCHECK(pc * 32 + 31 + (2 * w + 1) * O < 8 * O);
#pragma unroll
    for (int i = 0; i < 4; ++i) h[i] = ld_half_nt((i & 1) ? TY : TX, pc * 32 + (2 * w + (i >> 1)) * O);
  };
  auto load = [&](uint64_t q) {  // logical chunk q
    const uint64_t pc = phys(q);
    ZK_DCHECK(pc * 32 + 31 + (2 * w + 1) * O < 8 * O);
    cn[0] = ld_fe(T, pc * 32 + ql + (2 * w) * O);
    cn[1] = ld_fe(T, pc * 32 + ql + (2 * w + 1) * O);
  };
  if (ch < nch) {
    if constexpr (LC) {
#pragma unroll
      for (int a = 0; a < ZK_D0T_AHEAD; ++a) load_lc(ch + a * nb, hn[a]);
    } else {
      load(ch);
    }
  }
  uint32_t buf = 0;
  for (; ch < nch; ch += nb, buf ^= 1) {
    if constexpr (LC) {
      to_digits_halves<4>(hn[0]);
#pragma unroll
      for (int i = 0; i < 4; ++i)
        *reinterpret_cast<u32x4*>(&sc.img[buf][2 * w + (i >> 1)][i & 1][ql][16 * half]) = hn[0][i];
#pragma unroll
      for (int a = 0; a + 1 < ZK_D0T_AHEAD; ++a)
#pragma unroll
        for (int i = 0; i < 4; ++i) hn[a][i] = hn[a + 1][i];
      load_lc(ch + ZK_D0T_AHEAD * nb, hn[ZK_D0T_AHEAD - 1]);  // in flight during this chunk's products
    } else {
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        to_digits(cn[i]);
        st_row(&sc.img[buf][2 * w + i][half][ql][0], cn[i]);
      }
      if (ch + nb < nch) load(ch + nb);  // the next chunk's corners, in flight during this chunk's products
    }
    __syncthreads();  // the image of this chunk is complete (double buffering: one barrier per chunk)
    d0t_mfmas(sc.img[buf], acc);
  }
  if (blockIdx.x == 0) ZK_SINK_STAMP(sink, 3);  // block 0 leaves its main loop
  ZK_BLOCK_STAMP(sink, 0);
  __syncthreads();
  d0t_flush(acc, sc.T);
  __syncthreads();
  tiles_to_words<F, kD0TCats>(sc.T, sc.w17);
  words_to_limbs9<F, kD0TCats>(sc.w17, sc.p2w, sc.tot);
  __syncthreads();
  grid_finish<kD0TLimbs>(sc, sink);
}


// ---------------------------------------------------------------------------
// k_gkr_dm3: the double step after k_gkr_d0t — THREE pending challenges
// (ra, rb, rc) = (r_{i-3}, r_{i-2}, r_{i-1}). The level-(i-3) tables fold to
// level i in one pass by the multilinear extension's own weights:
//   Z[e] = sum_c eq((ra, rb, rc), c) X[e + c 4Q],  c = 4a + 2b + c0 (a: ra's variable),
// (partial_evaluate three times, multilinear_polynomial_evaluation.rs:52-63), as ONE
// K = 256 MFMA product per 32 elements: A = digits of w_c[k] = eq(r, c)
// 2^(8k + 64) mod p, B = the inputs' own digits (every input is < p: no
// differences, no lazy ranges). Then the eight grid-point products of
// rounds i, i+1 over level i's quads, exactly as k_gkr_dm.
// ---------------------------------------------------------------------------
struct DM3Scratch : DMScratch {
  Fe eqw[8];
};
// 8 inputs of a fold (weights wf[0..7]) into its two MFMA accumulators
__device__ __forceinline__ void fold_acc8(Fe (&x)[8], const i32x4* wf, i32x16& acc0, i32x16& acc1) {
#pragma unroll
  for (int c = 0; c < 8; ++c) {
    to_digits(x[c]);
    i32x4 b0, b1;
    fold_operands(x[c], b0, b1);
    acc0 = __builtin_amdgcn_mfma_i32_32x32x32_i8(wf[c], b0, acc0, 0, 0, 0);
    acc1 = __builtin_amdgcn_mfma_i32_32x32x32_i8(wf[c], b1, acc1, 0, 0, 0);
  }
}
template <class F, int NP = 3>
__device__ __forceinline__ Fe dm3_fold(Fe (&x)[1 << NP], const i32x4 (&wf)[1 << NP]) {
  i32x16 acc0, acc1;
#pragma unroll
  for (int r = 0; r < 16; ++r) acc0[r] = acc1[r] = 0;
#pragma unroll
  for (int c = 0; c < (1 << NP); ++c) {
    to_digits(x[c]);
    i32x4 b0, b1;
    fold_operands(x[c], b0, b1);
    acc0 = __builtin_amdgcn_mfma_i32_32x32x32_i8(wf[c], b0, acc0, 0, 0, 0);
    acc1 = __builtin_amdgcn_mfma_i32_32x32x32_i8(wf[c], b1, acc1, 0, 0, 0);
  }
  int64_t W[8];
  fold_words(acc0, acc1, W);
  return dm_finish<F>(W, fe_zero<F>());
}

template <class F>
__global__ __launch_bounds__(kBlock, 2) void k_gkr_dm3(const Fe* __restrict__ A, const Fe* __restrict__ S,
                                                      const Fe* __restrict__ M, const Fe* __restrict__ P,
                                                      Fe* __restrict__ A2, Fe* __restrict__ S2, Fe* __restrict__ M2,
                                                      Fe* __restrict__ P2, uint64_t Q, DIn din, RoundSink sink) {
  if (blockIdx.x == 0) ZK_SINK_STAMP(sink, 0);
  __shared__ DM3Scratch sc;
  block_get_eq8<F>(din, sc.eqw, gridDim.x > 1);  // eq((ra, rb, rc), c), c = 4a + 2b + c0
  if (blockIdx.x == 0) ZK_SINK_STAMP(sink, 1);
  const uint32_t t = threadIdx.x, w = t >> 6, l = t & 63;
  for (uint32_t i = t; i < kDCats * 64; i += kBlock) (&sc.T[0][0])[i] = 0;
  __syncthreads();
  // the constants' digit rows borrow the product image until their fragments are in registers
  uint8_t(*wimg)[32][32] = reinterpret_cast<uint8_t(*)[32][32]>(&sc.img[0][0][0][0]);
  dm_row<F>(wimg[t >> 5][t & 31], fe_mul<F>(sc.eqw[t >> 5], p2dig<F>(t & 31)));
  __syncthreads();
  i32x4 wf[8];
#pragma unroll
  for (int c = 0; c < 8; ++c) wf[c] = tr_frag(&wimg[c][0][0]);
  __syncthreads();
  const Fe* __restrict__ X = w == 0 ? A : (w == 1 ? S : (w == 2 ? M : P));
  Fe* __restrict__ X2 = w == 0 ? A2 : (w == 1 ? S2 : (w == 2 ? M2 : P2));
  i32x16 acc[4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[i][r] = 0;
  const uint64_t nch = Q / kDMQuads, h4 = 4 * Q;
  for (uint64_t ch = blockIdx.x; ch < nch; ch += gridDim.x) {
    const uint64_t j = ch * kDMQuads + l;
    Fe z[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      Fe x[8];
#pragma unroll
      for (int c = 0; c < 8; ++c) {
        ZK_DCHECK(j + k * Q + c * h4 < 8 * h4);
        x[c] = ld_fe(X, j + k * Q + c * h4);
      }
      z[k] = dm3_fold<F>(x, wf);
      ZK_DCHECK(j + k * Q < 4 * Q);
      st_fold(X2, j + k * Q, z[k]);
    }
    dm_products<F>(z, sc, acc);
  }
  if (blockIdx.x == 0) ZK_SINK_STAMP(sink, 3);  // block 0 leaves its main loop
  ZK_BLOCK_STAMP(sink, 0);
  dm_epilogue<F>(acc, sc, sink);
}


// ---------------------------------------------------------------------------
// k_gkr_t33: the step after k_gkr_d0t on even schedules — fold the inputs
// (level i-3) by the three pending challenges to level i (k_gkr_dm3's K = 256
// eq-weight MFMA) and sum rounds i, i+1, i+2 over level i's octants as 27
// moment tiles (k_gkr_d0t's products, both pairs into the same tiles). Per
// chunk of 32 octants wave w folds table w's 256 outputs in four 64-lane
// calls (lane l: octant l & 31, corner 2f + (l >> 5)) and writes their digit
// rows into a double-buffered image [corner][table][32][32]; after one
// barrier wave w = 2 aX + aY runs 2 x 16 products into its 9 tiles. One
// wave per SIMD (the tiles, the eight weight fragments and a fold's inputs
// in flight: ~370 registers); the next fold's inputs are loaded before the
// current one is reduced.
// ---------------------------------------------------------------------------
// Chunk of k_gkr_t33 (template OCT): 64 octants, one per lane, eight folds (one
// per corner: each input a contiguous 2 KiB per wave, 4-6 % faster as a memory
// pattern than 32 octants x two corners, and 476 vs 499 us for the first
// triple step) and a single-buffered image — for large levels; 32 octants, two
// corners per fold and a double-buffered image — twice the blocks for small ones.
// int32 tile bound: an MFMA adds at most 32 x 128^2 = 2^19 in magnitude to a
// slot, and the busiest slot (moment s on both b and c: 4 of a wave's 16
// corner-pair products) takes 4 MFMAs per (product, K half): 16 per chunk of
// 64 octants, 8 per chunk of 32. A block's chunk count stays <= kT33ChunksMax
// (the host sizes the grid so, step_grid), so |slot| <= 2^30 (the
// previous 256 / 512 reached exactly 2^31).
template <int OCT>
constexpr uint32_t kT33SlotMfmas = OCT == 64 ? 16 : 8;
template <int OCT>
constexpr uint32_t kT33ChunksMax = OCT == 64 ? 128 : 256;
static_assert((uint64_t)kT33SlotMfmas<64> * (1u << 19) * kT33ChunksMax<64> <= (1ull << 30), "t33 tile bound");
static_assert((uint64_t)kT33SlotMfmas<32> * (1u << 19) * kT33ChunksMax<32> <= (1ull << 30), "t33 tile bound");
struct T33Scratch {
  uint8_t img[2][8][4][32][32];  // [buffer][corner][table][octant][digit row] (OCT 32), or [corner][table][64][32] (OCT 64)
  unsigned long long T[kD0TCats][64];
  uint64_t w17[kD0TCats][17];
  uint64_t tot[kSlotU64];
  uint64_t pp[kBlock];
  uint32_t am_last;
  uint32_t p2w[9][8];  // 2^(32 (8 + k)) mod p, staged at kernel start for words_to_limbs9
  Fe eqw[8];
};

// PIPE (OCT 64, ZK_T33_PIPE): a double-buffered image and ONE barrier per
// chunk; the previous chunk's 64 product MFMAs run in four groups of 16 after
// folds 1, 3, 5 and 7 of the current chunk (while its loads are in flight)
// instead of after a second barrier
struct T33ScratchP {
  uint8_t img[2][8][4][64][32];  // [buffer][corner][table][octant][digit row]
  unsigned long long T[kD0TCats][64];
  uint64_t w17[kD0TCats][17];
  uint64_t tot[kSlotU64];
  uint64_t pp[kBlock];
  uint32_t am_last;
  uint32_t p2w[9][8];
  Fe eqw[8];
};

// LC (ZK_LC_LOADS, the pipelined 64-octant loop): a fold's eight inputs load
// as whole lines with the non-temporal policy straight into the fold MFMAs' B
// operands (ld_half_nt: elements ch 64 + u O + [0, 32) and + [32, 64) of each
// input; to_digits_halves) instead of one element per lane (fold_operands).
template <class F, int OCT, bool PIPE = false, bool LC = false>
__global__ __launch_bounds__(kBlock, 1) void k_gkr_t33(const Fe* __restrict__ A, const Fe* __restrict__ S,
                                                      const Fe* __restrict__ M, const Fe* __restrict__ P,
                                                      Fe* __restrict__ A2, Fe* __restrict__ S2, Fe* __restrict__ M2,
                                                      Fe* __restrict__ P2, uint64_t O, uint32_t order, DIn din,
                                                      RoundSink sink) {
  constexpr int NI = 8;  // inputs per output
  if (blockIdx.x == 0) ZK_SINK_STAMP(sink, 0);
  const uint32_t t = threadIdx.x, w = t >> 6, l = t & 63, ql = l & 31, hh = l >> 5;
  const Fe* __restrict__ X = uniform_ptr(w == 0 ? A : (w == 1 ? S : (w == 2 ? M : P)));
  Fe* __restrict__ X2 = w == 0 ? A2 : (w == 1 ? S2 : (w == 2 ? M2 : P2));
  const uint64_t nch = O / OCT, h8 = 8 * O;  // level-i tables hold 8 O elements
  // order 1 (ZK_MALL_ORDER, the pass after an order-1 k_gkr_d0t): logical chunk
  // ch is physical chunk nch - 1 - ch — the chunks the previous pass read last
  // first; order 2: through t33_group_perm as the order-2 input pass
  auto pch = [&](uint64_t ch) -> uint64_t {
    if (!order) return ch;
    return order == 2 ? t33_group_perm(nch - 1 - ch, nch) : nch - 1 - ch;
  };
  // A fold of a chunk past the block's last one (the prefetch two folds
  // ahead) loads chunk 0 instead: the load stays unconditional (a conditional
  // load made hipcc drain every load at each chunk boundary) and every block's
  // stray loads hit the same L2-resident lines (loading the block's own chunk
  // again reached HBM: 1.13 x the algorithmic bytes at two chunks per block).
  // (Measured and dropped: the same through bounds-checked buffer loads, which
  // read zeros without an access — the 8 descriptors cost the kernel 16 VGPR
  // spills and 11 SGPR spills, 512 vs 470 us for the first launch.)
  // OCT 32: fold f = corners 2f (lanes 0-31) and 2f + 1 (lanes 32-63) of octants ch*32 + ql
  auto in_at = [&](uint64_t ch, int f, Fe (&x)[NI]) {
    ch = pch(ch < nch ? ch : 0);
    const uint64_t e = ch * 32 + ql + (uint64_t)(2 * f + hh) * O;
#pragma unroll
    for (int k = 0; k < NI; ++k) {
      ZK_DCHECK(e + k * h8 < 8 * h8);
      x[k] = ld_fe(X, e + k * h8);
    }
  };
  // Inputs two folds ahead for OCT 64, one for OCT 32 (one wave per SIMD: the
  // loads in flight are what hides HBM latency). The first ones (written by
  // the previous kernel) are in flight while the host posts the challenges.
  // Block 0's wave 0 polls the host for the challenges and relays them to
  // every block: its poll would wait behind these loads (vmcnt is in order),
  // so it loads after the challenges arrive.
  auto unit_at = [&](uint64_t ch, int u, Fe (&x)[8]) {  // OCT 64: the eight inputs of fold u (corner u of octants ch*64 + l)
    ch = pch(ch < nch ? ch : 0);
    const uint64_t e = ch * 64 + l + (uint64_t)u * O;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      ZK_DCHECK(e + k * h8 < 8 * h8);
      x[k] = ld_fe(X, e + k * h8);
    }
  };
  // (LC) the halves of fold u's inputs: [k] elements ch 64 + u O + k 8 O + [0, 32), [8 + k] + [32, 64)
  auto unit_lc = [&](uint64_t ch, int u, u32x4 (&h)[16]) {
    ch = pch(ch < nch ? ch : 0);
    const uint64_t e0 = ch * 64 + (uint64_t)u * O;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      ZK_DCHECK(e0 + 63 + k * h8 < 8 * h8);
      h[k] = ld_half_nt(X, e0 + k * h8);
      h[8 + k] = ld_half_nt(X, e0 + 32 + k * h8);
    }
  };
  static_assert(!LC || (PIPE && OCT == 64), "lane-contiguous loads: the pipelined 64-octant loop");
  Fe nx[8], nx2[8];
  u32x4 ux[16], ux2[16];
  const bool early = (uint64_t)blockIdx.x < nch && (blockIdx.x != 0 || w != 0);
  auto first_loads = [&]() {
    if constexpr (LC) {
      unit_lc(blockIdx.x, 0, ux);
      unit_lc(blockIdx.x, 1, ux2);
    } else if constexpr (OCT == 64) {
      unit_at(blockIdx.x, 0, nx);
      unit_at(blockIdx.x, 1, nx2);
    } else {
      in_at(blockIdx.x, 0, nx);
    }
  };
  if (early) first_loads();
  static_assert(!PIPE || OCT == 64, "the pipelined loop is the 64-octant one");
  using Scratch = std::conditional_t<PIPE, T33ScratchP, T33Scratch>;
  __shared__ Scratch sc;
  block_get_eq8<F>(din, sc.eqw, gridDim.x > 1);  // eq(r, c), the oldest pending challenge on c's top bit
  if (!early && (uint64_t)blockIdx.x < nch) first_loads();
  if (blockIdx.x == 0) ZK_SINK_STAMP(sink, 1);
  for (uint32_t i = t; i < kD0TCats * 64; i += kBlock) (&sc.T[0][0])[i] = 0;
  stage_p2w<F>(sc.p2w);
  __syncthreads();
  uint8_t(*wimg)[32][32] = reinterpret_cast<uint8_t(*)[32][32]>(&sc.img[0][0][0][0][0]);
  for (uint32_t q = t; q < 32u * NI; q += kBlock) dm_row<F>(wimg[q >> 5][q & 31], fe_mul<F>(sc.eqw[q >> 5], p2dig<F>(q & 31)));
  __syncthreads();
  i32x4 wf[NI];
#pragma unroll
  for (int c = 0; c < NI; ++c) wf[c] = tr_frag(&wimg[c][0][0]);
  __syncthreads();
  i32x16 acc[9];
#pragma unroll
  for (int i = 0; i < 9; ++i)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[i][r] = 0;
  if constexpr (OCT == 64 && PIPE) {
  uint8_t(*img2)[8][4][64][32] = reinterpret_cast<uint8_t(*)[8][4][64][32]>(&sc.img[0][0][0][0][0]);
  const uint32_t aX = w >> 1, aY = w & 1;
  auto products = [&](uint32_t b, int grp) {  // group grp = (pp, K half) of a chunk's products from image b
    const int pp = grp >> 1, half = grp & 1;
    i32x4 fa[4], fb[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      fa[k] = tr_frag(&img2[b][4 * aX + k][2 * pp][32 * half][0]);
      fb[k] = tr_frag(&img2[b][4 * aY + k][2 * pp + 1][32 * half][0]);
    }
#pragma unroll
    for (int ux = 0; ux < 4; ++ux)
#pragma unroll
      for (int vy = 0; vy < 4; ++vy) {
        const int slot = 3 * moment_digit(ux >> 1, vy >> 1) + moment_digit(ux & 1, vy & 1);
        acc[slot] = __builtin_amdgcn_mfma_i32_32x32x32_i8(fa[ux], fb[vy], acc[slot], 0, 0, 0);
      }
  };
  uint32_t buf = 0;
  bool prev = false;
  for (uint64_t ch = blockIdx.x; ch < nch; ch += gridDim.x, buf ^= 1) {
#pragma unroll
    for (int f = 0; f < 8; ++f) {
      i32x16 a0, a1;
#pragma unroll
      for (int r = 0; r < 16; ++r) a0[r] = a1[r] = 0;
      if constexpr (LC) {
        u32x4 x[16];
#pragma unroll
        for (int k = 0; k < 16; ++k) {
          x[k] = ux[k];
          ux[k] = ux2[k];
        }
        const int u2 = f + 2;  // the fold two ahead
        if (u2 < 8)
          unit_lc(ch, u2, ux2);
        else
          unit_lc(ch + gridDim.x, u2 - 8, ux2);
        to_digits_halves<16>(x);
#pragma unroll
        for (int c = 0; c < 8; ++c) {
          a0 = __builtin_amdgcn_mfma_i32_32x32x32_i8(wf[c], as_i32x4(x[c]), a0, 0, 0, 0);
          a1 = __builtin_amdgcn_mfma_i32_32x32x32_i8(wf[c], as_i32x4(x[8 + c]), a1, 0, 0, 0);
        }
      } else {
        Fe x[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          x[k] = nx[k];
          nx[k] = nx2[k];
        }
        const int u2 = f + 2;  // the fold two ahead
        if (u2 < 8)
          unit_at(ch, u2, nx2);
        else
          unit_at(ch + gridDim.x, u2 - 8, nx2);
        fold_acc8(x, wf, a0, a1);
      }
      int64_t W[8];
      fold_words(a0, a1, W);
      const Fe z = dm_finish<F>(W, fe_zero<F>());
      ZK_DCHECK(pch(ch) * 64 + l + (uint64_t)f * O < 8 * O);
      st_fold(X2, pch(ch) * 64 + l + (uint64_t)f * O, z);
      dm_row<F>(img2[buf][f][w][l], z);
      if ((f & 1) && prev) products(buf ^ 1, f >> 1);  // the previous chunk's products, a quarter at a time
    }
    __syncthreads();  // this chunk's image is complete; the previous one's products are done (its buffer is free)
    prev = true;
  }
  if (prev)
#pragma unroll
    for (int grp = 0; grp < 4; ++grp) products(buf ^ 1, grp);  // the last chunk's products
  } else if constexpr (OCT == 64) {
  uint8_t(*img)[4][64][32] = reinterpret_cast<uint8_t(*)[4][64][32]>(&sc.img[0][0][0][0][0]);
  for (uint64_t ch = blockIdx.x; ch < nch; ch += gridDim.x) {
#pragma unroll
    for (int f = 0; f < 8; ++f) {
      i32x16 a0, a1;
#pragma unroll
      for (int r = 0; r < 16; ++r) a0[r] = a1[r] = 0;
      {
        Fe x[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          x[k] = nx[k];
          nx[k] = nx2[k];
        }
        const int u2 = f + 2;  // the fold two ahead
        if (u2 < 8)
          unit_at(ch, u2, nx2);
        else
          unit_at(ch + gridDim.x, u2 - 8, nx2);
        fold_acc8(x, wf, a0, a1);
      }
      int64_t W[8];
      fold_words(a0, a1, W);
      const Fe z = dm_finish<F>(W, fe_zero<F>());
      ZK_DCHECK(pch(ch) * 64 + l + (uint64_t)f * O < 8 * O);
      st_fold(X2, pch(ch) * 64 + l + (uint64_t)f * O, z);
      dm_row<F>(img[f][w][l], z);
    }
    __syncthreads();  // this chunk's image is complete
    const uint32_t aX = w >> 1, aY = w & 1;
#pragma unroll
    for (int pp = 0; pp < 2; ++pp)
#pragma unroll
      for (int half = 0; half < 2; ++half) {  // K = the 64 octants in two MFMA steps
        i32x4 fa[4], fb[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          fa[k] = tr_frag(&img[4 * aX + k][2 * pp][32 * half][0]);
          fb[k] = tr_frag(&img[4 * aY + k][2 * pp + 1][32 * half][0]);
        }
#pragma unroll
        for (int ux = 0; ux < 4; ++ux)
#pragma unroll
          for (int vy = 0; vy < 4; ++vy) {
            const int slot = 3 * moment_digit(ux >> 1, vy >> 1) + moment_digit(ux & 1, vy & 1);
            acc[slot] = __builtin_amdgcn_mfma_i32_32x32x32_i8(fa[ux], fb[vy], acc[slot], 0, 0, 0);
          }
      }
    __syncthreads();  // the image is rewritten by the next chunk
  }
  } else {
  // (OCT 32: one fold ahead and a rolled fold loop — the small levels are
  // latency-bound, and the unrolled loop with two folds in flight spilled 55
  // VGPRs, whose scratch traffic was 0.4 x the kernel's bytes)
  uint32_t buf = 0;
  for (uint64_t ch = blockIdx.x; ch < nch; ch += gridDim.x, buf ^= 1) {
#pragma unroll 1
    for (int f = 0; f < 4; ++f) {
      Fe x[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) x[k] = nx[k];
      // the next fold (one load site, no branch; past the end: chunk 0, L2-resident)
      in_at(f < 3 ? ch : ch + gridDim.x, f < 3 ? f + 1 : 0, nx);
      const uint32_t corner = 2 * f + hh;
      const Fe z = dm3_fold<F>(x, wf);
      ZK_DCHECK(pch(ch) * 32 + ql + (uint64_t)corner * O < 8 * O);
      st_fold(X2, pch(ch) * 32 + ql + (uint64_t)corner * O, z);
      dm_row<F>(sc.img[buf][corner][w][ql], z);
    }
    __syncthreads();  // this chunk's image is complete (double buffering: one barrier per chunk)
    const uint32_t aX = w >> 1, aY = w & 1;
#pragma unroll
    for (int pp = 0; pp < 2; ++pp) {
      i32x4 fa[4], fb[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        fa[k] = tr_frag(&sc.img[buf][4 * aX + k][2 * pp][0][0]);
        fb[k] = tr_frag(&sc.img[buf][4 * aY + k][2 * pp + 1][0][0]);
      }
#pragma unroll
      for (int ux = 0; ux < 4; ++ux)
#pragma unroll
        for (int vy = 0; vy < 4; ++vy) {
          const int slot = 3 * moment_digit(ux >> 1, vy >> 1) + moment_digit(ux & 1, vy & 1);
          acc[slot] = __builtin_amdgcn_mfma_i32_32x32x32_i8(fa[ux], fb[vy], acc[slot], 0, 0, 0);
        }
    }
  }
  }
  if (blockIdx.x == 0) ZK_SINK_STAMP(sink, 3);  // block 0 leaves its main loop
  ZK_BLOCK_STAMP(sink, 0);
  __syncthreads();
  d0t_flush(acc, sc.T);
  __syncthreads();
  ZK_BLOCK_STAMP(sink, 4);
  tiles_to_words<F, kD0TCats>(sc.T, sc.w17);
  ZK_BLOCK_STAMP(sink, 5);
  words_to_limbs9<F, kD0TCats>(sc.w17, sc.p2w, sc.tot);
  __syncthreads();
  grid_finish<kD0TLimbs>(sc, sink);
}

}  // namespace zk
