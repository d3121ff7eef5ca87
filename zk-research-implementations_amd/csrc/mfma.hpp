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
// k_gkr_d0r, same nine categories and limb-sum output) with the products on
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
// 17-word product sum of the VALU kernels — and grid_finish as k_gkr_d0r.
// Bounds: |C| <= 2^19 per chunk, so a wave takes at most kD0MChunksMax
// chunks (int32 tiles); |G| < 2 * 2^16 * 2^510 < M < 2^530 for a block.
// ---------------------------------------------------------------------------
constexpr uint32_t kD0MChunksMax = 2048;  // chunks of 32 quads per wave (int32 tile bound)
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
    for (int k = 0; k < 4; ++k) c[k] = ld_fe(T, j + k * Q);
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

}  // namespace zk
