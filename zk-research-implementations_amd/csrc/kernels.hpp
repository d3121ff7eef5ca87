// gfx950 kernels of the sum-check hot path (device code; included once by
// sumcheck.hip). Tables are arrays of 32-byte Montgomery elements in HBM,
// index bit (n-1-i) <-> variable i (variable 0 = MSB), exactly the
// `Vec<F>` layout of MultilinearPoly (multilinear_polynomial_evaluation.rs:19-37).
//
// Every fold in the hot path is `partial_evaluate(0, r)` (:52-63): the pair
// (j, j + L/2) collapses to a + r(b - a), so both operands of every pair sit
// in two contiguous half-tables and every load/store is a coalesced 32-byte
// per-lane access (two dwordx4).
#pragma once
#include "field.hpp"

namespace zk {

constexpr int kBlock = 256;  // 4 waves of 64

__device__ __forceinline__ Fe ld_fe(const Fe* __restrict__ p, uint64_t i) {
  const uint4* q = reinterpret_cast<const uint4*>(p) + 2 * i;
  const uint4 a = q[0], b = q[1];
  Fe r;
  r.v[0] = a.x; r.v[1] = a.y; r.v[2] = a.z; r.v[3] = a.w;
  r.v[4] = b.x; r.v[5] = b.y; r.v[6] = b.z; r.v[7] = b.w;
  return r;
}
__device__ __forceinline__ void st_fe(Fe* __restrict__ p, uint64_t i, const Fe& x) {
  uint4* q = reinterpret_cast<uint4*>(p) + 2 * i;
  q[0] = make_uint4(x.v[0], x.v[1], x.v[2], x.v[3]);
  q[1] = make_uint4(x.v[4], x.v[5], x.v[6], x.v[7]);
}

// a + r (b - a)
template <class F>
__device__ __forceinline__ Fe fold1(const Fe& a, const Fe& b, const Fe& r) {
  return fe_add<F>(a, fe_mul<F>(r, fe_sub<F>(b, a)));
}
// X(2) = 2 X_hi - X_lo  (partial_evaluate at F::from(2))
template <class F>
__device__ __forceinline__ Fe at2(const Fe& lo, const Fe& hi) {
  return fe_sub<F>(fe_dbl<F>(hi), lo);
}

// Sum K field elements over the workgroup; thread 0..K-1 write block partial k.
template <class F, int K>
__device__ __forceinline__ void block_reduce_store(Fe (&acc)[K], Fe* __restrict__ partials) {
  __shared__ Fe sm[kBlock / 64][K];
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
#pragma unroll
    for (int k = 0; k < K; ++k) {
      Fe o;
#pragma unroll
      for (int i = 0; i < 8; ++i) o.v[i] = __shfl_xor(acc[k].v[i], off, 64);
      acc[k] = fe_add<F>(acc[k], o);
    }
  }
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  if (lane == 0) {
#pragma unroll
    for (int k = 0; k < K; ++k) sm[wave][k] = acc[k];
  }
  __syncthreads();
  if (threadIdx.x < K) {
    Fe s = sm[0][threadIdx.x];
#pragma unroll
    for (int w = 1; w < kBlock / 64; ++w) s = fe_add<F>(s, sm[w][threadIdx.x]);
    st_fe(partials, (uint64_t)blockIdx.x * K + threadIdx.x, s);
  }
}

// ---------------------------------------------------------------------------
// GKR round 0: e_t = sum_j A_t S_t + M_t P_t for t = 0,1,2 over the input
// tables (size 2h), X_t = X_lo + t (X_hi - X_lo)  — sum_check_protocol.rs:152-166
// with composed_polynomial.rs:78-99 (reduce = A*S + M*P). 6 muls / pair.
// ---------------------------------------------------------------------------
template <class F>
__global__ __launch_bounds__(kBlock) void k_gkr_round0(const Fe* __restrict__ A, const Fe* __restrict__ S,
                                                       const Fe* __restrict__ M, const Fe* __restrict__ P,
                                                       uint64_t h, Fe* __restrict__ partials) {
  Fe acc[3] = {fe_zero<F>(), fe_zero<F>(), fe_zero<F>()};
  const uint64_t stride = (uint64_t)gridDim.x * kBlock;
  for (uint64_t j = (uint64_t)blockIdx.x * kBlock + threadIdx.x; j < h; j += stride) {
    const Fe a0 = ld_fe(A, j), a1 = ld_fe(A, j + h), s0 = ld_fe(S, j), s1 = ld_fe(S, j + h);
    acc[0] = fe_add<F>(acc[0], fe_mul<F>(a0, s0));
    acc[1] = fe_add<F>(acc[1], fe_mul<F>(a1, s1));
    acc[2] = fe_add<F>(acc[2], fe_mul<F>(at2<F>(a0, a1), at2<F>(s0, s1)));
    const Fe m0 = ld_fe(M, j), m1 = ld_fe(M, j + h), p0 = ld_fe(P, j), p1 = ld_fe(P, j + h);
    acc[0] = fe_add<F>(acc[0], fe_mul<F>(m0, p0));
    acc[1] = fe_add<F>(acc[1], fe_mul<F>(m1, p1));
    acc[2] = fe_add<F>(acc[2], fe_mul<F>(at2<F>(m0, m1), at2<F>(p0, p1)));
  }
  block_reduce_store<F, 3>(acc, partials);
}

// ---------------------------------------------------------------------------
// GKR round k >= 1, fused: fold the previous round's tables (size 4h) by
// r_{k-1} (SumPoly::partial_evaluate(r), sum_check_protocol.rs:107) into
// out (size 2h) and accumulate this round's e0 and e2 on the folded values.
// Output pair j needs old j, j+h, j+2h, j+3h: folded lo = old[j] + r(old[j+2h]-old[j]),
// folded hi = old[j+h] + r(old[j+3h]-old[j+h]). e1 is not computed: the host
// derives it exactly as s_{k-1}(r_{k-1}) - e0. out must not alias
// in (the host ping-pongs two workspaces). 12 muls / pair.
// ---------------------------------------------------------------------------
template <class F>
__global__ __launch_bounds__(kBlock) void k_gkr_round(const Fe* __restrict__ A, const Fe* __restrict__ S,
                                                      const Fe* __restrict__ M, const Fe* __restrict__ P,
                                                      Fe* __restrict__ A2, Fe* __restrict__ S2,
                                                      Fe* __restrict__ M2, Fe* __restrict__ P2, uint64_t h, Fe r,
                                                      Fe* __restrict__ partials) {
  Fe acc[2] = {fe_zero<F>(), fe_zero<F>()};
  const uint64_t stride = (uint64_t)gridDim.x * kBlock;
  for (uint64_t j = (uint64_t)blockIdx.x * kBlock + threadIdx.x; j < h; j += stride) {
    Fe a0, a1, s0, s1;
    {
      const Fe x0 = ld_fe(A, j), x1 = ld_fe(A, j + h), x2 = ld_fe(A, j + 2 * h), x3 = ld_fe(A, j + 3 * h);
      a0 = fold1<F>(x0, x2, r);
      a1 = fold1<F>(x1, x3, r);
    }
    {
      const Fe x0 = ld_fe(S, j), x1 = ld_fe(S, j + h), x2 = ld_fe(S, j + 2 * h), x3 = ld_fe(S, j + 3 * h);
      s0 = fold1<F>(x0, x2, r);
      s1 = fold1<F>(x1, x3, r);
    }
    st_fe(A2, j, a0);
    st_fe(A2, j + h, a1);
    st_fe(S2, j, s0);
    st_fe(S2, j + h, s1);
    acc[0] = fe_add<F>(acc[0], fe_mul<F>(a0, s0));
    acc[1] = fe_add<F>(acc[1], fe_mul<F>(at2<F>(a0, a1), at2<F>(s0, s1)));
    Fe m0, m1, p0, p1;
    {
      const Fe x0 = ld_fe(M, j), x1 = ld_fe(M, j + h), x2 = ld_fe(M, j + 2 * h), x3 = ld_fe(M, j + 3 * h);
      m0 = fold1<F>(x0, x2, r);
      m1 = fold1<F>(x1, x3, r);
    }
    {
      const Fe x0 = ld_fe(P, j), x1 = ld_fe(P, j + h), x2 = ld_fe(P, j + 2 * h), x3 = ld_fe(P, j + 3 * h);
      p0 = fold1<F>(x0, x2, r);
      p1 = fold1<F>(x1, x3, r);
    }
    st_fe(M2, j, m0);
    st_fe(M2, j + h, m1);
    st_fe(P2, j, p0);
    st_fe(P2, j + h, p1);
    acc[0] = fe_add<F>(acc[0], fe_mul<F>(m0, p0));
    acc[1] = fe_add<F>(acc[1], fe_mul<F>(at2<F>(m0, m1), at2<F>(p0, p1)));
  }
  block_reduce_store<F, 2>(acc, partials);
}

// ---------------------------------------------------------------------------
// Plain sum-check round (sum_check_protocol.rs:36-46, :168-175).
// FIRST: s0 = sum X[0,h), s1 = sum X[h,2h) over the input table.
// else : fold the previous table (size 4h) by r into out (size 2h) and sum
//        the folded halves. out must not alias X.
// ---------------------------------------------------------------------------
template <class F, bool FIRST>
__global__ __launch_bounds__(kBlock) void k_sc_round(const Fe* __restrict__ X, Fe* __restrict__ Y, uint64_t h, Fe r,
                                                     Fe* __restrict__ partials) {
  Fe acc[2] = {fe_zero<F>(), fe_zero<F>()};
  const uint64_t stride = (uint64_t)gridDim.x * kBlock;
  for (uint64_t j = (uint64_t)blockIdx.x * kBlock + threadIdx.x; j < h; j += stride) {
    if (FIRST) {
      acc[0] = fe_add<F>(acc[0], ld_fe(X, j));
      acc[1] = fe_add<F>(acc[1], ld_fe(X, j + h));
    } else {
      const Fe x0 = ld_fe(X, j), x1 = ld_fe(X, j + h), x2 = ld_fe(X, j + 2 * h), x3 = ld_fe(X, j + 3 * h);
      const Fe f0 = fold1<F>(x0, x2, r), f1 = fold1<F>(x1, x3, r);
      st_fe(Y, j, f0);
      st_fe(Y, j + h, f1);
      acc[0] = fe_add<F>(acc[0], f0);
      acc[1] = fe_add<F>(acc[1], f1);
    }
  }
  block_reduce_store<F, 2>(acc, partials);
}

// ---------------------------------------------------------------------------
// MultilinearPoly::partial_evaluate(bit, r) (:52-63) with pair_points/insert_bit
// (:39-50, :158-164): out[v] = in[lo] + r (in[hi] - in[lo]),
// lo = insert_bit(v, s) (s = nvars-1-bit), hi = lo | 1<<s.  bit 0 -> s = n-1 ->
// lo = v, hi = v + half (contiguous halves).
// ---------------------------------------------------------------------------
template <class F>
__global__ __launch_bounds__(kBlock) void k_fold(const Fe* __restrict__ X, Fe* __restrict__ Y, uint64_t half,
                                                 uint32_t s, Fe r) {
  const uint64_t stride = (uint64_t)gridDim.x * kBlock;
  const uint64_t mask = ((uint64_t)1 << s) - 1;
  for (uint64_t v = (uint64_t)blockIdx.x * kBlock + threadIdx.x; v < half; v += stride) {
    const uint64_t lo = ((v >> s) << (s + 1)) | (v & mask);
    const uint64_t hi = lo | ((uint64_t)1 << s);
    st_fe(Y, v, fold1<F>(ld_fe(X, lo), ld_fe(X, hi), r));
  }
}

// fold four tables by r at bit 0 (used before the multi-GPU all-gather)
template <class F>
__global__ __launch_bounds__(kBlock) void k_fold4(const Fe* __restrict__ A, const Fe* __restrict__ S,
                                                  const Fe* __restrict__ M, const Fe* __restrict__ P,
                                                  Fe* __restrict__ A2, Fe* __restrict__ S2, Fe* __restrict__ M2,
                                                  Fe* __restrict__ P2, uint64_t half, Fe r) {
  const uint64_t stride = (uint64_t)gridDim.x * kBlock;
  for (uint64_t v = (uint64_t)blockIdx.x * kBlock + threadIdx.x; v < half; v += stride) {
    st_fe(A2, v, fold1<F>(ld_fe(A, v), ld_fe(A, v + half), r));
    st_fe(S2, v, fold1<F>(ld_fe(S, v), ld_fe(S, v + half), r));
    st_fe(M2, v, fold1<F>(ld_fe(M, v), ld_fe(M, v + half), r));
    st_fe(P2, v, fold1<F>(ld_fe(P, v), ld_fe(P, v + half), r));
  }
}

// ---------------------------------------------------------------------------
// Block partials [nblk][K] -> K sums, written limb-split: out[k*8+i] = limb i
// (32 bits in a u64 lane). The split form is what the multi-GPU all-reduce
// sums exactly (ncclUint64); the host folds it back mod p.
// ---------------------------------------------------------------------------
template <class F, int K>
__global__ __launch_bounds__(kBlock) void k_reduce_partials(const Fe* __restrict__ partials, uint32_t nblk,
                                                            uint64_t* __restrict__ out) {
  Fe acc[K];
#pragma unroll
  for (int k = 0; k < K; ++k) acc[k] = fe_zero<F>();
  for (uint32_t b = threadIdx.x; b < nblk; b += kBlock) {
#pragma unroll
    for (int k = 0; k < K; ++k) acc[k] = fe_add<F>(acc[k], ld_fe(partials, (uint64_t)b * K + k));
  }
  __shared__ Fe sm[kBlock / 64][K];
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
#pragma unroll
    for (int k = 0; k < K; ++k) {
      Fe o;
#pragma unroll
      for (int i = 0; i < 8; ++i) o.v[i] = __shfl_xor(acc[k].v[i], off, 64);
      acc[k] = fe_add<F>(acc[k], o);
    }
  }
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  if (lane == 0) {
#pragma unroll
    for (int k = 0; k < K; ++k) sm[wave][k] = acc[k];
  }
  __syncthreads();
  if (threadIdx.x < K) {
    Fe s = sm[0][threadIdx.x];
#pragma unroll
    for (int w = 1; w < kBlock / 64; ++w) s = fe_add<F>(s, sm[w][threadIdx.x]);
#pragma unroll
    for (int i = 0; i < 8; ++i) out[threadIdx.x * 8 + i] = s.v[i];
  }
}

// ---------------------------------------------------------------------------
// canonical <-> Montgomery (in place allowed)
// ---------------------------------------------------------------------------
template <class F, bool TO_MONT>
__global__ __launch_bounds__(kBlock) void k_convert(const Fe* X, Fe* Y, uint64_t n) {
  const uint64_t stride = (uint64_t)gridDim.x * kBlock;
  for (uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += stride) {
    const Fe x = ld_fe(X, i);
    st_fe(Y, i, TO_MONT ? fe_to_mont<F>(x) : fe_from_mont<F>(x));
  }
}
// flag non-canonical inputs (>= p) so the host can reject them (ark would
// never hold such a value)
template <class F>
__global__ __launch_bounds__(kBlock) void k_check_canonical(const Fe* X, uint64_t n, uint32_t* bad) {
  const uint64_t stride = (uint64_t)gridDim.x * kBlock;
  uint32_t b = 0;
  for (uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += stride)
    b |= fe_is_canonical<F>(ld_fe(X, i)) ? 0u : 1u;
  if (b) atomicOr(bad, 1u);
}

// ---------------------------------------------------------------------------
// Synthetic tables: limb k of global element i of table t is
// splitmix64(key + 4i + k), key = splitmix64(splitmix64(seed) + t); the
// 256-bit LE value is reduced mod p and stored in Montgomery form.
// ---------------------------------------------------------------------------
__host__ __device__ __forceinline__ uint64_t splitmix64(uint64_t x) {
  uint64_t z = x + 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
template <class F>
__global__ __launch_bounds__(kBlock) void k_synth(Fe* Y, uint64_t n, uint64_t key, uint64_t index0, uint64_t step) {
  const uint64_t stride = (uint64_t)gridDim.x * kBlock;
  for (uint64_t m = (uint64_t)blockIdx.x * kBlock + threadIdx.x; m < n; m += stride) {
    const uint64_t i = index0 + m * step;
    Fe x;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const uint64_t w = splitmix64(key + 4 * i + (uint64_t)k);
      x.v[2 * k] = (uint32_t)w;
      x.v[2 * k + 1] = (uint32_t)(w >> 32);
    }
    // value < 2^256 < 6p for every supported p: at most 5 subtractions
#pragma unroll
    for (int t = 0; t < 5; ++t) x = fe_reduce_once<F>(x);
    st_fe(Y, m, fe_to_mont<F>(x));
  }
}

}  // namespace zk
