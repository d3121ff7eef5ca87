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

// Where a round kernel's K partial sums go. Every block publishes its
// partial with write-through (sc1) 8-byte stores, drains them, and one lane
// bumps an agent-scope counter; the block whose add returns gridDim-1 reads
// all partials back with sc1 loads (MI355X_MICROARCH.md "Valid forms", first
// row of the sc1 hand-off table: no release/acquire fence, so the dirty L2
// full of freshly folded table lines is never written back mid-kernel). It
// writes the K totals limb-split (one u64 per 32-bit limb — the form the
// multi-GPU all-reduce sums exactly) to dev_out and/or pinned host memory and
// raises host_flag = tag with a system-scope release; the host spins on that
// flag instead of synchronising the stream.
struct RoundSink {
  Fe* partials;         // [gridDim.x + 8][4]: one 128-B slot per block, then 8 shard slots
  uint32_t* counter;    // 9 counters, 128 B apart: 8 XCD shards + top; zero at launch, reset by their last user
  uint64_t* accum;      // K*8 u64 limb-split accumulator (small grids); zero at launch, reset by the last block
  uint64_t* dev_out;    // K*8 u64 in device memory, or null
  uint64_t* host_out;   // K*8 u64 in pinned host memory, or null
  uint32_t* host_flag;  // pinned host word, or null
  uint32_t tag;
};

__device__ __forceinline__ void st_fe_sc1(Fe* p, uint64_t i, const Fe& x) {
  uint64_t* q = reinterpret_cast<uint64_t*>(p + i);
#pragma unroll
  for (int w = 0; w < 4; ++w)
    __hip_atomic_store(q + w, (uint64_t)x.v[2 * w] | ((uint64_t)x.v[2 * w + 1] << 32), __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ Fe ld_fe_sc1(Fe* p, uint64_t i) {
  uint64_t* q = reinterpret_cast<uint64_t*>(p + i);
  Fe x;
#pragma unroll
  for (int w = 0; w < 4; ++w) {
    const uint64_t v = __hip_atomic_load(q + w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    x.v[2 * w] = (uint32_t)v;
    x.v[2 * w + 1] = (uint32_t)(v >> 32);
  }
  return x;
}

// Block-level sums use plain 288-bit integer adds (9 words, no modular
// reduction per step): 256 values < p sum to < 2^264. One reduction mod p at
// the end (lo256 mod p + hi * 2^256 mod p).
struct W9 {
  uint32_t w[9];
};
__device__ __forceinline__ void w9_add(W9& a, const W9& b) {
  uint32_t c = 0;
#pragma unroll
  for (int i = 0; i < 9; ++i) a.w[i] = addc32(a.w[i], b.w[i], c, &c);
}
template <class F>
__device__ __forceinline__ Fe w9_reduce(const W9& a) {
  Fe lo;
#pragma unroll
  for (int i = 0; i < 8; ++i) lo.v[i] = a.w[i];
#pragma unroll
  for (int i = 0; i < 5; ++i) lo = fe_reduce_once<F>(lo);  // 2^256 < 6p
  if (a.w[8] == 0) return lo;
  Fe hi = fe_zero<F>(), r2;
  hi.v[0] = a.w[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) r2.v[i] = F::R2[i];
  return fe_add<F>(lo, fe_mul<F>(hi, r2));  // hi * 2^256 mod p
}

// sum K elements over the workgroup; the result is valid in threads 0..K-1
template <class F, int K>
__device__ __forceinline__ Fe block_sum(const Fe (&acc)[K], W9 (&sm)[kBlock / 64][K]) {
  W9 v[K];
#pragma unroll
  for (int k = 0; k < K; ++k) {
#pragma unroll
    for (int i = 0; i < 8; ++i) v[k].w[i] = acc[k].v[i];
    v[k].w[8] = 0;
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
#pragma unroll
    for (int k = 0; k < K; ++k) {
      W9 o;
#pragma unroll
      for (int i = 0; i < 9; ++i) o.w[i] = __shfl_xor(v[k].w[i], off, 64);
      w9_add(v[k], o);
    }
  }
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  if (lane == 0) {
#pragma unroll
    for (int k = 0; k < K; ++k) sm[wave][k] = v[k];
  }
  __syncthreads();
  Fe s = fe_zero<F>();
  if (threadIdx.x < K) {
    W9 t = sm[0][threadIdx.x];
#pragma unroll
    for (int w = 1; w < kBlock / 64; ++w) w9_add(t, sm[w][threadIdx.x]);
    s = w9_reduce<F>(t);
  }
  return s;
}

// final K totals -> limb-split outputs + host flag
template <int K>
__device__ __forceinline__ void publish_totals(const Fe& t, const RoundSink& sk) {
  if (threadIdx.x < K) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      if (sk.dev_out) sk.dev_out[threadIdx.x * 8 + i] = t.v[i];
      if (sk.host_out) sk.host_out[threadIdx.x * 8 + i] = t.v[i];
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0 && sk.host_flag) {
    __threadfence_system();
    __hip_atomic_store(sk.host_flag, sk.tag, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

// sum slots [first, first + count*stride) of `slots` (sc1 loads), spread over the block
template <class F, int K>
__device__ __forceinline__ Fe sum_slots(Fe* slots, uint32_t first, uint32_t stride, uint32_t count,
                                        W9 (&sm)[kBlock / 64][K]) {
  W9 tot[K];
#pragma unroll
  for (int k = 0; k < K; ++k)
#pragma unroll
    for (int i = 0; i < 9; ++i) tot[k].w[i] = 0;
  for (uint32_t b = threadIdx.x; b < count; b += kBlock) {
    Fe x[K];
#pragma unroll
    for (int k = 0; k < K; ++k) x[k] = ld_fe_sc1(slots, (uint64_t)(first + b * stride) * 4 + k);
#pragma unroll
    for (int k = 0; k < K; ++k) {
      W9 y;
#pragma unroll
      for (int i = 0; i < 8; ++i) y.w[i] = x[k].v[i];
      y.w[8] = 0;
      w9_add(tot[k], y);
    }
  }
  Fe red[K];
#pragma unroll
  for (int k = 0; k < K; ++k) red[k] = w9_reduce<F>(tot[k]);
  __syncthreads();  // sm is reused
  return block_sum<F, K>(red, sm);
}

constexpr uint32_t kAtomicFaninMax = 64;  // grids up to this size fan in through limb atomics

// Cross-block fan-in in two levels so no counter sees more than ~gridDim/8
// arrivals (one device-scope counter serialises ~12 ns per arrival:
// MI355X_MICROARCH.md "fanin"): blocks of shard s = blockIdx % 8 (one XCD
// under round-robin placement — speed only, never correctness) meet on
// counter s; each shard's last block sums the shard and meets the other
// shards' last blocks on the top counter; the very last one publishes.
template <class F, int K>
__device__ __forceinline__ void block_reduce_finish(Fe (&acc)[K], const RoundSink& sk) {
  __shared__ W9 sm[kBlock / 64][K];
  __shared__ uint32_t am_last;
  const Fe s = block_sum<F, K>(acc, sm);
  const uint32_t G = gridDim.x;
  if (G == 1) {  // single block: its sum is the total
    publish_totals<K>(s, sk);
    return;
  }
  if (G <= kAtomicFaninMax) {
    // Small grid: every block adds its K sums limb by limb (no-return u64
    // atomics at the device-coherent level; G * 2^32 < 2^64 stays exact),
    // drains, and counts in; the last block reads the totals with sc1 loads.
    if (threadIdx.x < K) {
#pragma unroll
      for (int i = 0; i < 8; ++i)
        __hip_atomic_fetch_add(sk.accum + threadIdx.x * 8 + i, (uint64_t)s.v[i], __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
      const uint32_t prev = __hip_atomic_fetch_add(sk.counter, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      am_last = prev == G - 1;
    }
    __syncthreads();
    if (!am_last) return;
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    Fe t = fe_zero<F>();
    if (threadIdx.x < K) {
      uint64_t w[8];
#pragma unroll
      for (int i = 0; i < 8; ++i)
        w[i] = __hip_atomic_exchange(sk.accum + threadIdx.x * 8 + i, (uint64_t)0, __ATOMIC_RELAXED,
                                     __HIP_MEMORY_SCOPE_AGENT);  // read and re-arm for the next launch
      W9 y;
      uint64_t c = 0;
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const uint64_t v = w[i] + c;
        y.w[i] = (uint32_t)v;
        c = v >> 32;
      }
      y.w[8] = (uint32_t)c;
      t = w9_reduce<F>(y);
    }
    if (threadIdx.x == 0) __hip_atomic_store(sk.counter, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    publish_totals<K>(t, sk);
    return;
  }
  const uint32_t shard = blockIdx.x & 7u, nshards = G < 8 ? G : 8u;
  const uint32_t in_shard = (G - shard + 7u) / 8u;
  if (threadIdx.x < K) st_fe_sc1(sk.partials, (uint64_t)blockIdx.x * 4 + threadIdx.x, s);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the storing wave drains before the signal
  __syncthreads();
  if (threadIdx.x == 0) {
    const uint32_t prev =
        __hip_atomic_fetch_add(sk.counter + 32 * shard, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    am_last = prev == in_shard - 1;
  }
  __syncthreads();
  if (!am_last) return;
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // no instruction: keeps the loads below the add
  const Fe ts = sum_slots<F, K>(sk.partials, shard, 8u, in_shard, sm);
  if (threadIdx.x < K) st_fe_sc1(sk.partials, (uint64_t)(G + shard) * 4 + threadIdx.x, ts);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    __hip_atomic_store(sk.counter + 32 * shard, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // next launch
    const uint32_t prev = __hip_atomic_fetch_add(sk.counter + 32 * 8, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    am_last = prev == nshards - 1;
  }
  __syncthreads();
  if (!am_last) return;
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  const Fe t = sum_slots<F, K>(sk.partials, G, 1u, nshards, sm);
  if (threadIdx.x == 0) __hip_atomic_store(sk.counter + 32 * 8, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  publish_totals<K>(t, sk);
}

// copy K*8 u64 (e.g. after an RCCL all-reduce) to pinned host memory + flag
__global__ void k_publish(const uint64_t* __restrict__ src, int n, uint64_t* host_out, uint32_t* host_flag,
                          uint32_t tag) {
  if (threadIdx.x < n) host_out[threadIdx.x] = src[threadIdx.x];
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    __threadfence_system();
    __hip_atomic_store(host_flag, tag, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

// ---------------------------------------------------------------------------
// GKR round 0: e_t = sum_j A_t S_t + M_t P_t for t = 0,1,2 over the input
// tables (size 2h), X_t = X_lo + t (X_hi - X_lo)  — sum_check_protocol.rs:152-166
// with composed_polynomial.rs:78-99 (reduce = A*S + M*P). 6 unreduced products / pair.
// ---------------------------------------------------------------------------
// Two threads per pair: waves alternate between the product A*S (q = 0) and
// M*P (q = 1), so a thread issues its 4 (round 0) or 8 (fused round) loads at
// once and keeps register pressure low enough for 4 waves/SIMD.
__device__ __forceinline__ void pair_slot(uint64_t& j, uint32_t& q, uint64_t& step) {
  const uint64_t g = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
  q = (uint32_t)(g >> 6) & 1u;
  j = ((g >> 7) << 6) | (g & 63);
  step = (uint64_t)gridDim.x * (kBlock / 2);
}

template <class F>
__global__ __launch_bounds__(kBlock) void k_gkr_round0(const Fe* __restrict__ A, const Fe* __restrict__ S,
                                                       const Fe* __restrict__ M, const Fe* __restrict__ P,
                                                       uint64_t h, RoundSink sink) {
  // products accumulate unreduced (Wide) and are reduced once per thread
  Wide w0 = wide_zero<F>(), w1 = wide_zero<F>(), w2 = wide_zero<F>();
  uint64_t j, step;
  uint32_t q;
  pair_slot(j, q, step);
  const Fe* __restrict__ X = q ? M : A;
  const Fe* __restrict__ Z = q ? P : S;
  for (; j < h; j += step) {
    const Fe x0 = ld_fe(X, j), x1 = ld_fe(X, j + h), z0 = ld_fe(Z, j), z1 = ld_fe(Z, j + h);
    __builtin_amdgcn_sched_barrier(0);  // issue all loads before any arithmetic
    wide_mac<F>(w0, x0, z0);
    wide_mac<F>(w1, x1, z1);
    wide_mac<F>(w2, at2<F>(x0, x1), at2<F>(z0, z1));
  }
  Fe acc[3] = {wide_redc<F>(w0), wide_redc<F>(w1), wide_redc<F>(w2)};
  block_reduce_finish<F, 3>(acc, sink);
}

// ---------------------------------------------------------------------------
// GKR round k >= 1, fused: fold the previous round's tables (size 4h) by
// r_{k-1} (SumPoly::partial_evaluate(r), sum_check_protocol.rs:107) into
// out (size 2h) and accumulate this round's e0 and e2 on the folded values.
// Output pair j needs old j, j+h, j+2h, j+3h: folded lo = old[j] + r(old[j+2h]-old[j]),
// folded hi = old[j+h] + r(old[j+3h]-old[j+h]). e1 is not computed: the host
// derives it exactly as s_{k-1}(r_{k-1}) - e0. out must not alias
// in (the host ping-pongs two workspaces). 8 reduced muls + 4 unreduced products / pair.
// ---------------------------------------------------------------------------
// A/B knobs (defaults are the tuned values): minimum waves per SIMD for the
// fused round kernel, and whether all loads are forced ahead of the arithmetic.
#ifndef ZK_ROUND_WAVES
#define ZK_ROUND_WAVES 1
#endif
#ifndef ZK_ROUND_LOADS_FIRST
#define ZK_ROUND_LOADS_FIRST 1
#endif
template <class F>
__global__ __launch_bounds__(kBlock, ZK_ROUND_WAVES) void k_gkr_round(const Fe* __restrict__ A, const Fe* __restrict__ S,
                                                      const Fe* __restrict__ M, const Fe* __restrict__ P,
                                                      Fe* __restrict__ A2, Fe* __restrict__ S2,
                                                      Fe* __restrict__ M2, Fe* __restrict__ P2, uint64_t h, Fe r,
                                                      RoundSink sink) {
  Wide w0 = wide_zero<F>(), w2 = wide_zero<F>();
  uint64_t j, step;
  uint32_t q;
  pair_slot(j, q, step);
  const Fe* __restrict__ X = q ? M : A;
  const Fe* __restrict__ Z = q ? P : S;
  Fe* __restrict__ X2 = q ? M2 : A2;
  Fe* __restrict__ Z2 = q ? P2 : S2;
  for (; j < h; j += step) {
    const Fe x0 = ld_fe(X, j), x1 = ld_fe(X, j + h), x2 = ld_fe(X, j + 2 * h), x3 = ld_fe(X, j + 3 * h);
    const Fe z0 = ld_fe(Z, j), z1 = ld_fe(Z, j + h), z2 = ld_fe(Z, j + 2 * h), z3 = ld_fe(Z, j + 3 * h);
#if ZK_ROUND_LOADS_FIRST
    __builtin_amdgcn_sched_barrier(0);  // issue all loads before any arithmetic
#endif
    const Fe a0 = fold1<F>(x0, x2, r), a1 = fold1<F>(x1, x3, r);
    const Fe s0 = fold1<F>(z0, z2, r), s1 = fold1<F>(z1, z3, r);
    st_fe(X2, j, a0);
    st_fe(X2, j + h, a1);
    st_fe(Z2, j, s0);
    st_fe(Z2, j + h, s1);
    wide_mac<F>(w0, a0, s0);
    wide_mac<F>(w2, at2<F>(a0, a1), at2<F>(s0, s1));
  }
  Fe acc[2] = {wide_redc<F>(w0), wide_redc<F>(w2)};
  block_reduce_finish<F, 2>(acc, sink);
}

// ---------------------------------------------------------------------------
// Same round as k_gkr_round for SMALL tables, where a thread-per-pair kernel is
// latency-bound (one wave serialises 12 dependent 256-bit multiplies). Here 8
// lanes share a pair: lane s folds table s>>1, half s&1 (one multiply); odd
// lanes turn (lo, hi) into X(2) = 2 hi - lo; lanes {0,1,4,5} multiply with lane
// s+2 (A*S / M*P at t = 0 and t = 2). Critical path: 2 multiplies.
// ---------------------------------------------------------------------------
__device__ __forceinline__ Fe shfl_fe(const Fe& x, int src) {
  Fe r;
#pragma unroll
  for (int i = 0; i < 8; ++i) r.v[i] = __shfl(x.v[i], src, 64);
  return r;
}
template <class F>
__global__ __launch_bounds__(kBlock) void k_gkr_round_lanes(const Fe* __restrict__ A, const Fe* __restrict__ S,
                                                            const Fe* __restrict__ M, const Fe* __restrict__ P,
                                                            Fe* __restrict__ A2, Fe* __restrict__ S2,
                                                            Fe* __restrict__ M2, Fe* __restrict__ P2, uint64_t h,
                                                            Fe r, RoundSink sink) {
  const uint32_t lane = threadIdx.x & 63, s = threadIdx.x & 7, tb = s >> 1, half = s & 1;
  const Fe* __restrict__ X = tb == 0 ? A : tb == 1 ? S : tb == 2 ? M : P;
  Fe* __restrict__ Y = tb == 0 ? A2 : tb == 1 ? S2 : tb == 2 ? M2 : P2;
  Fe acc[2] = {fe_zero<F>(), fe_zero<F>()};
  const uint64_t stride = (uint64_t)gridDim.x * (kBlock / 8);
  // the loop bound is uniform per 8-lane group (and per wave: 8 groups share j's stride)
  for (uint64_t j = ((uint64_t)blockIdx.x * kBlock + threadIdx.x) >> 3; j < h; j += stride) {
    const uint64_t o = j + half * h;
    const Fe f = fold1<F>(ld_fe(X, o), ld_fe(X, o + 2 * h), r);
    st_fe(Y, o, f);
    const Fe lo = shfl_fe(f, (int)(lane & ~1u));        // the group's lo for this table
    const Fe v = half ? at2<F>(lo, f) : f;               // even: X(0), odd: X(2)
    const Fe partner = shfl_fe(v, (int)((lane + 2) & 63));
    const Fe prod = fe_mul<F>(v, partner);
    if (s == 0 || s == 4) acc[0] = fe_add<F>(acc[0], prod);
    if (s == 1 || s == 5) acc[1] = fe_add<F>(acc[1], prod);
  }
  block_reduce_finish<F, 2>(acc, sink);
}

// ---------------------------------------------------------------------------
// Plain sum-check round (sum_check_protocol.rs:36-46, :168-175).
// FIRST: s0 = sum X[0,h), s1 = sum X[h,2h) over the input table.
// else : fold the previous table (size 4h) by r into out (size 2h) and sum
//        the folded halves. out must not alias X.
// ---------------------------------------------------------------------------
template <class F, bool FIRST>
__global__ __launch_bounds__(kBlock) void k_sc_round(const Fe* __restrict__ X, Fe* __restrict__ Y, uint64_t h, Fe r,
                                                     RoundSink sink) {
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
  block_reduce_finish<F, 2>(acc, sink);
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
