// gfx950 kernels of the multilinear KZG commitment over BLS12-381 G1
// (pcs/src/kzg_pcs/kzg.rs). Host orchestration in
// zk_sumcheck.hip ("KZG").
//
// MSM (Pippenger). The reference commits with a naive sum of n full scalar
// multiplications (evaluate_poly_with_l_basis_in_g1, kzg.rs:131-144). Here:
// scalars are cut into W = ceil(255 / c) windows of c bits; every nonzero
// digit puts its point into bucket (w, d) (a blocked counting sort, below);
// buckets are summed by a segmented reduction (tasks of <= kSegTask points, repeated over the partial sums until every bucket is one task, so a
// skewed scalar distribution — all equal, all zero — never serialises on one
// thread); each window's sum_d d * B_d comes from running sums over chunks of
// buckets; the host combines the W window sums (Horner, c doublings each).
// Every step is exact group arithmetic, so the result is the same group
// element as the reference's.
#pragma once
#include "ec.hpp"
#include "kernels.hpp"

namespace zk {

constexpr uint32_t kSegTask = 32;    // points summed by one thread per reduction level
constexpr uint32_t kBucketChunkMax = 32;  // buckets per thread in the window reduction (host-chosen, a power of two <= 32: c >= 6)

__device__ __forceinline__ Fq ld_fq(const Fq* p, uint64_t i) { return p[i]; }

// ---- exclusive scan of u32 (in place), 2048 per block ------------------------
constexpr uint32_t kScanPer = 8, kScanBlock = kBlock * kScanPer;
__global__ __launch_bounds__(kBlock) void k_scan_block(uint32_t* __restrict__ a, uint64_t n,
                                                       uint32_t* __restrict__ block_sums) {
  __shared__ uint32_t s[kBlock];
  const uint64_t base = (uint64_t)blockIdx.x * kScanBlock + (uint64_t)threadIdx.x * kScanPer;
  uint32_t v[kScanPer], tot = 0;
#pragma unroll
  for (uint32_t k = 0; k < kScanPer; ++k) {
    v[k] = base + k < n ? a[base + k] : 0u;
    tot += v[k];
  }
  s[threadIdx.x] = tot;
  __syncthreads();
  for (uint32_t off = 1; off < kBlock; off <<= 1) {  // Hillis-Steele inclusive scan of the thread totals
    const uint32_t x = threadIdx.x >= off ? s[threadIdx.x - off] : 0u;
    __syncthreads();
    s[threadIdx.x] += x;
    __syncthreads();
  }
  uint32_t run = s[threadIdx.x] - tot;  // exclusive prefix of this thread
#pragma unroll
  for (uint32_t k = 0; k < kScanPer; ++k) {
    if (base + k < n) a[base + k] = run;
    run += v[k];
  }
  if (threadIdx.x == kBlock - 1 && block_sums) block_sums[blockIdx.x] = s[kBlock - 1];
}
__global__ __launch_bounds__(kBlock) void k_scan_add(uint32_t* __restrict__ a, uint64_t n,
                                                     const uint32_t* __restrict__ block_off) {
  const uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
  if (i < n) a[i] += block_off[i / kScanBlock];
}

// ---- bucket sort --------------------------------------------------------------
// digit w of a canonical 255-bit scalar (8 x u32 LE)
// (words picked by selects: a dynamic index into s.v would put s in scratch)
__device__ __forceinline__ uint32_t fe_word(const Fe& s, uint32_t k) {
  uint32_t r = 0;
#pragma unroll
  for (uint32_t j = 0; j < 8; ++j) r = k == j ? s.v[j] : r;
  return r;
}
__device__ __forceinline__ uint32_t scalar_digit(const Fe& s, uint32_t bit, uint32_t c) {
  const uint32_t wi = bit >> 5, sh = bit & 31;
  const uint64_t x = (uint64_t)fe_word(s, wi) | (uint64_t)fe_word(s, wi + 1) << 32;  // (word 8 reads as 0)
  return (uint32_t)(x >> sh) & ((1u << c) - 1u);
}
// Signed digits (round 4): W windows of c bits with W c >= 256, each digit in
// (-2^(c-1), 2^(c-1)] (a window above 2^(c-1) becomes negative and carries one
// into the next; the last carry fits in the top window). A point goes to the
// bucket of its digit's magnitude m — m mod 2^(c-1), so m = 2^(c-1) shares
// bucket 0, which the host weighs separately — with y negated for a negative
// digit: half the buckets of unsigned digits for the same additions.
template <class Fn>
__device__ __forceinline__ void signed_digits(const Fe& s, uint32_t c, uint32_t W, Fn&& f) {
  const uint32_t half = 1u << (c - 1);
  uint32_t carry = 0;
  for (uint32_t w = 0; w < W; ++w) {
    const uint32_t raw = scalar_digit(s, w * c, c) + carry;
    const uint32_t neg = raw > half ? 1u : 0u;
    carry = neg;
    const uint32_t m = neg ? (1u << c) - raw : raw;
    if (m) f(w, m & (half - 1u), neg);
  }
}
// The entries sorted by (window, bucket) without a global atomic per entry (a
// count / scan / scatter with one global atomic per entry took 8.2 + 21.6 ms
// at 2^24 points against 0.5 + 3.2 + 5.6 ms here, round 4). Bucket keys
// (b = c - 1 bits) split into C coarse = LOW bits and F fine = HIGH bits
// (F = b / 2): the top window's keys are small (its digits hold the scalar's
// last bits), and low coarse bits spread them over every bin. Buckets are
// therefore stored at bucket_slot(key) = low << F | high (window sums read
// them through it):
//  1. k_sort_hist: block b counts its `pts` points' entries per (window,
//     coarse bin) in LDS and stores the counts bin-major, H[bin NB + b];
//  2. an exclusive scan of H gives every block its run in every coarse bin;
//  3. k_sort_scatter: the block writes (point, sign, fine) into its runs (LDS
//     cursors, runs of ~pts / 2^C entries);
//  4. k_sort_fine: one block per coarse bin counting-sorts its entries by the
//     fine bits in LDS and writes the bucket offsets (the exclusive scan of the
//     per-bucket counts, `cnt`) and the point order `ord` (bit 31: negate).
// Within a bucket the order is arbitrary (LDS atomics): bucket sums are group
// sums.
// points per block in passes 1 and 3: kSortPts for large MSMs; small ones use
// fewer (sort_block_pts), so that their passes run on more than a few blocks
constexpr uint32_t kSortPts = 16384;
__host__ __device__ __forceinline__ uint32_t sort_block_pts(uint64_t n) {
  const uint64_t p = (n + 255) / 256;
  return (uint32_t)(p < 1024 ? 1024 : (p > kSortPts ? kSortPts : p));
}
// coarse-bin tables in LDS (Wt 2^C entries): single MSMs need at most 13 x 1024
// (c = 20); the level-batched pass up to 520 x 32 (20 levels of 10 bits).
// k_sort_hist / k_sort_scatter are instantiated for both, so ordinary MSMs keep
// the smaller table (occupancy of the sort passes).
constexpr uint32_t kSortBinsSingle = 13312;
constexpr uint32_t kSortBinsMax = 16896;
static_assert(kSortBinsMax * 4 <= 160 * 1024, "the batched pass's bin table exceeds gfx950's LDS per workgroup");
__host__ __device__ __forceinline__ uint32_t sort_fine_bits(uint32_t b) { return b / 2; }
__host__ __device__ __forceinline__ uint32_t bucket_slot(uint32_t key, uint32_t b) {
  const uint32_t F = sort_fine_bits(b), C = b - F;
  return ((key & ((1u << C) - 1u)) << F) | (key >> C);
}
// Level-batched MSMs (msm_levels, kzg_get_proof's small quotients): point i
// belongs to level floor(log2(i + 1)) — levels of 1, 2, 4, ... points laid out
// back to back, as the setup stores its Lagrange bases — and its digits go to
// that level's W windows: window index level W + w of Wt = levels W.
__device__ __forceinline__ uint32_t point_window0(uint64_t i, uint32_t W, uint32_t levels) {
  return levels ? (63u - (uint32_t)__builtin_clzll(i + 1)) * W : 0u;
}
template <uint32_t BINS>
__global__ __launch_bounds__(kBlock) void k_sort_hist(const Fe* __restrict__ scalars, uint64_t n, uint32_t c,
                                                      uint32_t W, uint32_t levels, uint32_t NB, uint32_t pts,
                                                      uint32_t* __restrict__ H) {
  __shared__ uint32_t hist[BINS];
  const uint32_t F = sort_fine_bits(c - 1), C = c - 1 - F, nbin = (levels ? levels * W : W) << C;
  for (uint32_t j = threadIdx.x; j < nbin; j += kBlock) hist[j] = 0;
  __syncthreads();
  const uint64_t p0 = (uint64_t)blockIdx.x * pts, p1 = p0 + pts < n ? p0 + pts : n;
  for (uint64_t i = p0 + threadIdx.x; i < p1; i += kBlock) {
    const uint32_t w0 = point_window0(i, W, levels);
    signed_digits(ld_fe(scalars, i), c, W, [&](uint32_t w, uint32_t key, uint32_t) {
      atomicAdd(&hist[((w0 + w) << C) + (key & ((1u << C) - 1u))], 1u);
    });
  }
  __syncthreads();
  for (uint32_t j = threadIdx.x; j < nbin; j += kBlock) H[(uint64_t)j * NB + blockIdx.x] = hist[j];
}
template <uint32_t BINS>
__global__ __launch_bounds__(kBlock) void k_sort_scatter(const Fe* __restrict__ scalars, uint64_t n, uint32_t c,
                                                         uint32_t W, uint32_t levels, uint32_t NB, uint32_t pts,
                                                         const uint32_t* __restrict__ Hs, uint64_t* __restrict__ E) {
  __shared__ uint32_t cur[BINS];
  const uint32_t F = sort_fine_bits(c - 1), C = c - 1 - F, nbin = (levels ? levels * W : W) << C;
  for (uint32_t j = threadIdx.x; j < nbin; j += kBlock) cur[j] = Hs[(uint64_t)j * NB + blockIdx.x];
  __syncthreads();
  const uint64_t p0 = (uint64_t)blockIdx.x * pts, p1 = p0 + pts < n ? p0 + pts : n;
  for (uint64_t i = p0 + threadIdx.x; i < p1; i += kBlock) {
    const uint32_t w0 = point_window0(i, W, levels);
    signed_digits(ld_fe(scalars, i), c, W, [&](uint32_t w, uint32_t key, uint32_t neg) {
      const uint32_t pos = atomicAdd(&cur[((w0 + w) << C) + (key & ((1u << C) - 1u))], 1u);
      ZK_DCHECK((uint64_t)pos < n * W);
      E[pos] = (i << (F + 1)) | ((uint64_t)neg << F) | (key >> C);
    });
  }
}
// grid = W 2^C blocks, one per coarse bin; cnt gets (W << b) + 1 offsets (b: bucket bits)
__global__ __launch_bounds__(kBlock) void k_sort_fine(const uint64_t* __restrict__ E, uint32_t b, uint32_t NB,
                                                      const uint32_t* __restrict__ Hs, uint32_t* __restrict__ cnt,
                                                      uint32_t* __restrict__ ord) {
  __shared__ uint32_t h[1024];
  __shared__ uint32_t part[kBlock];
  const uint32_t F = sort_fine_bits(b), nf = 1u << F, bin = blockIdx.x, t = threadIdx.x;
  const uint32_t start = Hs[(uint64_t)bin * NB], end = Hs[(uint64_t)(bin + 1) * NB];  // (H has one total entry past the bins)
  for (uint32_t f = t; f < nf; f += kBlock) h[f] = 0;
  __syncthreads();
  for (uint32_t e = start + t; e < end; e += kBlock) atomicAdd(&h[(uint32_t)E[e] & (nf - 1u)], 1u);
  __syncthreads();
  // exclusive scan of h[0, nf): each thread scans its 4 (nf <= 1024), then the thread totals
  uint32_t v[4], tot = 0;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const uint32_t f = 4 * t + k;
    v[k] = f < nf ? h[f] : 0u;
    tot += v[k];
  }
  part[t] = tot;
  __syncthreads();
  for (uint32_t off = 1; off < kBlock; off <<= 1) {
    const uint32_t x = t >= off ? part[t - off] : 0u;
    __syncthreads();
    part[t] += x;
    __syncthreads();
  }
  uint32_t run = start + part[t] - tot;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const uint32_t f = 4 * t + k;
    if (f < nf) {
      h[f] = run;  // becomes the cursor of fine digit f
      cnt[((uint64_t)bin << F) + f] = run;
    }
    run += v[k];
  }
  if (bin + 1 == gridDim.x && t == 0) cnt[(uint64_t)gridDim.x << F] = end;  // the total
  __syncthreads();
  for (uint32_t e = start + t; e < end; e += kBlock) {
    const uint64_t x = E[e];
    const uint32_t pos = atomicAdd(&h[(uint32_t)x & (nf - 1u)], 1u);
    ZK_DCHECK(pos >= start && pos < end);
    ord[pos] = (uint32_t)(x >> (F + 1)) | ((uint32_t)(x >> F) & 1u) << 31;
  }
}

// ---- segmented reduction --------------------------------------------------------
// Segment s = items [off[s], off[s+1]). Level: segment s gets ceil(len/T) tasks
// (at least 1, so empty segments yield infinity); task t of segment s sums
// items [off[s] + k T, min(off[s+1], off[s] + (k+1) T)).
__global__ __launch_bounds__(kBlock) void k_seg_task_counts(const uint32_t* __restrict__ off, uint64_t nseg,
                                                            uint32_t task, uint32_t* __restrict__ tasks) {
  const uint64_t s = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
  if (s >= nseg) return;
  const uint32_t len = off[s + 1] - off[s];
  tasks[s] = len ? (len + task - 1) / task : 1u;
}
// task_seg[task_off[s] + k] = s
__global__ __launch_bounds__(kBlock) void k_seg_task_owner(const uint32_t* __restrict__ task_off, uint64_t nseg,
                                                           uint32_t ntasks, uint32_t* __restrict__ task_seg) {
  const uint64_t s = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
  if (s >= nseg) return;
  const uint32_t a = task_off[s], b = s + 1 < nseg ? task_off[s + 1] : ntasks;
  for (uint32_t t = a; t < b; ++t) task_seg[t] = (uint32_t)s;
}
// GATHER: items are affine bases[order[j]]; else contiguous Jacobian points
template <bool GATHER>
__global__ __launch_bounds__(kBlock) void k_seg_sum(const G1A* __restrict__ bases, uint64_t nbases,
                                                    const uint32_t* __restrict__ order,
                                                    const G1J* __restrict__ items, const uint32_t* __restrict__ off,
                                                    const uint32_t* __restrict__ task_off,
                                                    const uint32_t* __restrict__ task_seg, uint32_t ntasks,
                                                    uint32_t task, G1J* __restrict__ out) {
  const uint32_t t = blockIdx.x * kBlock + threadIdx.x;
  if (t >= ntasks) return;
  const uint32_t s = task_seg[t], k = t - task_off[s];
  const uint32_t a = off[s] + k * task, e = off[s + 1];
  const uint32_t b = a + task < e ? a + task : e;
  if constexpr (GATHER) {  // XYZZ accumulator over affine points (ec.hpp); order bit 31: negative digit
    G1XYZZ acc = g1x_inf();
    for (uint32_t j = a; j < b; ++j) {
      const uint32_t o = order[j];
      ZK_DCHECK((o & 0x7fffffffu) < nbases);
      G1A p = bases[o & 0x7fffffffu];
      if (o >> 31) p.y = fq_neg(p.y);
      acc = g1x_add_mixed(acc, p);
    }
    out[t] = g1x_to_jac(acc);
  } else {
    G1J acc = g1_inf();
    for (uint32_t j = a; j < b; ++j) acc = g1_add(acc, items[j]);
    out[t] = acc;
  }
}

// ---- balanced bucket sums (round 5) ---------------------------------------------------
// The sorted entries (point order, bucket slot order) cut into equal tasks of
// `task` consecutive entries, one per thread, regardless of bucket
// boundaries — k_seg_sum<true> gave each bucket its own tasks of <= 32, so a
// wave ran 32 iterations for tasks averaging ~22 (random scalars: ~32 entries
// per bucket), ~70 % of its lanes busy. A thread emits one XYZZ partial per
// bucket slot its task touches (divergent stores only: no arithmetic under a
// branch) at pbal[s] + (task - first task of s); k_bal_empty writes the
// infinity of every empty slot; k_seg_sum_xyzz then sums each slot's partials
// (usually 1 or 2) to its Jacobian bucket sum. Group arithmetic is exact, so
// the bucket sums are the same group elements as before.
// (task = entries per thread, host-chosen: kBalTaskMax for large MSMs, fewer
// when that would leave the GPU with too few threads — a small MSM's time is
// one thread's serial chain of additions)
constexpr uint32_t kBalTaskMax = 64;
// partials of slot s: one per task its entries touch (an empty slot: 1, its infinity)
__global__ __launch_bounds__(kBlock) void k_bal_counts(const uint32_t* __restrict__ cnt, uint64_t nseg, uint32_t task,
                                                       uint32_t* __restrict__ counts) {
  const uint64_t s = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
  if (s >= nseg) return;
  const uint32_t a = cnt[s], b = cnt[s + 1];
  counts[s] = a == b ? 1u : (b - 1) / task - a / task + 1;
}
__global__ __launch_bounds__(kBlock) void k_bal_empty(const uint32_t* __restrict__ cnt, uint64_t nseg,
                                                      const uint32_t* __restrict__ pbal, G1XYZZ* __restrict__ out) {
  const uint64_t s = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
  if (s >= nseg) return;
  if (cnt[s] == cnt[s + 1]) out[pbal[s]] = g1x_inf();
}
__global__ __launch_bounds__(kBlock) void k_seg_sum_bal(const G1A* __restrict__ bases, uint64_t nbases,
                                                        const uint32_t* __restrict__ order,
                                                        const uint32_t* __restrict__ cnt, uint64_t nseg, uint32_t total,
                                                        uint32_t tsize, const uint32_t* __restrict__ pbal,
                                                        uint64_t npart, G1XYZZ* __restrict__ out) {
  const uint64_t task = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
  const uint64_t lo = task * tsize;
  if (lo >= total) return;
  const uint32_t hi = (uint32_t)(lo + tsize < total ? lo + tsize : total);
  // the slot holding entry lo: the first s with cnt[s + 1] > lo
  uint64_t L = 0, H = nseg - 1;
  while (L < H) {
    const uint64_t M = (L + H) >> 1;
    if (cnt[M + 1] > lo) H = M;
    else L = M + 1;
  }
  uint64_t s = L;
  uint32_t a = cnt[s], b = cnt[s + 1];
  auto emit = [&](const G1XYZZ& acc) {
    const uint64_t at = pbal[s] + (task - a / tsize);
    ZK_DCHECK(at < npart && at < pbal[s + 1]);
    out[at] = acc;
  };
  G1XYZZ acc = g1x_inf();
  for (uint32_t j = (uint32_t)lo; j < hi; ++j) {
    if (j == b) {  // slot s ends here: its partial, then the next non-empty slot (empty ones: k_bal_empty)
      emit(acc);
      do {
        ++s;
        a = cnt[s];
        b = cnt[s + 1];
      } while (a == b);
      acc = g1x_inf();
    }
    const uint32_t o = order[j];
    ZK_DCHECK((o & 0x7fffffffu) < nbases);
    G1A p = bases[o & 0x7fffffffu];
    if (o >> 31) p.y = fq_neg(p.y);
    acc = g1x_add_mixed(acc, p);
  }
  emit(acc);
}
// sum each slot's XYZZ partials [pbal[s], pbal[s + 1]) -> its Jacobian bucket sum
// (segments longer than a task — skewed scalars — leave partial sums for
// seg_reduce's next levels: out gets one item per task, task_off as k_seg_sum)
__global__ __launch_bounds__(kBlock) void k_seg_sum_xyzz(const G1XYZZ* __restrict__ items, const uint32_t* __restrict__ off,
                                                         const uint32_t* __restrict__ task_off,
                                                         const uint32_t* __restrict__ task_seg, uint32_t ntasks,
                                                         uint32_t task, G1J* __restrict__ out) {
  const uint32_t t = blockIdx.x * kBlock + threadIdx.x;
  if (t >= ntasks) return;
  const uint32_t s = task_seg[t], k = t - task_off[s];
  const uint32_t a = off[s] + k * task, e = off[s + 1];
  const uint32_t b = a + task < e ? a + task : e;
  G1XYZZ acc = g1x_inf();
  for (uint32_t j = a; j < b; ++j) acc = g1x_add(acc, items[j]);
  out[t] = g1x_to_jac(acc);
}

// ---- window reduction -----------------------------------------------------------
// For window w, chunk j of buckets d in [lo, hi): sum_d d B_d = u + lo * T with
// T = sum B_d, u = sum (d - lo) B_d (running sum from the top), at
// out[w (chunks + 1) + j]; W more threads put 2^c B_0 (bucket 0 holds the
// digits of magnitude 2^c, signed_digits) at out[w (chunks + 1) + chunks].
__global__ __launch_bounds__(kBlock) void k_window_chunks(const G1J* __restrict__ buckets, uint32_t c, uint32_t W,
                                                          uint32_t bchunk, G1J* __restrict__ out) {
  const uint32_t chunks = (1u << c) / bchunk;
  const uint32_t g = blockIdx.x * kBlock + threadIdx.x;
  if (g >= W * (chunks + 1)) return;
  if (g >= W * chunks) {
    const uint32_t w = g - W * chunks;
    G1J z = buckets[(uint64_t)w << c];
    for (uint32_t k = 0; k < c; ++k) z = g1_dbl(z);
    out[w * (chunks + 1) + chunks] = z;
    return;
  }
  const uint32_t w = g / chunks, j = g % chunks, lo = j * bchunk, hi = lo + bchunk;
  const G1J* B = buckets + ((uint64_t)w << c);
  G1J t = g1_inf(), u = g1_inf();
  for (uint32_t d = hi; d-- > lo;) {
    ZK_DCHECK(bucket_slot(d, c) < (1u << c));
    t = g1_add(t, B[bucket_slot(d, c)]);
    if (d > lo) u = g1_add(u, t);
  }
  out[w * (chunks + 1) + j] = lo ? g1_add(u, g1_mul_small(t, lo)) : u;  // d = 0 (lo = 0) has weight 0 here
}

// the window sums: nseg segments of exactly len consecutive Jacobian points,
// `task` points per thread per level; out[s olen + k] = the sum of points
// [k task, min((k + 1) task, len)) of segment s, olen = ceil(len / task).
// The sizes are known on the host, so the levels need no scan and no sync.
__global__ __launch_bounds__(kBlock) void k_sum_uniform(const G1J* __restrict__ in, uint32_t len, uint32_t nseg,
                                                        uint32_t task, G1J* __restrict__ out) {
  const uint64_t t = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
  const uint32_t olen = (len + task - 1) / task;
  if (t >= (uint64_t)nseg * olen) return;
  const uint32_t s = (uint32_t)(t / olen), k = (uint32_t)(t % olen);
  const uint64_t a = (uint64_t)s * len + (uint64_t)k * task;
  const uint64_t e = (uint64_t)s * len + ((k + 1) * task < len ? (k + 1) * task : len);
  G1J acc = g1_inf();
  for (uint64_t j = a; j < e; ++j) acc = g1_add(acc, in[j]);
  out[t] = acc;
}

// ---- fixed-base scalar multiplication (Lagrange basis setup) ----------------------
// 16-bit windows: table16[w * 65536 + d] = d * 2^(16w) * G (affine), built on
// the device from the 8-bit table (one mixed addition per entry, then one
// batch normalisation); the setup's table20 is built from it (16-bit windows
// took 16 mixed additions per point: 60.2 ms at 2^24 against 52.4 ms for 13)
constexpr uint32_t kFB16 = 65536;
__global__ __launch_bounds__(kBlock) void k_table16(const G1A* __restrict__ t8, G1J* __restrict__ out) {
  const uint64_t stride = (uint64_t)gridDim.x * kBlock;
  for (uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x; i < 16ull * kFB16; i += stride) {
    const uint32_t w = (uint32_t)(i >> 16), d = (uint32_t)i & 0xffffu;
    out[i] = g1_add_mixed(g1_from_affine(t8[(2 * w) * 256 + (d & 0xffu)]), t8[(2 * w + 1) * 256 + (d >> 8)]);
  }
}
// 20-bit signed windows (round 4): table20[w * 2^19 + j] = m * 2^(20w) * G with
// m = j (j >= 1) or 2^19 (j = 0), the magnitudes of signed_digits(c = 20, W =
// 13); built from table16 with one mixed addition per entry (a 20-bit range at
// bit 20w spans at most two 16-bit windows: 20w mod 16 is 0, 4, 8 or 12; the
// top window's entries are exact for m < 2^16 — a scalar below 2^255, as every
// canonical Fr is, gives it magnitudes <= 2^15).
// out[i] = scalars[i] * G (canonical scalars) with 13 mixed additions instead of 16.
constexpr uint32_t kFB20 = 1u << 19, kFB20W = 13;
__global__ __launch_bounds__(kBlock) void k_table20(const G1A* __restrict__ t16, G1J* __restrict__ out) {
  const uint64_t stride = (uint64_t)gridDim.x * kBlock;
  for (uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x; i < (uint64_t)kFB20W * kFB20; i += stride) {
    const uint32_t w = (uint32_t)(i >> 19), j = (uint32_t)i & (kFB20 - 1u), m = j ? j : kFB20;
    const uint32_t k = 20 * w / 16, o = 20 * w % 16;
    ZK_DCHECK(k < 16 && ((uint64_t)(j ? j : kFB20) << o) < (1ull << 32));
    const uint64_t x = (uint64_t)m << o;  // < 2^32: its low and high 16 bits
    const G1A hi = k + 1 < 16 ? t16[(uint64_t)(k + 1) * kFB16 + (uint32_t)(x >> 16)] : G1A{fq_zero(), fq_zero()};
    out[i] = g1_add_mixed(g1_from_affine(t16[(uint64_t)k * kFB16 + (uint32_t)(x & 0xffffu)]), hi);
  }
}
__global__ __launch_bounds__(kBlock) void k_fixed_base20(const G1A* __restrict__ table, const Fe* __restrict__ scalars,
                                                         uint64_t n, G1J* __restrict__ out) {
  const uint64_t stride = (uint64_t)gridDim.x * kBlock;
  for (uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += stride) {
    G1XYZZ acc = g1x_inf();
    signed_digits(ld_fe(scalars, i), 20, kFB20W, [&](uint32_t w, uint32_t key, uint32_t neg) {
      ZK_DCHECK(w < kFB20W && key < kFB20);
      G1A p = table[(uint64_t)w * kFB20 + key];
      if (neg) p.y = fq_neg(p.y);
      acc = g1x_add_mixed(acc, p);
    });
    out[i] = g1x_to_jac(acc);
  }
}

// small setups (round 5): out[i] = scalars[i] * G from the 8-bit table
// (t8[w * 256 + d] = d 2^(8w) G, 32 windows, 786 KB): 32 mixed additions per
// point, no 654 MB table20 for a handful of basis points
__global__ __launch_bounds__(kBlock) void k_fixed_base8(const G1A* __restrict__ t8, const Fe* __restrict__ scalars,
                                                        uint64_t n, G1J* __restrict__ out) {
  const uint64_t stride = (uint64_t)gridDim.x * kBlock;
  for (uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += stride) {
    const Fe s = ld_fe(scalars, i);
    G1XYZZ acc = g1x_inf();
    for (uint32_t w = 0; w < 32; ++w) {
      const uint32_t d = (fe_word(s, w >> 2) >> (8 * (w & 3))) & 0xffu;
      ZK_DCHECK(w * 256 + d < 32u * 256u);
      if (d) acc = g1x_add_mixed(acc, t8[w * 256 + d]);
    }
    out[i] = g1x_to_jac(acc);
  }
}

// eq(taus, i) over n variables, MSB first (get_lagrange_basis's scalars, kzg.rs:183-206); canonical out
template <class F>
__global__ __launch_bounds__(kBlock) void k_eq_scalars(const Fe* __restrict__ taus, uint32_t nv, uint64_t count,
                                                       Fe* __restrict__ out) {
  const uint64_t stride = (uint64_t)gridDim.x * kBlock;
  const Fe one = fe_one<F>();
  for (uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x; i < count; i += stride) {
    Fe e = one;
    for (uint32_t k = 0; k < nv; ++k) {
      const Fe tk = ld_fe(taus, k);
      e = fe_mul<F>(e, ((i >> (nv - 1 - k)) & 1) ? tk : fe_sub<F>(one, tk));
    }
    st_fe(out, i, fe_from_mont<F>(e));
  }
}

// Jacobian -> affine, `batch` (<= kBatchNorm) points per thread sharing one inversion
// (Montgomery's trick); the prefix products are parked in out[].x until the
// backward pass overwrites them; infinity stays (0, 0)
constexpr uint32_t kBatchNorm = 64;  // (host: fewer for small sets, the inversion is a serial chain)
__global__ __launch_bounds__(kBlock) void k_batch_normalize(const G1J* __restrict__ in, uint64_t n, uint32_t batch,
                                                            G1A* __restrict__ out) {
  const uint64_t t = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
  const uint64_t a = t * batch;
  if (a >= n) return;
  const uint32_t m = (uint32_t)(n - a < batch ? n - a : batch);
  Fq acc = fq_one();
  for (uint32_t k = 0; k < m; ++k) {
    out[a + k].x = acc;  // product of the nonzero Z's before k
    const Fq z = in[a + k].Z;
    if (!fq_is_zero(z)) acc = fq_mul(acc, z);
  }
  Fq inv = fq_inv(acc);  // (prod Z)^-1
  for (uint32_t k = m; k-- > 0;) {
    const G1J p = in[a + k];
    if (fq_is_zero(p.Z)) {
      out[a + k] = {fq_zero(), fq_zero()};
      continue;
    }
    const Fq zi = fq_mul(inv, out[a + k].x);
    inv = fq_mul(inv, p.Z);
    out[a + k] = g1_to_affine_zi(p, zi);
  }
}

// suffix basis: out[j] = in[j] + in[j + half], Jacobian in and out (every
// level is normalised afterwards in one batch)
__global__ __launch_bounds__(kBlock) void k_pair_sum(const G1J* __restrict__ in, uint64_t half, G1J* __restrict__ out) {
  const uint64_t stride = (uint64_t)gridDim.x * kBlock;
  for (uint64_t j = (uint64_t)blockIdx.x * kBlock + threadIdx.x; j < half; j += stride)
    out[j] = g1_add(in[j], in[j + half]);
}

// KZG quotient of the top variable: q[j] = f[j + half] - f[j] (get_quotient, kzg.rs:150-161)
template <class F>
__global__ __launch_bounds__(kBlock) void k_top_diff(const Fe* __restrict__ f, uint64_t half, Fe* __restrict__ q) {
  const uint64_t stride = (uint64_t)gridDim.x * kBlock;
  for (uint64_t j = (uint64_t)blockIdx.x * kBlock + threadIdx.x; j < half; j += stride)
    st_fe(q, j, fe_sub<F>(ld_fe(f, j + half), ld_fe(f, j)));
}
// f - v (poly_minus_v, kzg.rs:65-70)
template <class F>
__global__ __launch_bounds__(kBlock) void k_sub_const(const Fe* __restrict__ f, uint64_t n, Fe v, Fe* __restrict__ out) {
  const uint64_t stride = (uint64_t)gridDim.x * kBlock;
  for (uint64_t j = (uint64_t)blockIdx.x * kBlock + threadIdx.x; j < n; j += stride)
    st_fe(out, j, fe_sub<F>(ld_fe(f, j), v));
}

}  // namespace zk
