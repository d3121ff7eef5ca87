// Multilinear KZG over BLS12-381 G1: host driver and C ABI.
#include <array>
#include <map>
#include <mutex>
#include <thread>

#include "host.hpp"
#include "msm.hpp"
#include "pairing.hpp"

using namespace zkh;

// a KZG setup: the Lagrange basis over the last v taus for v = 0..nv, affine
// Montgomery on the device (bases[nv] is get_lagrange_basis's output), and the
// G2 taus tau_i * G2 (run_trusted_setup :43-46) on the host, for verify
struct zk_kzg {
  uint32_t nv = 0;
  int device = 0;
  DevBuf basis;  // affine Lagrange bases of every suffix level v = 0..nv, level v at offset 2^v - 1
  std::vector<zk::G2A> g2_taus;
  const zk::G1A* level(uint32_t v) const { return reinterpret_cast<const zk::G1A*>(basis.p) + (((uint64_t)1 << v) - 1); }
  ~zk_kzg() { basis.release(); }
};


namespace {
// ---------------------------------------------------------------------------
// KZG over BLS12-381 G1 (pcs/src/kzg_pcs/kzg.rs). Kernels in
// msm.hpp. Scalars are BLS12-381 Fr (the field the reference's KZG is used
// with, gkr_protocol.rs:360); points cross the ABI as canonical affine (x, y)
// of 48-byte LE coordinates, (0, 0) for the point at infinity.
// ---------------------------------------------------------------------------
using zk::Fq;
using zk::G1A;
using zk::G1J;
using Fr381 = zk::Bls12_381Fr;

template <class T>
T* dptr(DevBuf& b) {
  return reinterpret_cast<T*>(b.p);
}

// exclusive scan of n u32 in place
void scan_u32(zk_ctx* c, uint32_t* a, uint64_t n, int depth = 0) {
  const uint64_t nb = (n + zk::kScanBlock - 1) / zk::kScanBlock;
  if (nb <= 1) {
    launch(c, ZK_K_MSM, 8.0 * n, 0, zk::k_scan_block, 1u, a, n, (uint32_t*)nullptr);
    return;
  }
  require(depth < 4, "scan too large");
  DevBuf& sums = c->scan_tmp[depth];
  sums.ensure(nb * 4);
  launch(c, ZK_K_MSM, 8.0 * n, 0, zk::k_scan_block, (uint32_t)nb, a, n, dptr<uint32_t>(sums));
  scan_u32(c, dptr<uint32_t>(sums), nb, depth + 1);
  launch(c, ZK_K_MSM, 8.0 * n, 0, zk::k_scan_add, (uint32_t)((n + zk::kBlock - 1) / zk::kBlock), a, n,
         (const uint32_t*)dptr<uint32_t>(sums));
}

uint32_t blocks_for(uint64_t n) { return (uint32_t)std::max<uint64_t>(1, (n + zk::kBlock - 1) / zk::kBlock); }

// Sum each segment s = items [off[s], off[s+1]) (device u32 offsets, nseg + 1).
// Level 0 reads affine bases[order[j]] (order != null) or Jacobian items0[j].
// Uses c->msm[pool .. pool+4]; returns a device pointer to nseg sums.
G1J* seg_reduce(zk_ctx* c, const G1A* bases, uint64_t nbases, const uint32_t* order, const G1J* items0,
                const uint32_t* off, uint64_t nseg, int pool, const zk::G1XYZZ* xitems0 = nullptr,
                uint32_t task = zk::kSegTask) {
  const G1J* items = items0;
  bool gather = order != nullptr;
  bool xyzz = xitems0 != nullptr;  // level 0 sums XYZZ partials (k_seg_sum_xyzz)
  const uint32_t* cur_off = off;
  int flip = 0;
  for (int level = 0;; ++level) {
    require(level < 64, "segmented reduction did not converge");  // (task >= 2: <= 32 levels for 2^32 items)
    DevBuf& toff = c->msm[pool + flip];
    DevBuf& tseg = c->msm[pool + 2];
    DevBuf& part = c->msm[pool + 3 + flip];
    toff.ensure((nseg + 1) * 4);
    uint32_t* to = dptr<uint32_t>(toff);
    launch(c, ZK_K_MSM, 12.0 * nseg, 0, zk::k_seg_task_counts, blocks_for(nseg), cur_off, nseg, task, to);
    HIPCK(hipMemsetAsync(to + nseg, 0, 4, c->stream));
    scan_u32(c, to, nseg + 1);
    uint32_t total = 0;
    HIPCK(hipMemcpyAsync(&total, to + nseg, 4, hipMemcpyDeviceToHost, c->stream));
    sync(c);
    tseg.ensure((size_t)total * 4);
    launch(c, ZK_K_MSM, 4.0 * total, 0, zk::k_seg_task_owner, blocks_for(nseg), (const uint32_t*)to, nseg, total,
           dptr<uint32_t>(tseg));
    part.ensure((size_t)total * sizeof(G1J));
    if (xyzz)
      launch(c, ZK_K_MSM, 0, 0, zk::k_seg_sum_xyzz, blocks_for(total), xitems0, cur_off, (const uint32_t*)to,
             (const uint32_t*)dptr<uint32_t>(tseg), total, task, dptr<G1J>(part));
    else if (gather)
      launch(c, ZK_K_MSM, 0, 0, zk::k_seg_sum<true>, blocks_for(total), bases, nbases, order, (const G1J*)nullptr, cur_off,
             (const uint32_t*)to, (const uint32_t*)dptr<uint32_t>(tseg), total, task, dptr<G1J>(part));
    else
      launch(c, ZK_K_MSM, 0, 0, zk::k_seg_sum<false>, blocks_for(total), (const G1A*)nullptr, (uint64_t)0,
             (const uint32_t*)nullptr, items, cur_off, (const uint32_t*)to, (const uint32_t*)dptr<uint32_t>(tseg),
             total, task, dptr<G1J>(part));
    if (total == nseg) return dptr<G1J>(part);
    items = dptr<G1J>(part);
    cur_off = to;
    gather = false;
    xyzz = false;
    flip ^= 1;
  }
}

// fn(0 .. n-1) on up to kHostThreads host threads (the box gives a GPU 16
// CPUs): independent chains of host group operations — Horners over window
// sums, G2 scalar multiplications. A thread that cannot be created leaves its
// share to the calling thread; every thread started is joined.
constexpr uint32_t kHostThreads = 16;
template <class Fn>
void host_parallel(uint32_t n, Fn&& fn) {
  const uint32_t nth = std::min<uint32_t>(n, kHostThreads);
  if (nth <= 1) {
    for (uint32_t i = 0; i < n; ++i) fn(i);
    return;
  }
  auto work = [&](uint32_t w) {
    for (uint32_t i = w; i < n; i += nth) fn(i);
  };
  std::vector<std::thread> pool;
  std::vector<uint32_t> mine;
  pool.reserve(nth);
  mine.reserve(nth);
  mine.push_back(0);
  for (uint32_t w = 1; w < nth; ++w) {
    try {
      pool.emplace_back(work, w);
    } catch (...) {
      mine.push_back(w);
    }
  }
  for (uint32_t w : mine) work(w);
  for (auto& th : pool) th.join();
}

// a small MSM's time is one thread's serial chain of group additions: the
// per-thread work of the bucket and window sums shrinks until at least this
// many threads run (2 waves per SIMD of a 256-CU MI355X)
constexpr uint64_t kMsmMinThreads = 1u << 17;

// window width of a c-bit signed-digit Pippenger (msm_g1_device). The window
// sums cost ~0.9-2 ns per bucket against ~0.21 ns per bucket-sum entry (round 5
// rocprof of get_proof's MSMs): kBucketCost 5.
constexpr double kBucketCost = 5.0;
// levels > 0: `levels` level-batched MSMs of 1, 2, 4, ... points (n = 2^levels - 1),
// each with its own windows: the window sums cost levels times as much.
inline uint32_t msm_window_bits(uint64_t n, uint32_t lg, uint32_t levels = 0) {
  if (const char* e = getenv("ZK_MSM_C")) {  // (diagnostic) a fixed width, 6..20
    const uint32_t f = (uint32_t)strtoul(e, nullptr, 0);
    if (f >= 6 && f <= 20) return f;
  }
  if (lg < 12 && levels == 0) return std::min<uint32_t>(20, std::max<uint32_t>(6, lg > 9 ? lg - 3 : 6));
  uint32_t best = 0;
  double best_cost = 1e300;
  for (uint32_t cc : {6u, 8u, 10u, 13u, 16u, 20u}) {
    const uint32_t W = (256 + cc - 1) / cc, bb = (256 + W - 1) / W - 1;
    const uint32_t Wt = levels ? levels * W : W;
    if ((uint64_t)Wt << (bb - zk::sort_fine_bits(bb)) > zk::kSortBinsMax) continue;  // the sort's coarse bins
    if (levels == 0 && cc == 6) continue;  // (single MSMs of 2^12+ points: 8 bits and up)
    const double cost = (double)n * W + kBucketCost * Wt * (double)(1ull << bb);
    if (cost < best_cost) {
      best_cost = cost;
      best = cc;
    }
  }
  if (!best) fail(ZK_EINVAL, "internal: no MSM window width fits the sort's bins");
  return best;
}

// The window sums of a c-bit signed-digit Pippenger of sum_i scalars[i] *
// bases[i] (scalars canonical Fr, bases affine Montgomery, both on the
// device): W windows of cb bits, or with levels > 0 the levels x W window sums
// of `levels` level-batched MSMs (n = 2^levels - 1: level v = points
// [2^v - 1, 2^(v+1) - 1), window v W + w) in one pass.
std::vector<G1J> msm_window_sums(zk_ctx* c, const G1A* bases, const Fe* scalars, uint64_t n, uint32_t levels,
                                 uint32_t& W_out, uint32_t& cb_out) {
  using namespace zk;
  require(n > 0 && n < (1ull << 28), "MSM too large");
  uint32_t lg = 0;
  while ((2ull << lg) <= n) ++lg;
  // c-bit signed digits (msm.hpp signed_digits): W c >= 256, 2^(c-1) buckets per window.
  // Small MSMs: c = log2 n - 3 in [6, 20], evened out over its W windows.
  // From 2^12 points (c_msm_bits): the width among 8, 10, 13, 16, 20 bits —
  // the ones whose top window keeps >= 6 bits (19, 18, 15, 14 leave 9, 4, 1, 4:
  // a sliver sends every point to a handful of buckets, whose long segments
  // take extra reduction levels) — that minimises n W + kBucketCost W 2^(c-1)
  // (bucket additions against the window sums' per-bucket cost).
  const uint32_t c0 = msm_window_bits(n, lg, levels);
  const uint32_t W = (256 + c0 - 1) / c0;
  const uint32_t cb = (256 + W - 1) / W;
  const uint32_t bb = cb - 1;  // bucket key bits
  const uint32_t Wt = levels ? levels * W : W;  // windows of the pass
  const uint64_t nb = (uint64_t)Wt << bb;
  W_out = W;
  cb_out = cb;
  require((uint64_t)n * W < (1ull << 32), "MSM too large");  // u32 entry offsets
  DevBuf& cnt = c->msm[10];
  DevBuf& cur = c->msm[11];
  DevBuf& ord = c->msm[12];
  cnt.ensure((nb + 1) * 4);
  ord.ensure(std::max<uint64_t>(1, n * W) * 4);
  {  // bucket sort (msm.hpp k_sort_hist / k_sort_scatter / k_sort_fine)
    const uint32_t C = bb - sort_fine_bits(bb), nbin = Wt << C;
    require(nbin <= kSortBinsMax, "internal: MSM coarse bins exceed the LDS table");
    const uint32_t pts = sort_block_pts(n);
    const uint32_t NB = (uint32_t)((n + pts - 1) / pts);
    const uint64_t nh = (uint64_t)nbin * NB + 1;
    cur.ensure(nh * 4);
    DevBuf& ent = c->msm[16];
    ent.ensure(std::max<uint64_t>(1, n * W) * 8);
    HIPCK(hipMemsetAsync(cur.p, 0, nh * 4, c->stream));
    const bool big = nbin > kSortBinsSingle;  // (the level-batched pass's larger LDS table)
    if (big)
      launch(c, ZK_K_MSM, 32.0 * n, 0, k_sort_hist<kSortBinsMax>, NB, scalars, n, cb, W, levels, NB, pts,
             dptr<uint32_t>(cur));
    else
      launch(c, ZK_K_MSM, 32.0 * n, 0, k_sort_hist<kSortBinsSingle>, NB, scalars, n, cb, W, levels, NB, pts,
             dptr<uint32_t>(cur));
    scan_u32(c, dptr<uint32_t>(cur), nh);
    if (big)
      launch(c, ZK_K_MSM, 32.0 * n, 0, k_sort_scatter<kSortBinsMax>, NB, scalars, n, cb, W, levels, NB, pts,
             (const uint32_t*)dptr<uint32_t>(cur), dptr<uint64_t>(ent));
    else
      launch(c, ZK_K_MSM, 32.0 * n, 0, k_sort_scatter<kSortBinsSingle>, NB, scalars, n, cb, W, levels, NB, pts,
             (const uint32_t*)dptr<uint32_t>(cur), dptr<uint64_t>(ent));
    launch(c, ZK_K_MSM, 0, 0, k_sort_fine, nbin, (const uint64_t*)dptr<uint64_t>(ent), bb, NB,
           (const uint32_t*)dptr<uint32_t>(cur), dptr<uint32_t>(cnt), dptr<uint32_t>(ord));
  }
  // bucket sums (mixed additions of the gathered affine bases): balanced tasks
  // of kBalTask entries across bucket boundaries, one XYZZ partial per bucket
  // a task touches, then each bucket's partials summed (msm.hpp "balanced")
  G1J* buckets;
  if (c->msm_balanced) {
    DevBuf& bc = c->msm[17];
    bc.ensure((nb + 1) * 4);
    uint32_t* pbal = dptr<uint32_t>(bc);
    // entries per thread: kBalTaskMax unless that leaves fewer than ~2 waves per SIMD
    uint32_t tsize = kBalTaskMax;
    while (tsize > 4 && (uint64_t)n * W / tsize < kMsmMinThreads) tsize >>= 1;
    launch(c, ZK_K_MSM, 12.0 * nb, 0, k_bal_counts, blocks_for(nb), (const uint32_t*)dptr<uint32_t>(cnt), nb, tsize,
           pbal);
    HIPCK(hipMemsetAsync(pbal + nb, 0, 4, c->stream));
    scan_u32(c, pbal, nb + 1);
    uint32_t sizes[2] = {0, 0};  // entries, partials
    HIPCK(hipMemcpyAsync(&sizes[0], dptr<uint32_t>(cnt) + nb, 4, hipMemcpyDeviceToHost, c->stream));
    HIPCK(hipMemcpyAsync(&sizes[1], pbal + nb, 4, hipMemcpyDeviceToHost, c->stream));
    sync(c);
    DevBuf& pb = c->msm[18];
    pb.ensure(std::max<uint64_t>(1, sizes[1]) * sizeof(G1XYZZ));
    G1XYZZ* parts = dptr<G1XYZZ>(pb);
    launch(c, ZK_K_MSM, 0, 0, k_bal_empty, blocks_for(nb), (const uint32_t*)dptr<uint32_t>(cnt), nb,
           (const uint32_t*)pbal, parts);
    const uint64_t ntask = ((uint64_t)sizes[0] + tsize - 1) / tsize;
    if (ntask)
      launch(c, ZK_K_MSM, 0, 0, k_seg_sum_bal, blocks_for(ntask), bases, n, (const uint32_t*)dptr<uint32_t>(ord),
             (const uint32_t*)dptr<uint32_t>(cnt), nb, sizes[0], tsize, (const uint32_t*)pbal, (uint64_t)sizes[1],
             parts);
    uint32_t ptask = kSegTask;  // partials per thread: fewer for small MSMs (serial chains)
    while (ptask > 2 && sizes[1] / ptask < kMsmMinThreads) ptask >>= 1;
    buckets = seg_reduce(c, nullptr, 0, nullptr, nullptr, pbal, nb, 0, parts, ptask);
  } else {
    buckets = seg_reduce(c, bases, n, dptr<uint32_t>(ord), nullptr, dptr<uint32_t>(cnt), nb, 0);
  }
  // per window: sum_d d B_d over chunks of buckets, then over the chunks
  uint32_t bchunk = kBucketChunkMax;  // buckets per thread: fewer when the windows are small (thread count)
  while (bchunk > 1 && ((uint64_t)Wt << bb) / bchunk < kMsmMinThreads) bchunk >>= 1;
  const uint32_t chunks = (1u << bb) / bchunk;
  DevBuf& chb = c->msm[13];
  chb.ensure((size_t)Wt * (chunks + 1) * sizeof(G1J));
  launch(c, ZK_K_MSM, 0, 0, k_window_chunks, blocks_for((uint64_t)Wt * (chunks + 1)), (const G1J*)buckets, bb, Wt,
         bchunk, dptr<G1J>(chb));
  // the W window sums: equal segments of chunks + 1 points, reduced in levels
  // of msm_win_task points per thread (short tasks keep every level parallel;
  // the sizes are known here, so no scans and no host syncs)
  const G1J* ws = dptr<G1J>(chb);
  {
    uint32_t len = chunks + 1;
    const uint32_t task = std::max<uint32_t>(2, c->msm_win_task);
    int flip = 0;
    while (len > 1) {
      const uint32_t olen = (len + task - 1) / task;
      DevBuf& ob = c->msm[5 + flip];
      ob.ensure((size_t)Wt * olen * sizeof(G1J));
      launch(c, ZK_K_MSM, 0, 0, k_sum_uniform, blocks_for((uint64_t)Wt * olen), ws, len, Wt, task, dptr<G1J>(ob));
      ws = dptr<G1J>(ob);
      len = olen;
      flip ^= 1;
    }
  }
  std::vector<G1J> S(Wt);
  HIPCK(hipMemcpyAsync(S.data(), ws, Wt * sizeof(G1J), hipMemcpyDeviceToHost, c->stream));
  sync(c);
  return S;
}

// Horner over W windows of cb bits on the host: sum_w 2^(cb w) S[w]
G1J windows_horner(const G1J* S, uint32_t W, uint32_t cb) {
  using namespace zk;
  G1J R = S[W - 1];
  for (uint32_t w = W - 1; w-- > 0;) {
    for (uint32_t k = 0; k < cb; ++k) R = g1_dbl(R);
    R = g1_add(R, S[w]);
  }
  return R;
}

// sum_i scalars[i] * bases[i]; scalars canonical Fr (device), bases affine Montgomery (device)
G1J msm_g1_device(zk_ctx* c, const G1A* bases, const Fe* scalars, uint64_t n) {
  if (n == 0) return zk::g1_inf();
  uint32_t W = 0, cb = 0;
  const std::vector<G1J> S = msm_window_sums(c, bases, scalars, n, 0, W, cb);
  return windows_horner(S.data(), W, cb);
}

// `levels` MSMs in one pass: out[v] = sum over points [2^v - 1, 2^(v+1) - 1)
// (level v: 2^v points) of scalars[i] * bases[i] — kzg_get_proof's small
// quotient commitments against the setup's suffix bases, which it stores in
// exactly this layout (zk_kzg::level)
std::vector<G1J> msm_levels(zk_ctx* c, const G1A* bases, const Fe* scalars, uint32_t levels) {
  uint32_t W = 0, cb = 0;
  const std::vector<G1J> S = msm_window_sums(c, bases, scalars, ((uint64_t)1 << levels) - 1, levels, W, cb);
  std::vector<G1J> out(levels);
  // each level's Horner is a serial chain of ~W cb host doublings (250 at 20
  // levels of 10-bit windows): the levels run on host threads
  host_parallel(levels, [&](uint32_t v) { out[v] = windows_horner(S.data() + (size_t)v * W, W, cb); });
  return out;
}

// batch Jacobian -> affine on the host (Montgomery's trick)
std::vector<G1A> host_normalize(const std::vector<G1J>& pts) {
  using namespace zk;
  std::vector<Fq> pre(pts.size());
  Fq acc = fq_one();
  for (size_t i = 0; i < pts.size(); ++i) {
    pre[i] = acc;
    if (!g1_is_inf(pts[i])) acc = fq_mul(acc, pts[i].Z);
  }
  Fq inv = fq_inv(acc);
  std::vector<G1A> out(pts.size());
  for (size_t i = pts.size(); i-- > 0;) {
    if (g1_is_inf(pts[i])) {
      out[i] = {fq_zero(), fq_zero()};
      continue;
    }
    out[i] = g1_to_affine_zi(pts[i], fq_mul(inv, pre[i]));
    inv = fq_mul(inv, pts[i].Z);
  }
  return out;
}

G1A g1_generator() {
  Fq x, y;
  memcpy(x.v, zk::kG1GenX, 48);
  memcpy(y.v, zk::kG1GenY, 48);
  return {zk::fq_to_mont(x), zk::fq_to_mont(y)};
}

// table[w * 256 + d] = d * 2^(8w) * G, affine on the device (built once per ctx)
const G1A* g1_fixed_table(zk_ctx* c) {
  using namespace zk;
  if (c->g1_table.p) return dptr<G1A>(c->g1_table);
  std::vector<G1J> t(32 * 256, g1_inf());
  G1J gw = g1_from_affine(g1_generator());
  for (int w = 0; w < 32; ++w) {
    for (int d = 1; d < 256; ++d) t[w * 256 + d] = d == 1 ? gw : g1_add(t[w * 256 + d - 1], gw);
    for (int k = 0; k < 8; ++k) gw = g1_dbl(gw);
  }
  const std::vector<G1A> a = host_normalize(t);
  c->g1_table.ensure(a.size() * sizeof(G1A));
  HIPCK(hipMemcpyAsync(c->g1_table.p, a.data(), a.size() * sizeof(G1A), hipMemcpyHostToDevice, c->stream));
  sync(c);
  return dptr<G1A>(c->g1_table);
}

// table16[w * 65536 + d] = d * 2^(16w) * G, affine on the device (built once per ctx
// from the 8-bit table: 2^20 mixed additions and one batch normalisation)
const G1A* g1_fixed_table16(zk_ctx* c) {
  using namespace zk;
  if (c->g1_table16.p) return dptr<G1A>(c->g1_table16);
  const G1A* t8 = g1_fixed_table(c);
  const uint64_t n = 16ull * kFB16;
  ScopedBuf jac;
  jac.b.ensure(n * sizeof(G1J));
  launch(c, ZK_K_MSM, 0, 0, k_table16, grid_for(c, n, k_table16), t8, dptr<G1J>(jac.b));
  c->g1_table16.ensure(n * sizeof(G1A));
  launch(c, ZK_K_MSM, 240.0 * n, 0, k_batch_normalize, blocks_for((n + kBatchNorm - 1) / kBatchNorm),
         (const G1J*)dptr<G1J>(jac.b), n, kBatchNorm, dptr<G1A>(c->g1_table16));
  sync(c);
  return dptr<G1A>(c->g1_table16);
}

// table20[w * 2^19 + j]: the 13 signed 20-bit windows' magnitudes (msm.hpp
// k_table20), affine, built from table16 (6.8 M mixed additions, one batch
// normalisation; table16 is released afterwards) ONCE PER DEVICE AND PROCESS:
// every context on the device shares it (654 MB, kept until the process
// exits — it depends on nothing but the curve's generator). Round 4 rebuilt
// it per context (cold setup 125 ms against 76 ms warm).
// zk_kzg_release_fixed_base_cache frees an entry; a setup holds a
// lease on its device's entry (`users`) from the lookup until its fixed-base
// kernel has finished, and a release refuses while one is held.
struct FixedBaseCache {
  std::mutex m;
  std::map<int, void*> table20;  // device -> affine table (until released)
  std::map<int, int> users;      // device -> setups using the table now
};
FixedBaseCache& fixed_base_cache() {
  static FixedBaseCache* cache = new FixedBaseCache();  // (leaked on purpose: no teardown order with the HIP runtime)
  return *cache;
}
// (the caller holds a lease: FixedBaseLease)
const G1A* g1_fixed_table20(zk_ctx* c) {
  using namespace zk;
  FixedBaseCache& fc = fixed_base_cache();
  std::lock_guard<std::mutex> lock(fc.m);
  auto it = fc.table20.find(c->device);
  if (it != fc.table20.end()) return static_cast<const G1A*>(it->second);
  const G1A* t16 = g1_fixed_table16(c);
  const uint64_t n = (uint64_t)kFB20W * kFB20;
  ScopedBuf jac;
  jac.b.ensure(n * sizeof(G1J));
  launch(c, ZK_K_MSM, 0, 0, k_table20, grid_for(c, n, k_table20), t16, dptr<G1J>(jac.b));
  DevBuf t20;  // owned by the cache once built
  t20.ensure(n * sizeof(G1A));
  try {
    launch(c, ZK_K_MSM, 240.0 * n, 0, k_batch_normalize, blocks_for((n + kBatchNorm - 1) / kBatchNorm),
           (const G1J*)dptr<G1J>(jac.b), n, kBatchNorm, dptr<G1A>(t20));
    sync(c);
  } catch (...) {
    t20.release();
    throw;
  }
  c->g1_table16.release();
  fc.table20[c->device] = t20.p;
  return dptr<G1A>(t20);
}
struct FixedBaseLease {  // a setup's use of its device's table20 (see FixedBaseCache)
  zk_ctx* c;
  int device;
  explicit FixedBaseLease(zk_ctx* cc) : c(cc), device(cc->device) {
    FixedBaseCache& fc = fixed_base_cache();
    std::lock_guard<std::mutex> lock(fc.m);
    fc.users[device] += 1;
  }
  ~FixedBaseLease() {
    (void)hipStreamSynchronize(c->stream);  // (an unwinding setup: its kernel has finished reading the table)
    FixedBaseCache& fc = fixed_base_cache();
    std::lock_guard<std::mutex> lock(fc.m);
    fc.users[device] -= 1;
  }
  FixedBaseLease(const FixedBaseLease&) = delete;
  FixedBaseLease& operator=(const FixedBaseLease&) = delete;
};
// below this many basis points a setup uses the 8-bit table (k_fixed_base8:
// 32 mixed additions per point) instead of building / holding table20
constexpr uint64_t kSetupTable20Min = 1ull << 16;

zk_g1 g1_out(const G1J& p) {
  const G1A a = zk::g1_to_affine(p);
  zk_g1 r;
  const Fq x = zk::fq_from_mont(a.x), y = zk::fq_from_mont(a.y);
  memcpy(r.x, x.v, 48);
  memcpy(r.y, y.v, 48);
  return r;
}
zk_g1 g1a_out(const G1A& a) {
  zk_g1 r;
  const Fq x = zk::g1a_is_inf(a) ? zk::fq_zero() : zk::fq_from_mont(a.x);
  const Fq y = zk::g1a_is_inf(a) ? zk::fq_zero() : zk::fq_from_mont(a.y);
  memcpy(r.x, x.v, 48);
  memcpy(r.y, y.v, 48);
  return r;
}

// caller point (canonical affine, (0, 0) = infinity) -> Montgomery, checked on the curve
G1A parse_g1(const zk_g1& p) {
  Fq x, y;
  memcpy(x.v, p.x, 48);
  memcpy(y.v, p.y, 48);
  require(zk::fq_is_canonical(x) && zk::fq_is_canonical(y), "point coordinate >= modulus");
  if (zk::fq_is_zero(x) && zk::fq_is_zero(y)) return {zk::fq_zero(), zk::fq_zero()};
  const G1A a{zk::fq_to_mont(x), zk::fq_to_mont(y)};
  Fq four = zk::fq_zero();
  four.v[0] = 4;
  const Fq rhs = zk::fq_add(zk::fq_mul(zk::fq_sqr(a.x), a.x), zk::fq_to_mont(four));
  require(zk::fq_eq(zk::fq_sqr(a.y), rhs), "point not on the curve");
  return a;
}

// G2 (canonical affine over Fq2, all zero = infinity) <-> Montgomery, checked on the twist
zk::G2A parse_g2(const zk_g2& p) {
  Fq c[4];
  memcpy(c[0].v, p.x[0], 48);
  memcpy(c[1].v, p.x[1], 48);
  memcpy(c[2].v, p.y[0], 48);
  memcpy(c[3].v, p.y[1], 48);
  bool zero = true;
  for (auto& e : c) {
    require(zk::fq_is_canonical(e), "G2 coordinate >= modulus");
    zero = zero && zk::fq_is_zero(e);
    e = zk::fq_to_mont(e);
  }
  if (zero) return {zk::fq2_zero(), zk::fq2_zero(), true};
  const zk::G2A a{{c[0], c[1]}, {c[2], c[3]}, false};
  require(zk::g2_on_curve(a), "G2 point not on the twist");
  return a;
}
zk_g2 g2_out(const zk::G2A& a) {
  zk_g2 r;
  memset(&r, 0, sizeof r);
  if (a.inf) return r;
  const Fq c[4] = {zk::fq_from_mont(a.x.c0), zk::fq_from_mont(a.x.c1), zk::fq_from_mont(a.y.c0),
                   zk::fq_from_mont(a.y.c1)};
  memcpy(r.x[0], c[0].v, 48);
  memcpy(r.x[1], c[1].v, 48);
  memcpy(r.y[0], c[2].v, 48);
  memcpy(r.y[1], c[3].v, 48);
  return r;
}

// Fr scalar (host, repr) -> canonical little-endian u32 limbs (into_bigint)
void fr_canon(zk_repr repr, const zk_fe& s, uint32_t out[8]) {
  const Fe c = zk::fe_from_mont<Fr381>(in_mont<Fr381>(repr, s));
  memcpy(out, c.v, 32);
}

// G1 affine (Montgomery) of a Jacobian point
G1A g1_affine(const G1J& p) { return zk::g1_to_affine(p); }

// Fr values (host, repr) -> canonical Fr on the device (k_check_canonical + conversion)
void upload_fr_canonical(zk_ctx* c, zk_repr repr, const zk_fe* host, uint64_t n, Fe* dev) {
  upload<Fr381>(c, repr, host, n, dev);  // -> Montgomery, checked < r
  launch(c, ZK_K_CONVERT, 64.0 * n, (double)n, zk::k_convert<Fr381, false>, grid_for(c, n, zk::k_convert<Fr381, false>),
         (const Fe*)dev, dev, n);
}

// kzg_get_proof commits the quotients of its last this many levels (<= 2^20 - 1
// points in all) in one level-batched MSM pass (ZK_PROOF_BATCH_LEVELS: fewer,
// 0 = one MSM per level)
constexpr uint32_t kProofBatchLevelsMax = 20;
uint32_t proof_batch_levels() {
  const char* e = getenv("ZK_PROOF_BATCH_LEVELS");
  const uint32_t x = e ? (uint32_t)strtoul(e, nullptr, 0) : kProofBatchLevelsMax;
  return std::min(x, kProofBatchLevelsMax);
}
#define kProofBatchLevels proof_batch_levels()

G1J kzg_commit_canonical(zk_ctx* c, const zk_kzg* k, uint32_t v, const Fe* scalars) {
  return msm_g1_device(c, k->level(v), scalars, (uint64_t)1 << v);
}

// KZG::get_proof (kzg.rs:59-95): quotient i of (f - v) w.r.t. its top variable,
// committed against the basis of the remaining variables — the same group
// element as the reference's commitment of the blown-up quotient against the
// full basis, since sum_k L_(k, j) over the blown-up top variables is L_j of
// the suffix basis (eq sums to 1) — then fold f by point[i].
void kzg_get_proof(zk_ctx* c, const zk_kzg* k, const Fe* f_mont, const Fe& v_mont, const std::vector<Fe>& point,
                   std::vector<G1J>& out) {
  using namespace zk;
  const uint32_t nv = k->nv;
  const uint64_t N = (uint64_t)1 << nv;
  DevBuf& a = c->msm[15];
  a.ensure(N * 32 + (N / 2 + 1) * 32 * 2);
  Fe* cur = reinterpret_cast<Fe*>(a.p);
  Fe* nxt = cur + N;
  Fe* q = nxt + N / 2;
  launch(c, ZK_K_FOLD, 64.0 * N, 0, k_sub_const<Fr381>, grid_for(c, N, k_sub_const<Fr381>), f_mont, N, v_mont, cur);
  out.assign(nv, g1_inf());
  // the quotients of the last kProofBatchLevels levels (<= 2^19 points each):
  // written at the offsets of their suffix bases and committed together in one
  // level-batched pass (msm_levels) — alone, each small one is a chain of
  // latency-bound launches (1.5-2.7 ms at 2^14 points and fewer)
  const uint32_t nbatch = std::min<uint32_t>(nv, kProofBatchLevels);
  DevBuf& qb = c->msm[8];
  qb.ensure((((uint64_t)1 << nbatch) - 1 + 1) * 32);
  Fe* qall = reinterpret_cast<Fe*>(qb.p);
  for (uint32_t i = 0; i < nv; ++i) {
    const uint32_t m = nv - i;  // variables of cur
    const uint64_t half = (uint64_t)1 << (m - 1);
    const bool batched = m - 1 < nbatch;
    Fe* qi = batched ? qall + (half - 1) : q;
    launch(c, ZK_K_FOLD, 96.0 * half, 0, k_top_diff<Fr381>, grid_for(c, half, k_top_diff<Fr381>), (const Fe*)cur,
           half, qi);
    launch(c, ZK_K_CONVERT, 64.0 * half, (double)half, k_convert<Fr381, false>,
           grid_for(c, half, k_convert<Fr381, false>), (const Fe*)qi, qi, half);
    if (!batched) out[i] = kzg_commit_canonical(c, k, m - 1, q);
    launch(c, ZK_K_FOLD, 96.0 * half, (double)half, k_fold<Fr381>, grid_for(c, half, k_fold<Fr381>), (const Fe*)cur,
           nxt, half, m - 1, point[i]);
    std::swap(cur, nxt);
  }
  if (nbatch) {
    const std::vector<G1J> lv = msm_levels(c, k->level(0), qall, nbatch);
    for (uint32_t v = 0; v < nbatch; ++v) out[nv - 1 - v] = lv[v];  // level v = quotient i = nv - 1 - v
  }
}
}  // namespace

extern "C" {

// ---- KZG over BLS12-381 G1 ----
int zk_kzg_setup(zk_ctx* c, zk_repr repr, const zk_fe* taus, uint32_t nvars, zk_kzg** out) {
  return guarded([&] {
    require(c && taus && out, "null argument");
    require(nvars >= 1, "Invalid num of vars for lagrange basis");  // kzg.rs:184-186
    require(nvars <= 26, "KZG setup too large");
    bind(c);
    *out = nullptr;
    auto k = std::make_unique<zk_kzg>();
    k->nv = nvars;
    k->device = c->device;
    const uint64_t N = (uint64_t)1 << nvars, total = 2 * N - 1;  // every suffix level, level v at 2^v - 1
    const bool big = N >= kSetupTable20Min;
    std::unique_ptr<FixedBaseLease> lease;  // (held until this setup's kernels have finished)
    if (big) lease = std::make_unique<FixedBaseLease>(c);
    const G1A* table = big ? g1_fixed_table20(c) : g1_fixed_table(c);
    DevBuf& tb = c->msm[14];
    tb.ensure(nvars * 32);
    upload<Fr381>(c, repr, taus, nvars, reinterpret_cast<Fe*>(tb.p));
    DevBuf& sc = c->msm[15];
    sc.ensure(N * 32);
    launch(c, ZK_K_MSM, 32.0 * N, (double)N * nvars, zk::k_eq_scalars<Fr381>, grid_for(c, N, zk::k_eq_scalars<Fr381>),
           (const Fe*)tb.p, nvars, N, reinterpret_cast<Fe*>(sc.p));
    // the Jacobian points of every level (released after the normalisation)
    struct Scoped {
      DevBuf b;
      ~Scoped() { b.release(); }
    } jac;
    jac.b.ensure(total * sizeof(G1J));
    G1J* J = dptr<G1J>(jac.b);
    if (big)
      launch(c, ZK_K_MSM, 176.0 * N, 0, zk::k_fixed_base20, grid_for(c, N, zk::k_fixed_base20), table,
             (const Fe*)sc.p, N, J + (N - 1));
    else
      launch(c, ZK_K_MSM, 128.0 * N, 0, zk::k_fixed_base8, grid_for(c, N, zk::k_fixed_base8), table,
             (const Fe*)sc.p, N, J + (N - 1));
    // G2 half of run_trusted_setup (:43-46): tau_i * G2, on the host (nvars
    // scalar multiplications) while the basis kernels run
    // (on up to kHostThreads host threads; the scalars are converted and
    // checked on this thread first, so nothing below can throw)
    {
      const zk::G2J g2 = zk::g2_from_affine(zk::g2_generator());
      std::vector<std::array<uint32_t, 8>> tc(nvars);
      for (uint32_t i = 0; i < nvars; ++i) fr_canon(repr, taus[i], tc[i].data());
      k->g2_taus.resize(nvars);
      host_parallel(nvars, [&](uint32_t i) { k->g2_taus[i] = zk::g2_to_affine(zk::g2_mul(g2, tc[i].data())); });
    }
    // suffix bases L^(v)_j = L^(v+1)_j + L^(v+1)_(2^v + j) (eq sums to 1 over the
    // dropped variable), Jacobian, then ONE batch normalisation of all levels:
    // each normalisation launch carries a serial 381-bit inversion (~1 ms)
    for (uint32_t v = nvars; v-- > 0;) {
      const uint64_t n = (uint64_t)1 << v;
      launch(c, ZK_K_MSM, 432.0 * n, 0, zk::k_pair_sum, grid_for(c, n, zk::k_pair_sum), (const G1J*)(J + (2 * n - 1)),
             n, J + (n - 1));
    }
    k->basis.ensure(total * sizeof(G1A));
    uint32_t nbatch = zk::kBatchNorm;  // (points per inversion: fewer for small setups, whose time is the chain)
    while (nbatch > 1 && total / nbatch < kMsmMinThreads) nbatch >>= 1;
    launch(c, ZK_K_MSM, 240.0 * total, 0, zk::k_batch_normalize, blocks_for((total + nbatch - 1) / nbatch),
           (const G1J*)J, total, nbatch, dptr<G1A>(k->basis));
    sync(c);
    *out = k.release();
  });
}

void zk_kzg_free(zk_kzg* k) {
  if (!k) return;
  (void)hipSetDevice(k->device);
  delete k;
}

int zk_kzg_lagrange_basis(zk_ctx* c, const zk_kzg* k, uint32_t nvars_suffix, zk_g1* out) {
  return guarded([&] {
    require(c && k && out, "null argument");
    require(nvars_suffix <= k->nv, "no such basis");
    bind(c);
    const uint64_t n = (uint64_t)1 << nvars_suffix;
    std::vector<G1A> a(n);
    HIPCK(hipMemcpyAsync(a.data(), k->level(nvars_suffix), n * sizeof(G1A), hipMemcpyDeviceToHost, c->stream));
    sync(c);
    for (uint64_t i = 0; i < n; ++i) out[i] = g1a_out(a[i]);
  });
}

int zk_kzg_commit(zk_ctx* c, const zk_kzg* k, zk_repr repr, const zk_fe* evals, zk_g1* out) {
  return guarded([&] {
    require(c && k && evals && out, "null argument");
    bind(c);
    const uint64_t N = (uint64_t)1 << k->nv;
    c->input.ensure(N * 32);
    upload_fr_canonical(c, repr, evals, N, c->input.fe());
    *out = g1_out(kzg_commit_canonical(c, k, k->nv, c->input.fe()));
  });
}

int zk_dev_kzg_commit(zk_ctx* c, const zk_kzg* k, const void* dev_evals, zk_g1* out) {
  return guarded([&] {
    require(c && k && dev_evals && out, "null argument");
    bind(c);
    const uint64_t N = (uint64_t)1 << k->nv;
    c->input.ensure(N * 32);
    launch(c, ZK_K_CONVERT, 64.0 * N, (double)N, zk::k_convert<Fr381, false>, grid_for(c, N, zk::k_convert<Fr381, false>),
           reinterpret_cast<const Fe*>(dev_evals), c->input.fe(), N);
    *out = g1_out(kzg_commit_canonical(c, k, k->nv, c->input.fe()));
  });
}

int zk_kzg_get_proof(zk_ctx* c, const zk_kzg* k, zk_repr repr, const zk_fe* evals, const zk_fe* opened_value,
                     const zk_fe* point, zk_g1* out) {
  return guarded([&] {
    require(c && k && evals && opened_value && point && out, "null argument");
    bind(c);
    const uint64_t N = (uint64_t)1 << k->nv;
    c->input.ensure(N * 32);
    upload<Fr381>(c, repr, evals, N, c->input.fe());
    std::vector<Fe> pt(k->nv);
    for (uint32_t i = 0; i < k->nv; ++i) pt[i] = in_mont<Fr381>(repr, point[i]);
    std::vector<G1J> q;
    kzg_get_proof(c, k, c->input.fe(), in_mont<Fr381>(repr, *opened_value), pt, q);
    const std::vector<G1A> qa = host_normalize(q);  // (one inversion for all nv points)
    for (uint32_t i = 0; i < k->nv; ++i) out[i] = g1a_out(qa[i]);
  });
}

int zk_dev_kzg_get_proof(zk_ctx* c, const zk_kzg* k, zk_repr repr, const void* dev_evals, const zk_fe* opened_value,
                         const zk_fe* point, zk_g1* out) {
  return guarded([&] {
    require(c && k && dev_evals && opened_value && point && out, "null argument");
    bind(c);
    std::vector<Fe> pt(k->nv);
    for (uint32_t i = 0; i < k->nv; ++i) pt[i] = in_mont<Fr381>(repr, point[i]);
    std::vector<G1J> q;
    kzg_get_proof(c, k, reinterpret_cast<const Fe*>(dev_evals), in_mont<Fr381>(repr, *opened_value), pt, q);
    const std::vector<G1A> qa = host_normalize(q);
    for (uint32_t i = 0; i < k->nv; ++i) out[i] = g1a_out(qa[i]);
  });
}

int zk_kzg_release_fixed_base_cache(int device) {
  return guarded([&] {
    FixedBaseCache& fc = fixed_base_cache();
    std::lock_guard<std::mutex> lock(fc.m);
    int cur = 0;
    HIPCK(hipGetDevice(&cur));
    struct Restore {
      int d;
      ~Restore() { (void)hipSetDevice(d); }
    } restore{cur};
    for (auto it = fc.table20.begin(); it != fc.table20.end();) {
      if (device >= 0 && it->first != device) {
        ++it;
        continue;
      }
      require(fc.users[it->first] == 0, "a KZG setup on this device is using the fixed-base table");
      HIPCK(hipSetDevice(it->first));
      HIPCK(hipFree(it->second));
      it = fc.table20.erase(it);
    }
  });
}

int zk_msm_g1(zk_ctx* c, zk_repr repr, const zk_g1* bases, const zk_fe* scalars, size_t n, zk_g1* out) {
  return guarded([&] {
    require(c && out && (n == 0 || (bases && scalars)), "null argument");
    bind(c);
    std::vector<G1A> b(n);
    for (size_t i = 0; i < n; ++i) b[i] = parse_g1(bases[i]);
    DevBuf& db = c->msm[9];
    db.ensure(std::max<size_t>(1, n) * sizeof(G1A));
    if (n) HIPCK(hipMemcpyAsync(db.p, b.data(), n * sizeof(G1A), hipMemcpyHostToDevice, c->stream));
    c->input.ensure(std::max<size_t>(1, n) * 32);
    upload_fr_canonical(c, repr, scalars, n, c->input.fe());
    *out = g1_out(msm_g1_device(c, dptr<G1A>(db), c->input.fe(), n));
  });
}

// ---- KZG verifier half: G2 taus and the pairing (host; pairing.hpp) ----
int zk_kzg_g2_taus(const zk_kzg* k, zk_g2* out) {
  return guarded([&] {
    require(k && out, "null argument");
    for (uint32_t i = 0; i < k->nv; ++i) out[i] = g2_out(k->g2_taus[i]);
  });
}

int zk_g2_mul_generator(zk_repr repr, const zk_fe* scalars, size_t n, zk_g2* out) {
  return guarded([&] {
    require(n == 0 || (scalars && out), "null argument");
    const zk::G2J g2 = zk::g2_from_affine(zk::g2_generator());
    for (size_t i = 0; i < n; ++i) {
      uint32_t s[8];
      fr_canon(repr, scalars[i], s);
      out[i] = g2_out(zk::g2_to_affine(zk::g2_mul(g2, s)));
    }
  });
}

int zk_bls12_381_pairing(const zk_g1* p, const zk_g2* q, uint64_t out[72]) {
  return guarded([&] {
    require(p && q && out, "null argument");
    const zk::Fq12 e = zk::multi_pairing({parse_g1(*p)}, {parse_g2(*q)});
    const zk::Fq2* c[6] = {&e.c0.c0, &e.c0.c1, &e.c0.c2, &e.c1.c0, &e.c1.c1, &e.c1.c2};
    for (int i = 0; i < 6; ++i) {
      const Fq a = zk::fq_from_mont(c[i]->c0), b = zk::fq_from_mont(c[i]->c1);
      memcpy(out + 12 * i, a.v, 48);
      memcpy(out + 12 * i + 6, b.v, 48);
    }
  });
}

int zk_bls12_381_pairing_check(const zk_g1* p, const zk_g2* q, size_t n, int* out_ok) {
  return guarded([&] {
    require(out_ok && (n == 0 || (p && q)), "null argument");
    std::vector<G1A> P(n);
    std::vector<zk::G2A> Q(n);
    for (size_t i = 0; i < n; ++i) {
      P[i] = parse_g1(p[i]);
      Q[i] = parse_g2(q[i]);
    }
    *out_ok = zk::fq12_is_one(zk::multi_pairing(P, Q)) ? 1 : 0;
  });
}

// KZG::verify (kzg.rs:97-129): e(C - v G1, G2) == sum_i e(q_i, g2_taus[i] - a_i G2)
// (GT written additively in ark), checked as one product of Miller loops
// e(C - v G1, G2) * prod_i e(-q_i, g2_taus[i] - a_i G2) with one final
// exponentiation — the same boolean.
int zk_kzg_verify(zk_repr repr, const zk_g1* commitment, const zk_fe* opened_value, const zk_g1* proof,
                  uint32_t nproof, const zk_fe* point, uint32_t npoint, const zk_g2* g2_taus, int* out_verified) {
  return guarded([&] {
    require(commitment && opened_value && out_verified && ((proof && point && g2_taus) || npoint == 0),
            "null argument");
    // :104-106
    require(nproof == npoint, "num of quotients in proof not equal to num of opening values");
    using namespace zk;
    const G1J g1 = g1_from_affine(g1_generator());
    const G2J g2 = g2_from_affine(g2_generator());
    uint32_t v[8];
    fr_canon(repr, *opened_value, v);
    const G1J lhs = g1_add(g1_from_affine(parse_g1(*commitment)), g1_neg(g1_mul(g1, v)));
    // inputs parsed and checked on this thread (they may throw); the G2 factors
    // and the Miller loops — independent per point — on host threads, then
    // one product and one final exponentiation (multi_pairing's value)
    std::vector<G1A> P(npoint + 1);
    std::vector<G2A> Q(npoint + 1), tau(npoint);
    std::vector<std::array<uint32_t, 8>> a(npoint);
    P[0] = g1_affine(lhs);
    Q[0] = g2_generator();
    for (uint32_t i = 0; i < npoint; ++i) {
      fr_canon(repr, point[i], a[i].data());
      tau[i] = parse_g2(g2_taus[i]);
      G1A qi = parse_g1(proof[i]);
      if (!g1a_is_inf(qi)) qi.y = fq_neg(qi.y);
      P[i + 1] = qi;
    }
    host_parallel(npoint, [&](uint32_t i) {
      Q[i + 1] = g2_to_affine(g2_add(g2_from_affine(tau[i]), g2_neg(g2_mul(g2, a[i].data()))));
    });
    std::vector<Fq12> ml(npoint + 1, fq12_one());
    host_parallel(npoint + 1, [&](uint32_t i) {
      if (!g1a_is_inf(P[i]) && !Q[i].inf) ml[i] = miller_loop(P[i], Q[i]);
    });
    Fq12 f = fq12_one();
    for (const Fq12& m : ml) f = fq12_mul(f, m);
    *out_verified = fq12_is_one(final_exponentiation(f)) ? 1 : 0;
  });
}

}  // extern "C"
