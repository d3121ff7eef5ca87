// MI355X-native sum-check / GKR sum-check prover: host orchestration of the
// gfx950 kernels in kernels.hpp behind the C ABI of include/zk_sumcheck.h.
//
// Round structure:
//   GKR  (sum_check_protocol.rs:86-115): round 0 = k_gkr_round0 (e0,e1,e2);
//        round k>=1 = k_gkr_round (fold by r_{k-1} + e0,e2) -> k_reduce_partials
//        -> 96 B D2H -> host: e1 = s_{k-1}(r_{k-1}) - e0, closed-form
//        interpolation + trim, Keccak absorb, challenge r_k.
//   plain (sum_check_protocol.rs:25-52): k_sc_round (fold + half sums).
// The host side holds only O(1)-per-round scalar work and the transcript;
// every table-sized operation runs on the GPU.
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <new>
#include <string>
#include <utility>
#include <vector>

#include "../../include/zk_sumcheck.h"
#include "field.hpp"
#include "keccak.hpp"
#include "kernels.hpp"
#include "msm.hpp"

using zk::Fe;

// ===========================================================================
// errors
// ===========================================================================
namespace {
thread_local std::string g_last_error;

struct ZkError {
  int code;
  std::string msg;
};
[[noreturn]] void fail(int code, const std::string& msg) { throw ZkError{code, msg}; }

#define HIPCK(x)                                                                        \
  do {                                                                                  \
    hipError_t e_ = (x);                                                                \
    if (e_ != hipSuccess) fail(ZK_EDEVICE, std::string(#x) + ": " + hipGetErrorString(e_)); \
  } while (0)
#define NCCLCK(x)                                                                            \
  do {                                                                                       \
    ncclResult_t r_ = (x);                                                                   \
    if (r_ != ncclSuccess) fail(ZK_ECOMM, std::string(#x) + ": " + ncclGetErrorString(r_)); \
  } while (0)

template <class Fn>
int guarded(Fn&& fn) {
  try {
    fn();
    g_last_error.clear();
    return ZK_OK;
  } catch (const ZkError& e) {
    g_last_error = e.msg;
    return e.code;
  } catch (const std::bad_alloc&) {
    g_last_error = "host allocation failed";
    return ZK_ENOMEM;
  } catch (...) {
    g_last_error = "unknown error";
    return ZK_EDEVICE;
  }
}

void require(bool cond, const char* msg) {
  if (!cond) fail(ZK_EINVAL, msg);
}

// runtime field -> compile-time parameter set
template <class Fn>
void dispatch(zk_field field, Fn&& fn) {
  switch (field) {
    case ZK_BN254_FR: fn(zk::Bn254Fr{}); break;
    case ZK_BN254_FQ: fn(zk::Bn254Fq{}); break;
    case ZK_BLS12_381_FR: fn(zk::Bls12_381Fr{}); break;
    default: fail(ZK_EINVAL, "unknown field");
  }
}

// zk_fe (4 x u64 LE) <-> Fe (8 x u32 LE): same bytes on a little-endian host
inline Fe from_zk(const zk_fe& a) {
  Fe r;
  memcpy(r.v, a.limb, 32);
  return r;
}
inline zk_fe to_zk(const Fe& a) {
  zk_fe r;
  memcpy(r.limb, a.v, 32);
  return r;
}

template <class F>
Fe in_mont(zk_repr repr, const zk_fe& a) {  // host scalar in -> Montgomery
  Fe x = from_zk(a);
  require(zk::fe_is_canonical<F>(x), "field element >= modulus");
  return repr == ZK_REPR_MONTGOMERY ? x : zk::fe_to_mont<F>(x);
}
template <class F>
zk_fe out_repr(zk_repr repr, const Fe& m) {  // Montgomery -> host scalar out
  return to_zk(repr == ZK_REPR_MONTGOMERY ? m : zk::fe_from_mont<F>(m));
}
template <class F>
void canon_bytes(const Fe& m, uint8_t out[32]) {  // into_bigint().to_bytes_le()
  const Fe c = zk::fe_from_mont<F>(m);
  memcpy(out, c.v, 32);
}

}  // namespace

// ===========================================================================
// transcript (fiat_shamir_transcript.rs:5-37)
// ===========================================================================
struct zk_transcript {
  zk::Keccak256 h;
};

namespace {
// get_random_challenge: d = finalize_reset(); append(d); from_le_bytes_mod_order(d)
template <class F>
Fe challenge(zk_transcript* t) {
  uint8_t d[32];
  t->h.finalize_reset(d);
  t->h.update(d, 32);
  Fe x;
  memcpy(x.v, d, 32);
#pragma unroll
  for (int i = 0; i < 5; ++i) x = zk::fe_reduce_once<F>(x);  // 2^256 < 6p
  return zk::fe_to_mont<F>(x);
}
template <class F>
void absorb(zk_transcript* t, const Fe* m, size_t n) {  // append(fq_vec_to_bytes(v))
  uint8_t b[32];
  for (size_t i = 0; i < n; ++i) {
    canon_bytes<F>(m[i], b);
    t->h.update(b, 32);
  }
}
}  // namespace

// ===========================================================================
// context
// ===========================================================================
namespace {
struct DevBuf {
  void* p = nullptr;
  size_t bytes = 0;
  void ensure(size_t b) {
    if (b <= bytes) return;
    if (p) HIPCK(hipFree(p));
    p = nullptr;
    bytes = 0;
    if (hipMalloc(&p, b) != hipSuccess) {
      p = nullptr;
      (void)hipGetLastError();
      fail(ZK_ENOMEM, "hipMalloc of " + std::to_string(b) + " bytes failed");
    }
    bytes = b;
  }
  void release() {
    if (p) (void)hipFree(p);
    p = nullptr;
    bytes = 0;
  }
  Fe* fe(size_t off_elems = 0) const { return reinterpret_cast<Fe*>(p) + off_elems; }
};

enum CommKind { COMM_NONE = 0, COMM_HOST = 1, COMM_RCCL = 2 };
}  // namespace

struct zk_ctx {
  int device = 0;
  int num_cus = 256;
  hipStream_t stream = nullptr;
  DevBuf work[2];  // ping-pong fold workspaces: 4 tables each
  DevBuf input;    // host-API staging (4 tables)
  DevBuf partials;
  DevBuf small;    // round totals (<= 64 u64) + flag + gather buffers
  uint64_t* h_red = nullptr;  // pinned, device-mapped: round totals (<= 51 u64) + flag word at [64]
  uint32_t tag = 0;           // last round tag handed to a kernel
  uint64_t lanes_max_pairs = 1u << 15;  // rounds with <= this many pairs use 8 lanes per pair
  std::chrono::steady_clock::time_point work_t0;  // when the last round result was seen
  bool work_open = false;
  uint32_t timing = 0;  // bit k: time launches of kernel kind k
  zk_stats stats{};
  struct Pending {
    int kind;
    hipEvent_t a, b;
  };
  std::vector<std::pair<hipEvent_t, hipEvent_t>> ev_free;
  std::vector<Pending> pending;
  // communicator
  int rank = 0, world = 1;
  CommKind comm = COMM_NONE;
  zk_allreduce_u64_fn ar = nullptr;
  bool force_coll = false;  // debug: run the collective path even at world 1 (ZK_FORCE_COLLECTIVES)
  bool prelaunch = true;    // pre-enqueue round kernels (ZK_PRELAUNCH=0 launches each after its challenge)
  uint32_t rtag = 0;        // last tag handed to a pre-enqueued round kernel
  void* user = nullptr;
  ncclComm_t nccl = nullptr;
  // KZG / MSM scratch (grow-only) and the cached fixed-base table of G1
  DevBuf msm[16];
  DevBuf scan_tmp[4];
  DevBuf g1_table;
};

// a KZG setup: the Lagrange basis over the last v taus for v = 0..nv, affine
// Montgomery on the device (bases[nv] is get_lagrange_basis's output)
struct zk_kzg {
  uint32_t nv = 0;
  int device = 0;
  std::vector<DevBuf> bases;
  ~zk_kzg() {
    for (auto& b : bases) b.release();
  }
};

namespace {
// small device area: [0,512) round sums, [512] input check flag, [1024,2304)
// fan-in counters (9 x 128 B), [2560,3072) limb accumulator (<= 64 u64),
// [4096, +64 KiB) all-reduce bounce buffer
// (<= 256 ranks x 256 B), then the tail's 4 local elements and the gathered
// 4 x world tables
constexpr size_t kSmallBytes = 160 * 1024;
uint64_t* d_red(zk_ctx* c) { return reinterpret_cast<uint64_t*>(c->small.p); }
uint32_t* d_flag(zk_ctx* c) { return reinterpret_cast<uint32_t*>(reinterpret_cast<char*>(c->small.p) + 512); }
uint32_t* d_counter(zk_ctx* c) { return reinterpret_cast<uint32_t*>(reinterpret_cast<char*>(c->small.p) + 1024); }
uint64_t* d_accum(zk_ctx* c) { return reinterpret_cast<uint64_t*>(reinterpret_cast<char*>(c->small.p) + 2560); }
uint32_t* h_flag(zk_ctx* c) { return reinterpret_cast<uint32_t*>(c->h_red + 64); }
char* d_gather(zk_ctx* c) { return reinterpret_cast<char*>(c->small.p) + 4096; }
// pre-enqueued rounds: the pinned slot the host posts r to, the pinned error
// word, and the device relay slots (h_red page: [1024, 1088) and [2048];
// small area: [3072, 3584) = 8 x 64 B)
zk::RWait* h_rin(zk_ctx* c) { return reinterpret_cast<zk::RWait*>(reinterpret_cast<char*>(c->h_red) + 1024); }
uint32_t* h_err(zk_ctx* c) { return reinterpret_cast<uint32_t*>(reinterpret_cast<char*>(c->h_red) + 2048); }
zk::RWait* d_relay(zk_ctx* c) { return reinterpret_cast<zk::RWait*>(reinterpret_cast<char*>(c->small.p) + 3072); }

void bind(zk_ctx* c) { HIPCK(hipSetDevice(c->device)); }

// At most one resident wave of 256-thread blocks (blocks/CU from the
// kernel's register budget), grid-striding over the rest: no tail of
// half-empty CUs.
template <class K>
uint32_t grid_for(zk_ctx* c, uint64_t work, K kernel) {
  static thread_local std::vector<std::pair<const void*, int>> cache;
  int per_cu = 0;
  for (auto& e : cache)
    if (e.first == reinterpret_cast<const void*>(kernel)) per_cu = e.second;
  if (per_cu == 0) {
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kernel, zk::kBlock, 0) != hipSuccess || per_cu < 1)
      per_cu = 1;
    cache.push_back({reinterpret_cast<const void*>(kernel), per_cu});
  }
  const uint64_t cap = (uint64_t)c->num_cus * per_cu;
  uint64_t g = (work + zk::kBlock - 1) / zk::kBlock;
  if (g < 1) g = 1;
  return (uint32_t)std::min<uint64_t>(g, cap);
}

// Launch wrapper: counts algorithmic bytes / multiplications per kernel kind
// and, when timing is on, has the dispatch packet itself record start/stop
// events on c->stream (hipExtLaunchKernelGGL: no extra API calls per launch).
template <class Kern, class... Args>
void launch(zk_ctx* c, int kind, double bytes, double muls, Kern kernel, uint32_t grid, Args... args) {
  zk_ctx::Pending p{kind, nullptr, nullptr};
  const bool timed = (c->timing >> kind) & 1u;
  if (timed) {
    if (c->ev_free.empty()) {
      hipEvent_t a, b;
      HIPCK(hipEventCreate(&a));
      HIPCK(hipEventCreate(&b));
      c->ev_free.push_back({a, b});
    }
    p.a = c->ev_free.back().first;
    p.b = c->ev_free.back().second;
    c->ev_free.pop_back();
  }
  hipExtLaunchKernelGGL(kernel, dim3(grid), dim3(zk::kBlock), 0, c->stream, p.a, p.b, 0, args...);
  HIPCK(hipGetLastError());
  if (c->work_open) {
    c->stats.host_work_us +=
        std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - c->work_t0).count();
    c->work_open = false;
  }
  if (timed) c->pending.push_back(p);
  c->stats.launches[kind] += 1;
  c->stats.alg_bytes[kind] += bytes;
  c->stats.field_muls[kind] += muls;
}
// after a stream sync: fold event timings into the stats
void flush_timing(zk_ctx* c) {
  static const bool dbg = getenv("ZK_DEBUG_EVENTS") != nullptr;
  for (auto& p : c->pending) {
    float ms = 0.f;
    HIPCK(hipEventElapsedTime(&ms, p.a, p.b));
    if (dbg) fprintf(stderr, "zk: kind %d %.1f us\n", p.kind, ms * 1e3);
    c->stats.kernel_ms[p.kind] += ms;
    c->ev_free.push_back({p.a, p.b});
  }
  c->pending.clear();
}
void sync(zk_ctx* c) {
  c->work_open = false;
  HIPCK(hipStreamSynchronize(c->stream));
  c->stats.host_syncs += 1;
  flush_timing(c);
}

// limb-split element sum (8 x u64 holding 32-bit limbs, possibly summed over
// ranks) -> field element (Montgomery image of the sum)
template <class F>
Fe from_limb_sums(const uint64_t* w) {
  return zk::limbs_to_fe<F>(w, 8, false);
}

// ---------------------------------------------------------------------------
// Round sums: the round kernel's last block writes the K sums (limb-split)
// straight into pinned host memory and raises a flag; the host spins on the
// flag (no stream synchronisation, no copy kernel). Across ranks over RCCL the
// sums go to device memory, are all-reduced on the stream, then published.
// ---------------------------------------------------------------------------
bool multi_rank(zk_ctx* c) { return (c->world > 1 || c->force_coll) && c->comm != COMM_NONE; }

// In-place SUM of n u64 over all ranks (host memory in/out). RCCL runs on the
// ctx stream through a device bounce buffer; a host communicator runs its callback.
void allreduce_host(zk_ctx* c, uint64_t* w, size_t n) {
  if (c->comm == COMM_RCCL) {
    uint64_t* d = reinterpret_cast<uint64_t*>(d_gather(c));
    HIPCK(hipMemcpyAsync(d, w, n * 8, hipMemcpyHostToDevice, c->stream));
    NCCLCK(ncclAllReduce(d, d, n, ncclUint64, ncclSum, c->nccl, c->stream));
    HIPCK(hipMemcpyAsync(w, d, n * 8, hipMemcpyDeviceToHost, c->stream));
    sync(c);
  } else if (c->comm == COMM_HOST) {
    if (c->ar(c->user, w, n) != 0) fail(ZK_ECOMM, "host all-reduce callback failed");
  } else {
    fail(ZK_ECOMM, "no communicator attached");
  }
  c->stats.collectives += 1;
}

zk::RoundSink make_sink(zk_ctx* c, bool across_ranks) {
  zk::RoundSink s;
  s.partials = reinterpret_cast<uint64_t*>(c->partials.p);
  s.counter = d_counter(c);
  s.accum = d_accum(c);
  s.tag = ++c->tag;
  const bool via_rccl = across_ranks && multi_rank(c) && c->comm == COMM_RCCL;
  s.dev_out = via_rccl ? d_red(c) : nullptr;
  s.host_out = via_rccl ? nullptr : c->h_red;
  s.host_flag = via_rccl ? nullptr : h_flag(c);
  return s;
}

void wait_flag(zk_ctx* c, uint32_t tag) {
  const uint32_t* f = h_flag(c);
  uint64_t spins = 0;
  const auto t0 = std::chrono::steady_clock::now();
  if (c->work_open) {  // host work since the previous result ends at this wait
    c->stats.host_work_us += std::chrono::duration<double, std::micro>(t0 - c->work_t0).count();
    c->work_open = false;
  }
  while (__atomic_load_n(f, __ATOMIC_ACQUIRE) != tag) {
    __builtin_ia32_pause();
    if ((++spins & 0xFFFF) == 0) {
      const hipError_t e = hipStreamQuery(c->stream);
      if (e != hipSuccess && e != hipErrorNotReady) fail(ZK_EDEVICE, std::string("round kernel failed: ") + hipGetErrorString(e));
      const double s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
      if ((e == hipSuccess && s > 1.0) || s > 60.0) fail(ZK_EDEVICE, "round result flag never arrived");
    }
  }
  c->work_t0 = std::chrono::steady_clock::now();
  c->work_open = true;
  c->stats.host_wait_us += std::chrono::duration<double, std::micro>(c->work_t0 - t0).count();
  c->stats.host_syncs += 1;
}

// The round kernel's totals: K values of L limb sums each (L = 17: unreduced
// product sums, L = 8: element sums), summed over ranks when sharded.
// Stream side of a round's hand-off, enqueued right after its kernel: across
// ranks over RCCL the device totals are all-reduced and then published.
void enqueue_reduce(zk_ctx* c, const zk::RoundSink& sk, bool across_ranks, int n) {
  if (across_ranks && multi_rank(c) && c->comm == COMM_RCCL) {
    NCCLCK(ncclAllReduce(d_red(c), d_red(c), n, ncclUint64, ncclSum, c->nccl, c->stream));
    c->stats.collectives += 1;
    zk::k_publish<<<1, 64, 0, c->stream>>>(d_red(c), n, c->h_red, h_flag(c), sk.tag);
    HIPCK(hipGetLastError());
  }
}

template <class F, int K>
void collect_sums(zk_ctx* c, const zk::RoundSink& sk, bool across_ranks, int L, Fe (&out)[K]) {
  const bool multi = across_ranks && multi_rank(c);
  const int n = K * L;
  wait_flag(c, sk.tag);
  if (__atomic_load_n(h_err(c), __ATOMIC_ACQUIRE) != 0)
    fail(ZK_EDEVICE, "a pre-enqueued round kernel waited more than 1 s for its challenge");
  uint64_t w[K * 17];
  for (int i = 0; i < n; ++i) w[i] = __atomic_load_n(c->h_red + i, __ATOMIC_RELAXED);
  if (multi && c->comm == COMM_HOST) {
    if (c->ar(c->user, w, n) != 0) fail(ZK_ECOMM, "host all-reduce callback failed");
    c->stats.collectives += 1;
  }
  for (int k = 0; k < K; ++k) out[k] = zk::limbs_to_fe<F>(w + L * k, L, L == 17);
}

void ensure_partials(zk_ctx* c) { c->partials.ensure(((size_t)c->num_cus * 8 + 8) * zk::kSlotU64 * 8); }

// ---------------------------------------------------------------------------
// GKR sum-check rounds
// ---------------------------------------------------------------------------
struct GkrOut {
  std::vector<Fe> coeffs;     // 3 per round (Montgomery), trimmed count in ncoeffs
  std::vector<uint8_t> ncoeffs;
  std::vector<Fe> challenges;
};

// Round polynomial through (0,e0),(1,e1),(2,e2) — the unique degree<=2
// polynomial UnivariatePoly::interpolate returns (univariate_polynomial_dense.rs:48-74),
// trailing zero coefficients trimmed (:14-18). Absorbs it, draws r_k and
// returns s_k(r_k).
template <class F>
Fe finish_round(zk_transcript* tr, const Fe& e0, const Fe& e1, const Fe& e2, uint32_t k, GkrOut& out, Fe& r) {
  using namespace zk;
  Fe c[3];
  c[0] = e0;
  c[2] = fe_mul<F>(fe_add<F>(fe_sub<F>(e0, fe_dbl<F>(e1)), e2), fe_inv2<F>());
  c[1] = fe_sub<F>(fe_sub<F>(e1, e0), c[2]);
  int m = 3;
  while (m > 0 && fe_is_zero<F>(c[m - 1])) --m;
  absorb<F>(tr, c, (size_t)m);
  out.ncoeffs[k] = (uint8_t)m;
  for (int i = 0; i < 3; ++i) out.coeffs[3 * k + i] = i < m ? c[i] : fe_zero<F>();
  r = challenge<F>(tr);
  out.challenges[k] = r;
  // UnivariatePoly::evaluate(r) (:20-26) via Horner — same field value
  return fe_add<F>(c[0], fe_mul<F>(r, fe_add<F>(c[1], fe_mul<F>(r, c[2]))));
}

// Posts the challenge of a finished round to the pinned slot the next
// pre-enqueued round kernel polls. If the host unwinds mid-proof (exception),
// the destructor posts the last tag (kernels compare with >=, so every round
// still waiting proceeds with r = 0; its results are discarded) and drains
// the stream, so no kernel is left waiting.
struct PostR {
  zk_ctx* c;
  uint32_t last = 0;  // highest tag a kernel of this phase waits for (0: none)
  bool done = false;
  void post(const Fe& r, uint32_t tag) {
    zk::RWait* s = h_rin(c);
    for (int i = 0; i < 8; ++i) __atomic_store_n(&s->r.v[i], r.v[i], __ATOMIC_RELAXED);
    __atomic_store_n(&s->tag, tag, __ATOMIC_RELEASE);
  }
  ~PostR() {
    if (done || last == 0) return;
    post(zk::fe_zero<zk::Bn254Fr>(), last);
    (void)hipStreamSynchronize(c->stream);
  }
};

// Pre-enqueue the rounds of a phase (ZK_PRELAUNCH, default on)?
bool prelaunch(zk_ctx* c, uint32_t nv) { return c->prelaunch && nv > 1; }

// Run `nv` rounds over 4 device tables of 2^nv elements starting at global
// round k0. The first round of a phase computes e0,e1,e2 directly; later
// rounds fold by the previous challenge in the same kernel. On return `cur`
// points at the (unfolded) size-2 tables of the last round.
// Pre-enqueued (default): every round kernel (and, across ranks over RCCL,
// its all-reduce + publish) is enqueued before round 0's sums are read;
// round i's kernel waits in-kernel for r_{i-1}, which the host posts as soon
// as it has run the transcript. Otherwise each round is launched after the
// previous challenge is known.
template <class F>
void gkr_phase(zk_ctx* c, const Fe* cur[4], uint32_t nv, uint32_t k0, bool across_ranks, zk_transcript* tr,
               GkrOut& out, Fe& claim, Fe& r) {
  const uint64_t L = (uint64_t)1 << nv;
  const bool pre = prelaunch(c, nv);
  std::vector<zk::RoundSink> sinks(nv);
  std::vector<uint32_t> rtags(nv, 0);
  auto enqueue = [&](uint32_t i) {
    const uint64_t size = L >> i;  // table length in this round
    const uint64_t h = size / 2;   // pairs
    sinks[i] = make_sink(c, across_ranks);
    const zk::RoundSink& sk = sinks[i];
    if (i == 0) {
      const uint32_t grid = grid_for(c, 2 * h, zk::k_gkr_round0<F>);
      launch(c, ZK_K_GKR_ROUND0, 256.0 * h, 6.0 * h, zk::k_gkr_round0<F>, grid, cur[0], cur[1], cur[2], cur[3], h, sk);
      enqueue_reduce(c, sk, across_ranks, 3 * 17);
      return;
    }
    // fold previous (size 2*size) -> work[(i+1)&1] (size `size`) and evaluate;
    // work[0] holds the size-L/2 level, work[1] the size-L/4 level, ...
    Fe* w = c->work[(i + 1) & 1].fe();
    Fe* nx[4] = {w, w + size, w + 2 * size, w + 3 * size};
    zk::RoundIn rin{};
    if (pre) {
      rin.host = h_rin(c);
      rin.relay = d_relay(c);
      rin.err = h_err(c);
      rin.tag = rtags[i] = ++c->rtag;
    } else {
      rin.r = r;
    }
    if (h <= c->lanes_max_pairs) {  // latency-bound size: 8 lanes per pair
      const uint32_t g8 = grid_for(c, 8 * h, zk::k_gkr_round_lanes<F>);
      launch(c, ZK_K_GKR_ROUND, 768.0 * h, 12.0 * h, zk::k_gkr_round_lanes<F>, g8, cur[0], cur[1], cur[2], cur[3], nx[0], nx[1], nx[2], nx[3], h, rin, sk);
    } else {
      const uint32_t grid = grid_for(c, 2 * h, zk::k_gkr_round<F>);
      launch(c, ZK_K_GKR_ROUND, 768.0 * h, 12.0 * h, zk::k_gkr_round<F>, grid, cur[0], cur[1], cur[2], cur[3], nx[0], nx[1], nx[2], nx[3], h, rin, sk);
    }
    for (int t = 0; t < 4; ++t) cur[t] = nx[t];
    enqueue_reduce(c, sk, across_ranks, 2 * 17);
  };
  PostR post{c};
  if (pre) {
    const auto t0 = std::chrono::steady_clock::now();
    for (uint32_t i = 0; i < nv; ++i) {
      enqueue(i);
      post.last = rtags[i];  // from here on the guard releases what is enqueued
    }
    if (getenv("ZK_DEBUG_ENQUEUE"))
      fprintf(stderr, "zk: enqueued %u rounds in %.1f us\n", nv,
              std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count());
  }
  for (uint32_t i = 0; i < nv; ++i) {
    const uint32_t k = k0 + i;
    if (!pre) enqueue(i);
    Fe e0, e1, e2;
    if (i == 0) {
      Fe s[3];
      collect_sums<F, 3>(c, sinks[i], across_ranks, 17, s);
      e0 = s[0];
      e1 = s[1];
      e2 = s[2];
    } else {
      Fe s[2];
      collect_sums<F, 2>(c, sinks[i], across_ranks, 17, s);
      e0 = s[0];
      e2 = s[1];
      // s_{k-1}(X) = sum_j f(X, j) is exact (degree 2 in X), so
      // e0 + e1 = s_{k-1}(r_{k-1}) on the folded tables.
      e1 = zk::fe_sub<F>(claim, e0);
    }
    claim = finish_round<F>(tr, e0, e1, e2, k, out, r);
    if (pre && i + 1 < nv) post.post(r, rtags[i + 1]);
  }
  post.done = true;
}

template <class F>
void gkr_prove_device(zk_ctx* c, const Fe* const dT[4], uint32_t nloc, bool sharded, zk_transcript* tr, GkrOut& out) {
  const int G = sharded ? c->world : 1;
  uint32_t lg = 0;
  while ((1 << lg) < G) ++lg;
  const uint32_t n = nloc + lg;
  out.coeffs.assign(3 * (size_t)n, zk::fe_zero<F>());
  out.ncoeffs.assign(n, 0);
  out.challenges.assign(n, zk::fe_zero<F>());
  if (n == 0) return;
  ensure_partials(c);
  __atomic_store_n(h_err(c), 0u, __ATOMIC_RELAXED);
  const uint64_t Lloc = (uint64_t)1 << nloc;
  const uint64_t wmax = std::max<uint64_t>(Lloc / 2, (uint64_t)G);
  c->work[0].ensure(4 * wmax * 32);
  c->work[1].ensure(4 * std::max<uint64_t>(wmax / 2, 1) * 32);
  const Fe* cur[4] = {dT[0], dT[1], dT[2], dT[3]};
  Fe claim = zk::fe_zero<F>(), r = zk::fe_zero<F>();
  gkr_phase<F>(c, cur, nloc, 0, sharded, tr, out, claim, r);
  if (lg == 0) {
    sync(c);  // settles event timings; the results are already on the host
    return;
  }

  // ---- multi-GPU tail: every rank now holds 1 (folded) element per table ----
  // Gather the G x 4 elements with the same exact all-reduce as the rounds:
  // each rank fills only its own slot of a zeroed limb-split vector.
  Fe* send = reinterpret_cast<Fe*>(d_gather(c) + 65536);  // 4 elements, after the bounce buffer
  if (nloc > 0) {
    Fe* s4[4] = {send, send + 1, send + 2, send + 3};
    launch(c, ZK_K_FOLD, 4 * 96.0, 4.0, zk::k_fold4<F>, 1u, cur[0], cur[1], cur[2], cur[3], s4[0], s4[1], s4[2],
           s4[3], (uint64_t)1, r);
  } else {
    for (int t = 0; t < 4; ++t) HIPCK(hipMemcpyAsync(send + t, cur[t], 32, hipMemcpyDeviceToDevice, c->stream));
  }
  Fe mine[4];
  HIPCK(hipMemcpyAsync(mine, send, 128, hipMemcpyDeviceToHost, c->stream));
  sync(c);
  std::vector<uint64_t> w((size_t)G * 4 * 8, 0);
  for (int t = 0; t < 4; ++t)
    for (int i = 0; i < 8; ++i) w[((size_t)c->rank * 4 + t) * 8 + i] = mine[t].v[i];
  allreduce_host(c, w.data(), w.size());
  // global table t, index g = rank g's element (local index 0 <-> global g)
  std::vector<Fe> tabs((size_t)4 * G);
  for (int g = 0; g < G; ++g)
    for (int t = 0; t < 4; ++t) tabs[(size_t)t * G + g] = from_limb_sums<F>(&w[((size_t)g * 4 + t) * 8]);
  Fe* stage = send + 4;
  HIPCK(hipMemcpyAsync(stage, tabs.data(), tabs.size() * 32, hipMemcpyHostToDevice, c->stream));
  const Fe* tcur[4] = {stage, stage + G, stage + 2 * G, stage + 3 * G};
  gkr_phase<F>(c, tcur, lg, nloc, false, tr, out, claim, r);
  sync(c);
}

// ---------------------------------------------------------------------------
// plain sum-check
// ---------------------------------------------------------------------------
template <class F>
void sc_prove_device(zk_ctx* c, const Fe* dX, uint32_t n, zk_transcript* tr, const uint8_t* table_bytes,
                     size_t nbytes, Fe* rp, Fe& claimed) {
  // The transcript absorbs the whole table first (sum_check_protocol.rs:27):
  // a serial host Keccak. Round 0's half sums (and, pre-enqueued, every later
  // round) are launched before it so the GPU works underneath the hash.
  ensure_partials(c);
  __atomic_store_n(h_err(c), 0u, __ATOMIC_RELAXED);
  const uint64_t N = (uint64_t)1 << n;
  if (n == 0) {
    tr->h.update(table_bytes, nbytes);
    HIPCK(hipMemcpyAsync(&claimed, dX, 32, hipMemcpyDeviceToHost, c->stream));
    sync(c);
    absorb<F>(tr, &claimed, 1);
    return;
  }
  c->work[0].ensure(std::max<uint64_t>(N / 2, 1) * 32);
  c->work[1].ensure(std::max<uint64_t>(N / 4, 1) * 32);
  const bool pre = prelaunch(c, n);
  std::vector<zk::RoundSink> sinks(n);
  std::vector<uint32_t> rtags(n, 0);
  const Fe* cur = dX;
  Fe r = zk::fe_zero<F>();
  auto enqueue = [&](uint32_t k) {
    sinks[k] = make_sink(c, false);
    zk::RoundIn rin{};
    if (k == 0) {
      const uint64_t h = N / 2;
      const uint32_t grid = grid_for(c, h, zk::k_sc_round<F, true>);
      launch(c, ZK_K_SC_ROUND, 64.0 * h, 0, zk::k_sc_round<F, true>, grid, dX, nullptr, h, rin, sinks[k]);
      return;
    }
    const uint64_t h = (N >> k) / 2;
    const uint32_t grid = grid_for(c, h, zk::k_sc_round<F, false>);
    Fe* nx = c->work[(k + 1) & 1].fe();
    if (pre) {
      rin.host = h_rin(c);
      rin.relay = d_relay(c);
      rin.err = h_err(c);
      rin.tag = rtags[k] = ++c->rtag;
    } else {
      rin.r = r;
    }
    launch(c, ZK_K_SC_ROUND, 192.0 * h, 2.0 * h, zk::k_sc_round<F, false>, grid, cur, nx, h, rin, sinks[k]);
    cur = nx;
  };
  PostR post{c};
  if (pre)
    for (uint32_t k = 0; k < n; ++k) {
      enqueue(k);
      post.last = rtags[k];
    }
  else
    enqueue(0);
  tr->h.update(table_bytes, nbytes);  // serial Keccak overlaps the GPU
  for (uint32_t k = 0; k < n; ++k) {
    if (!pre && k > 0) enqueue(k);
    Fe s[2];
    collect_sums<F, 2>(c, sinks[k], false, 8, s);
    if (k == 0) {
      claimed = zk::fe_add<F>(s[0], s[1]);  // = sum of the table (:29)
      absorb<F>(tr, &claimed, 1);
    }
    rp[2 * k] = s[0];
    rp[2 * k + 1] = s[1];
    absorb<F>(tr, s, 2);
    r = challenge<F>(tr);
    if (pre && k + 1 < n) post.post(r, rtags[k + 1]);
  }
  post.done = true;
  sync(c);
}

// MultilinearPoly::evaluate on device: n folds at bit 0, ping-pong workspaces
template <class F>
Fe mle_evaluate_device(zk_ctx* c, const Fe* dX, uint32_t n, const std::vector<Fe>& pt) {
  const uint64_t N = (uint64_t)1 << n;
  Fe res;
  if (n == 0) {
    HIPCK(hipMemcpyAsync(&res, dX, 32, hipMemcpyDeviceToHost, c->stream));
    sync(c);
    return res;
  }
  c->work[0].ensure(std::max<uint64_t>(N / 2, 1) * 32);
  c->work[1].ensure(std::max<uint64_t>(N / 4, 1) * 32);
  const Fe* cur = dX;
  for (uint32_t i = 0; i < n; ++i) {
    const uint64_t half = N >> (i + 1);
    Fe* nx = c->work[i & 1].fe();
    const uint32_t grid = grid_for(c, half, zk::k_fold<F>);
    const Fe r = pt[i];
    const uint32_t s = n - 1 - i;  // bit 0 of the current (n-i)-variable table
    launch(c, ZK_K_FOLD, 96.0 * half, (double)half, zk::k_fold<F>, grid, cur, nx, half, s, r);
    cur = nx;
  }
  HIPCK(hipMemcpyAsync(&res, cur, 32, hipMemcpyDeviceToHost, c->stream));
  sync(c);
  return res;
}

// ---------------------------------------------------------------------------
// host <-> device staging with representation conversion
// ---------------------------------------------------------------------------
template <class F>
void upload(zk_ctx* c, zk_repr repr, const zk_fe* host, size_t n, Fe* dev) {
  if (n == 0) return;
  HIPCK(hipMemcpyAsync(dev, host, n * 32, hipMemcpyHostToDevice, c->stream));
  HIPCK(hipMemsetAsync(d_flag(c), 0, 4, c->stream));
  const uint32_t grid = grid_for(c, n, zk::k_check_canonical<F>);
  launch(c, ZK_K_CONVERT, 32.0 * n, 0, zk::k_check_canonical<F>, grid, dev, n, d_flag(c));
  if (repr == ZK_REPR_CANONICAL)
    launch(c, ZK_K_CONVERT, 64.0 * n, (double)n, zk::k_convert<F, true>, grid, dev, dev, n);
  uint32_t bad = 0;
  HIPCK(hipMemcpyAsync(&bad, d_flag(c), 4, hipMemcpyDeviceToHost, c->stream));
  sync(c);
  require(bad == 0, "field element >= modulus in input table");
}
template <class F>
void download(zk_ctx* c, zk_repr repr, const Fe* dev, size_t n, zk_fe* host) {
  if (n == 0) return;
  if (repr == ZK_REPR_CANONICAL) {
    c->work[1].ensure(std::max(c->work[1].bytes, n * 32));
    Fe* tmp = c->work[1].fe();
    const uint32_t grid = grid_for(c, n, zk::k_convert<F, false>);
    launch(c, ZK_K_CONVERT, 64.0 * n, (double)n, zk::k_convert<F, false>, grid, dev, tmp, n);
    dev = tmp;
  }
  HIPCK(hipMemcpyAsync(host, dev, n * 32, hipMemcpyDeviceToHost, c->stream));
  sync(c);
}

// canonical table bytes for the plain-prove transcript (fq_vec_to_bytes)
template <class F>
std::vector<uint8_t> table_bytes_from_device(zk_ctx* c, const Fe* dev, size_t n) {
  std::vector<uint8_t> b(n * 32);
  download<F>(c, ZK_REPR_CANONICAL, dev, n, reinterpret_cast<zk_fe*>(b.data()));
  return b;
}

bool pow2_ok(uint32_t nvars) { return nvars < 40; }

template <class F>
void emit_gkr(zk_repr repr, const GkrOut& g, uint32_t n, zk_fe* out_coeffs, uint8_t* out_ncoeffs,
              zk_fe* out_challenges) {
  for (uint32_t k = 0; k < n; ++k) {
    out_ncoeffs[k] = g.ncoeffs[k];
    for (int i = 0; i < 3; ++i) out_coeffs[3 * k + i] = out_repr<F>(repr, g.coeffs[3 * k + i]);
    out_challenges[k] = out_repr<F>(repr, g.challenges[k]);
  }
}

// ---------------------------------------------------------------------------
// GKR over a layered circuit: gkr_protocol.rs:31-126 with
// every table-sized step on the device — circuit evaluation, the four layer
// tables (kernels.hpp k_gate_weights / k_layer_tables, sparse wiring instead
// of the reference's dense 2^(3g+2) add_i/mul_i), the layer sum-check
// (gkr_prove_device) and w.evaluate(r_b / r_c) (mle_evaluate_device). The
// transcript and O(1) scalar steps stay on the host, as in the reference.
// Supported shape: the one for which the reference's table sizes agree — a
// binary tree of layers, ninputs = 2 G_0, G_{l+1} = G_l / 2, powers of two,
// output layer of 1 or 2 gates (initiate_protocol evaluates a 1-variable
// output poly, :229-241). The input-layer KZG opening (row f3) is replaced by
// returning the two input-MLE evaluations it opens (:106-111).
// ---------------------------------------------------------------------------
uint32_t lg2u(uint64_t x) {
  uint32_t k = 0;
  while (((uint64_t)1 << k) < x) ++k;
  return k;
}

void check_shape(uint32_t nlayers, const uint32_t* gates) {
  require(nlayers >= 1 && gates, "empty circuit");
  require(nlayers <= 24, "too many layers");
  for (uint32_t l = 0; l < nlayers; ++l) {
    require(gates[l] >= 1 && (gates[l] & (gates[l] - 1)) == 0, "layer sizes must be powers of two");
    if (l) require(2 * (uint64_t)gates[l] == gates[l - 1], "each layer must have half the gates of the one below");
  }
  require(gates[nlayers - 1] <= 2, "the output layer must have 1 or 2 gates");
  require(lg2u(2 * (uint64_t)gates[0]) <= 14, "circuit too large (input layer tables of (2 G_0)^2 entries)");
}

void check_circuit(uint32_t nlayers, const uint32_t* gates, const uint8_t* ops, uint32_t ninputs) {
  check_shape(nlayers, gates);
  require(ops != nullptr, "null argument");
  require((uint64_t)ninputs == 2 * (uint64_t)gates[0], "the first layer must have one gate per input pair");
  size_t nops = 0;
  for (uint32_t l = 0; l < nlayers; ++l) nops += gates[l];
  for (size_t i = 0; i < nops; ++i) require(ops[i] <= 1, "gate op must be 0 (add) or 1 (mul)");
}

uint32_t circuit_rounds(uint32_t nlayers, const uint32_t* gates) {
  uint32_t r = 0;
  for (uint32_t l = 0; l < nlayers; ++l) r += 2 * lg2u(2 * (uint64_t)gates[l]);
  return r;
}

struct CircuitOut {
  Fe out_poly[2];
  GkrOut sc;  // all layers' rounds, output layer first
  std::vector<Fe> claims;
  Fe in_eval[2];
};

template <class F>
void gkr_circuit_prove_device(zk_ctx* c, zk_repr repr, uint32_t nlayers, const uint32_t* gates, const uint8_t* ops,
                              const zk_fe* inputs, uint32_t ninputs, CircuitOut& o) {
  using namespace zk;
  struct Scoped {
    DevBuf b;
    ~Scoped() { b.release(); }
  } vals, dops, dwt, dpts;
  std::vector<size_t> off(nlayers + 1), opoff(nlayers + 1);
  off[0] = 0;
  opoff[0] = 0;
  for (uint32_t l = 0; l < nlayers; ++l) {
    off[l + 1] = off[l] + (l == 0 ? ninputs : gates[l - 1]);
    opoff[l + 1] = opoff[l] + gates[l];
  }
  const size_t nvals = off[nlayers] + gates[nlayers - 1];
  vals.b.ensure(nvals * 32);
  dops.b.ensure(opoff[nlayers]);
  dwt.b.ensure((size_t)gates[0] * 32);
  dpts.b.ensure(64 * 32);
  upload<F>(c, repr, inputs, ninputs, vals.b.fe(0));
  HIPCK(hipMemcpyAsync(dops.b.p, ops, opoff[nlayers], hipMemcpyHostToDevice, c->stream));
  const uint8_t* dop = reinterpret_cast<const uint8_t*>(dops.b.p);
  for (uint32_t l = 0; l < nlayers; ++l)  // Circuit::evaluate, input -> output (gkr_circuit.rs:127-143)
    launch(c, ZK_K_LAYER, 96.0 * gates[l], 0.5 * gates[l], k_circuit_layer<F>, (gates[l] + kBlock - 1) / kBlock,
           vals.b.fe(off[l]), dop + opoff[l], gates[l], vals.b.fe(off[l + 1]));
  const uint32_t gout = gates[nlayers - 1];
  Fe w0[2] = {fe_zero<F>(), fe_zero<F>()};
  HIPCK(hipMemcpyAsync(w0, vals.b.fe(off[nlayers]), 32 * gout, hipMemcpyDeviceToHost, c->stream));
  sync(c);  // (a 1-gate output is padded with zero, :36-38)
  o.out_poly[0] = w0[0];
  o.out_poly[1] = w0[1];

  zk_transcript tr;  // Transcript::new() (:32)
  absorb<F>(&tr, w0, 2);  // initiate_protocol (:229-241)
  const Fe r0 = challenge<F>(&tr);
  Fe claim = fe_add<F>(w0[0], fe_mul<F>(r0, fe_sub<F>(w0[1], w0[0])));
  absorb<F>(&tr, &claim, 1);
  std::vector<Fe> rb, rc;
  Fe alpha = fe_zero<F>(), beta = fe_zero<F>();
  const uint32_t total = circuit_rounds(nlayers, gates);
  o.sc.coeffs.assign(3 * (size_t)total, fe_zero<F>());
  o.sc.ncoeffs.assign(total, 0);
  o.sc.challenges.assign(total, fe_zero<F>());
  uint32_t k0 = 0;
  for (uint32_t idx = 0; idx < nlayers; ++idx) {
    const uint32_t l = nlayers - 1 - idx, G = gates[l], lgL = lg2u(2 * (uint64_t)G), nv = 2 * lgL;
    const uint64_t T = (uint64_t)1 << nv;
    const Fe* w = vals.b.fe(off[l]);  // the layer's inputs
    // gate weights: output layer folds its 1-bit index with r0 (get_fbc_poly, :243-263);
    // later layers alpha*eq(r_b, idx) + beta*eq(r_c, idx) (get_folded_fbc_poly, :265-292)
    std::vector<Fe> pts;
    uint32_t W;
    Fe a = fe_one<F>(), b = fe_zero<F>();
    uint32_t has_c = 0;
    if (idx == 0) {
      W = 1;
      pts = {r0};
    } else {
      W = lg2u(G);
      require(rb.size() == W && rc.size() == W, "internal: challenge split does not match the layer");
      pts = rb;
      pts.insert(pts.end(), rc.begin(), rc.end());
      a = alpha;
      b = beta;
      has_c = 1;
    }
    HIPCK(hipMemcpyAsync(dpts.b.p, pts.data(), pts.size() * 32, hipMemcpyHostToDevice, c->stream));
    launch(c, ZK_K_LAYER, 32.0 * G, (double)G * (W + 2), k_gate_weights<F>, (G + kBlock - 1) / kBlock, dpts.b.fe(0),
           dpts.b.fe(W), W, a, b, has_c, G, dwt.b.fe(0));
    c->input.ensure(4 * T * 32);
    Fe* tab = c->input.fe();
    const uint32_t grid = grid_for(c, T, k_layer_tables<F>);
    launch(c, ZK_K_LAYER, 128.0 * T, (double)T, k_layer_tables<F>, grid, w, lgL, dwt.b.fe(0), dop + opoff[l], tab,
           tab + T, tab + 2 * T, tab + 3 * T);
    const Fe* dT[4] = {tab, tab + T, tab + 2 * T, tab + 3 * T};
    GkrOut g;
    gkr_prove_device<F>(c, dT, nv, false, &tr, g);  // gkr_prove(claimed_sum, &fbc_poly, &mut transcript) (:68)
    for (uint32_t k = 0; k < nv; ++k) {
      for (int i = 0; i < 3; ++i) o.sc.coeffs[3 * (size_t)(k0 + k) + i] = g.coeffs[3 * (size_t)k + i];
      o.sc.ncoeffs[k0 + k] = g.ncoeffs[k];
      o.sc.challenges[k0 + k] = g.challenges[k];
    }
    k0 += nv;
    rb.assign(g.challenges.begin(), g.challenges.begin() + nv / 2);  // (:71-73)
    rc.assign(g.challenges.begin() + nv / 2, g.challenges.end());
    const Fe o1 = mle_evaluate_device<F>(c, w, lgL, rb), o2 = mle_evaluate_device<F>(c, w, lgL, rc);  // (:75-76)
    if (idx + 1 < nlayers) {  // (:80-89)
      absorb<F>(&tr, &o1, 1);
      alpha = challenge<F>(&tr);
      absorb<F>(&tr, &o2, 1);
      beta = challenge<F>(&tr);
      claim = fe_add<F>(fe_mul<F>(alpha, o1), fe_mul<F>(beta, o2));
      o.claims.push_back(o1);
      o.claims.push_back(o2);
    } else {
      o.in_eval[0] = o1;  // what KZG::open returns for r_b / r_c (:106-111)
      o.in_eval[1] = o2;
    }
  }
}

// eq(pt, v) over n bits, MSB first (the multilinear extension of a point indicator)
template <class F>
Fe eq_bits(const Fe* pt, uint64_t v, uint32_t n) {
  Fe e = zk::fe_one<F>();
  for (uint32_t k = 0; k < n; ++k) {
    const bool bit = (v >> (n - 1 - k)) & 1u;
    e = zk::fe_mul<F>(e, bit ? pt[k] : zk::fe_sub<F>(zk::fe_one<F>(), pt[k]));
  }
  return e;
}

template <class F>
Fe mle_eval_host(std::vector<Fe> t, const std::vector<Fe>& pt) {  // MultilinearPoly::evaluate (:79-91)
  for (const Fe& r : pt) {
    const size_t h = t.size() / 2;
    for (size_t j = 0; j < h; ++j) t[j] = zk::fe_add<F>(t[j], zk::fe_mul<F>(r, zk::fe_sub<F>(t[j + h], t[j])));
    t.resize(h);
  }
  return t[0];
}

// gkr::verify (gkr_protocol.rs:128-227). The wiring MLEs are evaluated
// sparsely (one eq term per gate) — the same value as the reference's dense
// add_i / mul_i evaluation. With inputs given, the input layer's two
// evaluations are recomputed from them (standing in for the KZG checks).
template <class F>
bool gkr_circuit_verify_host(zk_repr repr, uint32_t nlayers, const uint32_t* gates, const uint8_t* ops,
                             const zk_fe* inputs, uint32_t ninputs, const zk_fe* output_poly, const zk_fe* coeffs,
                             const uint8_t* ncoeffs, const zk_fe* claims, const zk_fe* input_evals) {
  using namespace zk;
  std::vector<size_t> opoff(nlayers + 1, 0);
  for (uint32_t l = 0; l < nlayers; ++l) opoff[l + 1] = opoff[l] + gates[l];
  zk_transcript tr;
  Fe w0[2] = {in_mont<F>(repr, output_poly[0]), in_mont<F>(repr, output_poly[1])};
  absorb<F>(&tr, w0, 2);
  const Fe r0 = challenge<F>(&tr);
  Fe claim = fe_add<F>(w0[0], fe_mul<F>(r0, fe_sub<F>(w0[1], w0[0])));
  absorb<F>(&tr, &claim, 1);
  Fe alpha = fe_zero<F>(), beta = fe_zero<F>();
  std::vector<Fe> prev;
  std::vector<Fe> in_m;
  if (inputs) {
    in_m.resize(ninputs);
    for (uint32_t i = 0; i < ninputs; ++i) in_m[i] = in_mont<F>(repr, inputs[i]);
  }
  size_t k0 = 0;
  const Fe zero = fe_zero<F>(), one = fe_one<F>();
  for (uint32_t idx = 0; idx < nlayers; ++idx) {
    const uint32_t l = nlayers - 1 - idx, G = gates[l], lgL = lg2u(2 * (uint64_t)G), nv = 2 * lgL;
    std::vector<Fe> chal;
    for (uint32_t k = 0; k < nv; ++k) {  // gkr_verify (sum_check_protocol.rs:117-150)
      const int m = ncoeffs[k0 + k];
      require(m <= 3, "round polynomial has more than 3 coefficients");
      Fe cf[3];
      for (int i = 0; i < m; ++i) cf[i] = in_mont<F>(repr, coeffs[3 * (k0 + k) + i]);
      auto ev = [&](const Fe& x) {
        Fe s = zero, xp = one;
        for (int i = 0; i < m; ++i) {
          s = fe_add<F>(s, fe_mul<F>(cf[i], xp));
          xp = fe_mul<F>(xp, x);
        }
        return s;
      };
      if (!fe_eq<F>(fe_add<F>(ev(zero), ev(one)), claim)) return false;
      absorb<F>(&tr, cf, (size_t)m);
      const Fe r = challenge<F>(&tr);
      chal.push_back(r);
      claim = ev(r);
    }
    k0 += nv;
    Fe o1, o2;
    if (idx + 1 == nlayers) {
      o1 = in_mont<F>(repr, input_evals[0]);
      o2 = in_mont<F>(repr, input_evals[1]);
      if (inputs) {
        const std::vector<Fe> rb(chal.begin(), chal.begin() + nv / 2), rc(chal.begin() + nv / 2, chal.end());
        if (!fe_eq<F>(o1, mle_eval_host<F>(in_m, rb)) || !fe_eq<F>(o2, mle_eval_host<F>(in_m, rc))) return false;
      }
    } else {
      o1 = in_mont<F>(repr, claims[2 * idx]);
      o2 = in_mont<F>(repr, claims[2 * idx + 1]);
    }
    Fe a_r = zero, m_r = zero;
    const uint32_t W = idx == 0 ? 1 : lg2u(G), Wbc = lgL;
    for (uint32_t gi = 0; gi < G; ++gi) {
      const uint64_t bc = ((uint64_t)(2 * gi) << Wbc) | (2 * gi + 1);
      Fe wgt;
      if (idx == 0) {  // get_verifier_claim: add_i.evaluate([r0] ++ chal) (:294-314)
        std::vector<Fe> pt{r0};
        pt.insert(pt.end(), chal.begin(), chal.end());
        wgt = eq_bits<F>(pt.data(), ((uint64_t)gi << (2 * Wbc)) | bc, W + 2 * Wbc);
      } else {  // get_folded_verifier_claim (:316-341)
        const size_t mid = prev.size() / 2;
        const Fe eb = eq_bits<F>(prev.data(), gi, W), ec = eq_bits<F>(prev.data() + mid, gi, W);
        wgt = fe_mul<F>(fe_add<F>(fe_mul<F>(alpha, eb), fe_mul<F>(beta, ec)), eq_bits<F>(chal.data(), bc, 2 * Wbc));
      }
      if (ops[opoff[l] + gi]) m_r = fe_add<F>(m_r, wgt);
      else a_r = fe_add<F>(a_r, wgt);
    }
    const Fe expect = fe_add<F>(fe_mul<F>(a_r, fe_add<F>(o1, o2)), fe_mul<F>(m_r, fe_mul<F>(o1, o2)));
    if (!fe_eq<F>(expect, claim)) return false;
    prev = chal;
    absorb<F>(&tr, &o1, 1);
    alpha = challenge<F>(&tr);
    absorb<F>(&tr, &o2, 1);
    beta = challenge<F>(&tr);
    claim = fe_add<F>(fe_mul<F>(alpha, o1), fe_mul<F>(beta, o2));
  }
  return true;
}

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
G1J* seg_reduce(zk_ctx* c, const G1A* bases, const uint32_t* order, const G1J* items0, const uint32_t* off,
                uint64_t nseg, int pool) {
  const G1J* items = items0;
  bool gather = order != nullptr;
  const uint32_t* cur_off = off;
  int flip = 0;
  for (int level = 0;; ++level) {
    require(level < 12, "segmented reduction did not converge");
    DevBuf& toff = c->msm[pool + flip];
    DevBuf& tseg = c->msm[pool + 2];
    DevBuf& part = c->msm[pool + 3 + flip];
    toff.ensure((nseg + 1) * 4);
    uint32_t* to = dptr<uint32_t>(toff);
    launch(c, ZK_K_MSM, 12.0 * nseg, 0, zk::k_seg_task_counts, blocks_for(nseg), cur_off, nseg, to);
    HIPCK(hipMemsetAsync(to + nseg, 0, 4, c->stream));
    scan_u32(c, to, nseg + 1);
    uint32_t total = 0;
    HIPCK(hipMemcpyAsync(&total, to + nseg, 4, hipMemcpyDeviceToHost, c->stream));
    sync(c);
    tseg.ensure((size_t)total * 4);
    launch(c, ZK_K_MSM, 4.0 * total, 0, zk::k_seg_task_owner, blocks_for(nseg), (const uint32_t*)to, nseg, total,
           dptr<uint32_t>(tseg));
    part.ensure((size_t)total * sizeof(G1J));
    if (gather)
      launch(c, ZK_K_MSM, 0, 0, zk::k_seg_sum<true>, blocks_for(total), bases, order, (const G1J*)nullptr, cur_off,
             (const uint32_t*)to, (const uint32_t*)dptr<uint32_t>(tseg), total, dptr<G1J>(part));
    else
      launch(c, ZK_K_MSM, 0, 0, zk::k_seg_sum<false>, blocks_for(total), (const G1A*)nullptr,
             (const uint32_t*)nullptr, items, cur_off, (const uint32_t*)to, (const uint32_t*)dptr<uint32_t>(tseg),
             total, dptr<G1J>(part));
    if (total == nseg) return dptr<G1J>(part);
    items = dptr<G1J>(part);
    cur_off = to;
    gather = false;
    flip ^= 1;
  }
}

// sum_i scalars[i] * bases[i]; scalars canonical Fr (device), bases affine Montgomery (device)
G1J msm_g1_device(zk_ctx* c, const G1A* bases, const Fe* scalars, uint64_t n) {
  using namespace zk;
  if (n == 0) return g1_inf();
  require(n < (1ull << 28), "MSM too large");
  uint32_t lg = 0;
  while ((2ull << lg) <= n) ++lg;
  const uint32_t cb = std::min<uint32_t>(20, std::max<uint32_t>(5, lg > 8 ? lg - 3 : 5));
  const uint32_t W = (255 + cb - 1) / cb;
  const uint64_t nb = (uint64_t)W << cb;
  DevBuf& cnt = c->msm[10];
  DevBuf& cur = c->msm[11];
  DevBuf& ord = c->msm[12];
  cnt.ensure((nb + 1) * 4);
  cur.ensure(nb * 4);
  ord.ensure(std::max<uint64_t>(1, n * W) * 4);
  HIPCK(hipMemsetAsync(cnt.p, 0, (nb + 1) * 4, c->stream));
  const uint32_t g = grid_for(c, n, k_msm_count);
  launch(c, ZK_K_MSM, 32.0 * n, 0, k_msm_count, g, scalars, n, cb, W, dptr<uint32_t>(cnt));
  scan_u32(c, dptr<uint32_t>(cnt), nb + 1);
  HIPCK(hipMemcpyAsync(cur.p, cnt.p, nb * 4, hipMemcpyDeviceToDevice, c->stream));
  launch(c, ZK_K_MSM, 32.0 * n, 0, k_msm_scatter, g, scalars, n, cb, W, dptr<uint32_t>(cur), dptr<uint32_t>(ord));
  // bucket sums (mixed additions of the gathered affine bases)
  G1J* buckets = seg_reduce(c, bases, dptr<uint32_t>(ord), nullptr, dptr<uint32_t>(cnt), nb, 0);
  // per window: sum_d d B_d over chunks of buckets, then over the chunks
  const uint32_t chunks = (1u << cb) / kBucketChunk;
  DevBuf& chb = c->msm[13];
  chb.ensure((size_t)W * chunks * sizeof(G1J));
  launch(c, ZK_K_MSM, 0, 0, k_window_chunks, blocks_for((uint64_t)W * chunks), (const G1J*)buckets, cb, W,
         dptr<G1J>(chb));
  std::vector<uint32_t> woff(W + 1);
  for (uint32_t w = 0; w <= W; ++w) woff[w] = w * chunks;
  DevBuf& wo = c->msm[14];
  wo.ensure((W + 1) * 4);
  HIPCK(hipMemcpyAsync(wo.p, woff.data(), (W + 1) * 4, hipMemcpyHostToDevice, c->stream));
  G1J* ws = seg_reduce(c, nullptr, nullptr, dptr<G1J>(chb), dptr<uint32_t>(wo), W, 5);
  std::vector<G1J> S(W);
  HIPCK(hipMemcpyAsync(S.data(), ws, W * sizeof(G1J), hipMemcpyDeviceToHost, c->stream));
  sync(c);
  // Horner over the windows on the host: R = sum_w 2^(c w) S_w
  G1J R = S[W - 1];
  for (uint32_t w = W - 1; w-- > 0;) {
    for (uint32_t k = 0; k < cb; ++k) R = g1_dbl(R);
    R = g1_add(R, S[w]);
  }
  return R;
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

// Fr values (host, repr) -> canonical Fr on the device (k_check_canonical + conversion)
void upload_fr_canonical(zk_ctx* c, zk_repr repr, const zk_fe* host, uint64_t n, Fe* dev) {
  upload<Fr381>(c, repr, host, n, dev);  // -> Montgomery, checked < r
  launch(c, ZK_K_CONVERT, 64.0 * n, (double)n, zk::k_convert<Fr381, false>, grid_for(c, n, zk::k_convert<Fr381, false>),
         (const Fe*)dev, dev, n);
}

G1J kzg_commit_canonical(zk_ctx* c, const zk_kzg* k, uint32_t v, const Fe* scalars) {
  return msm_g1_device(c, reinterpret_cast<const G1A*>(k->bases[v].p), scalars, (uint64_t)1 << v);
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
  out.clear();
  for (uint32_t i = 0; i < nv; ++i) {
    const uint32_t m = nv - i;  // variables of cur
    const uint64_t half = (uint64_t)1 << (m - 1);
    launch(c, ZK_K_FOLD, 96.0 * half, 0, k_top_diff<Fr381>, grid_for(c, half, k_top_diff<Fr381>), (const Fe*)cur,
           half, q);
    launch(c, ZK_K_CONVERT, 64.0 * half, (double)half, k_convert<Fr381, false>,
           grid_for(c, half, k_convert<Fr381, false>), (const Fe*)q, q, half);
    out.push_back(kzg_commit_canonical(c, k, m - 1, q));
    launch(c, ZK_K_FOLD, 96.0 * half, (double)half, k_fold<Fr381>, grid_for(c, half, k_fold<Fr381>), (const Fe*)cur,
           nxt, half, m - 1, point[i]);
    std::swap(cur, nxt);
  }
}
}  // namespace

// ===========================================================================
// C ABI
// ===========================================================================
extern "C" {

uint32_t zk_abi_version(void) { return ZK_ABI_VERSION; }
const char* zk_last_error(void) { return g_last_error.c_str(); }

int zk_ctx_create(int device, zk_ctx** out) {
  return guarded([&] {
    require(out != nullptr, "out is null");
    *out = nullptr;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) {
      (void)hipGetLastError();
      fail(ZK_EDEVICE, "no HIP device available (the prover has no CPU fallback)");
    }
    require(device >= 0 && device < ndev, "device index out of range");
    hipDeviceProp_t prop;
    HIPCK(hipGetDeviceProperties(&prop, device));
    if (std::string(prop.gcnArchName).rfind("gfx950", 0) != 0)
      fail(ZK_EDEVICE, std::string("kernels are built for gfx950, device is ") + prop.gcnArchName);
    auto* c = new zk_ctx();
    c->device = device;
    if (const char* e = getenv("ZK_LANES_MAX_PAIRS")) c->lanes_max_pairs = strtoull(e, nullptr, 0);  // tuning knob
    if (const char* e = getenv("ZK_FORCE_COLLECTIVES")) c->force_coll = atoi(e) != 0;
    if (const char* e = getenv("ZK_PRELAUNCH")) c->prelaunch = atoi(e) != 0;
    c->num_cus = prop.multiProcessorCount;
    try {
      bind(c);
      HIPCK(hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking));
      c->small.ensure(kSmallBytes);
      HIPCK(hipMemset(c->small.p, 0, kSmallBytes));
      HIPCK(hipHostMalloc(reinterpret_cast<void**>(&c->h_red), 4096, hipHostMallocMapped | hipHostMallocCoherent));
      memset(c->h_red, 0, 4096);
    } catch (...) {
      zk_ctx_destroy(c);
      throw;
    }
    *out = c;
  });
}

void zk_ctx_destroy(zk_ctx* c) {
  if (!c) return;
  (void)hipSetDevice(c->device);
  if (c->stream) (void)hipStreamSynchronize(c->stream);
  if (c->nccl) (void)ncclCommDestroy(c->nccl);
  for (auto& p : c->pending) c->ev_free.push_back({p.a, p.b});
  for (auto& e : c->ev_free) {
    (void)hipEventDestroy(e.first);
    (void)hipEventDestroy(e.second);
  }
  c->work[0].release();
  c->work[1].release();
  c->input.release();
  c->partials.release();
  c->small.release();
  for (auto& b : c->msm) b.release();
  for (auto& b : c->scan_tmp) b.release();
  c->g1_table.release();
  if (c->h_red) (void)hipHostFree(c->h_red);
  if (c->stream) (void)hipStreamDestroy(c->stream);
  delete c;
}

int zk_ctx_set_timing(zk_ctx* c, int enable) {
  return guarded([&] {
    require(c, "ctx is null");
    c->timing = enable ? (1u << ZK_K_KINDS) - 1 : 0u;
  });
}
int zk_ctx_set_timing_mask(zk_ctx* c, uint32_t kind_mask) {
  return guarded([&] {
    require(c, "ctx is null");
    c->timing = kind_mask & ((1u << ZK_K_KINDS) - 1);
  });
}
int zk_ctx_get_stats(const zk_ctx* c, zk_stats* out) {
  return guarded([&] {
    require(c && out, "null argument");
    *out = c->stats;
  });
}
int zk_ctx_reset_stats(zk_ctx* c) {
  return guarded([&] {
    require(c, "ctx is null");
    c->stats = zk_stats{};
  });
}

// ---- transcript ----
zk_transcript* zk_transcript_new(void) { return new (std::nothrow) zk_transcript(); }
zk_transcript* zk_transcript_clone(const zk_transcript* t) {
  return t ? new (std::nothrow) zk_transcript(*t) : nullptr;
}
void zk_transcript_free(zk_transcript* t) { delete t; }
int zk_transcript_append(zk_transcript* t, const uint8_t* data, size_t len) {
  return guarded([&] {
    require(t && (data || len == 0), "null argument");
    t->h.update(data, len);
  });
}
int zk_transcript_get_random_challenge(zk_transcript* t, zk_field field, zk_repr repr, zk_fe* out) {
  return guarded([&] {
    require(t && out, "null argument");
    dispatch(field, [&](auto f) {
      using F = decltype(f);
      *out = out_repr<F>(repr, challenge<F>(t));
    });
  });
}
int zk_fe_vec_to_bytes(zk_field field, zk_repr repr, const zk_fe* v, size_t n, uint8_t* out) {
  return guarded([&] {
    require((v && out) || n == 0, "null argument");
    dispatch(field, [&](auto f) {
      using F = decltype(f);
      for (size_t i = 0; i < n; ++i) canon_bytes<F>(in_mont<F>(repr, v[i]), out + 32 * i);
    });
  });
}

// ---- MultilinearPoly ----
int zk_mle_partial_evaluate(zk_ctx* c, zk_field field, zk_repr repr, const zk_fe* evals, uint32_t nvars,
                            uint32_t bit, const zk_fe* value, zk_fe* out) {
  return guarded([&] {
    require(c && evals && value && out, "null argument");
    require(pow2_ok(nvars), "table too large");
    require(nvars >= 1, "partial_evaluate of a 0-variable polynomial (pair_points underflow panics)");
    require(bit < nvars, "bit >= num_of_vars (pair_points underflow panics)");
    bind(c);
    dispatch(field, [&](auto f) {
      using F = decltype(f);
      const uint64_t N = (uint64_t)1 << nvars, half = N / 2;
      const Fe r = in_mont<F>(repr, *value);
      c->input.ensure(N * 32);
      upload<F>(c, repr, evals, N, c->input.fe());
      c->work[0].ensure(half * 32);
      const uint32_t grid = grid_for(c, half, zk::k_fold<F>);
      const uint32_t s = nvars - 1 - bit;
      launch(c, ZK_K_FOLD, 96.0 * half, (double)half, zk::k_fold<F>, grid, c->input.fe(), c->work[0].fe(), half, s, r);
      download<F>(c, repr, c->work[0].fe(), half, out);
    });
  });
}

int zk_mle_evaluate(zk_ctx* c, zk_field field, zk_repr repr, const zk_fe* evals, uint32_t nvars,
                    const zk_fe* point, uint32_t npoint, zk_fe* out) {
  return guarded([&] {
    require(c && evals && out && (point || npoint == 0), "null argument");
    require(pow2_ok(nvars), "table too large");
    require(npoint == nvars, "Invalid number of values");
    bind(c);
    dispatch(field, [&](auto f) {
      using F = decltype(f);
      const uint64_t N = (uint64_t)1 << nvars;
      std::vector<Fe> pt(nvars);
      for (uint32_t i = 0; i < nvars; ++i) pt[i] = in_mont<F>(repr, point[i]);
      c->input.ensure(N * 32);
      upload<F>(c, repr, evals, N, c->input.fe());
      *out = out_repr<F>(repr, mle_evaluate_device<F>(c, c->input.fe(), nvars, pt));
    });
  });
}

// ---- sum-check ----
int zk_sumcheck_prove(zk_ctx* c, zk_field field, zk_repr repr, const zk_fe* evals, uint32_t nvars,
                      zk_fe* out_round_polys, zk_fe* out_claimed_sum) {
  return guarded([&] {
    require(c && evals && out_claimed_sum && (out_round_polys || nvars == 0), "null argument");
    require(pow2_ok(nvars), "table too large");
    bind(c);
    dispatch(field, [&](auto f) {
      using F = decltype(f);
      const uint64_t N = (uint64_t)1 << nvars;
      c->input.ensure(N * 32);
      upload<F>(c, repr, evals, N, c->input.fe());
      std::vector<uint8_t> bytes;
      const uint8_t* tb = reinterpret_cast<const uint8_t*>(evals);  // canonical host bytes == fq_vec_to_bytes
      if (repr == ZK_REPR_MONTGOMERY) {
        bytes = table_bytes_from_device<F>(c, c->input.fe(), N);
        tb = bytes.data();
      }
      zk_transcript tr;
      std::vector<Fe> rp(2 * (size_t)nvars + 1);
      Fe claimed;
      sc_prove_device<F>(c, c->input.fe(), nvars, &tr, tb, N * 32, rp.data(), claimed);
      for (size_t i = 0; i < 2 * (size_t)nvars; ++i) out_round_polys[i] = out_repr<F>(repr, rp[i]);
      *out_claimed_sum = out_repr<F>(repr, claimed);
    });
  });
}

int zk_sumcheck_verify(zk_ctx* c, zk_field field, zk_repr repr, const zk_fe* evals, uint32_t nvars,
                       const zk_fe* round_polys, uint32_t nrounds, uint32_t poly_len, const zk_fe* claimed_sum,
                       int* out_verified) {
  return guarded([&] {
    require(c && evals && claimed_sum && out_verified && (round_polys || nrounds == 0), "null argument");
    require(pow2_ok(nvars), "table too large");
    // MultilinearPoly::new(poly.to_vec()) panics on non-power-of-two length (:64)
    require(nrounds == 0 || (poly_len != 0 && (poly_len & (poly_len - 1)) == 0), "Invalid evaluations");
    bind(c);
    dispatch(field, [&](auto f) {
      using F = decltype(f);
      const uint64_t N = (uint64_t)1 << nvars;
      c->input.ensure(N * 32);
      upload<F>(c, repr, evals, N, c->input.fe());
      zk_transcript tr;
      if (repr == ZK_REPR_MONTGOMERY) {
        auto b = table_bytes_from_device<F>(c, c->input.fe(), N);
        tr.h.update(b.data(), b.size());
      } else {
        tr.h.update(reinterpret_cast<const uint8_t*>(evals), N * 32);
      }
      Fe expected = in_mont<F>(repr, *claimed_sum);
      absorb<F>(&tr, &expected, 1);
      std::vector<Fe> chal, pv(poly_len ? poly_len : 1);
      uint32_t tables_left = nvars;  // the redundant fold (:76) panics once exhausted
      for (uint32_t k = 0; k < nrounds; ++k) {
        Fe s = zk::fe_zero<F>();
        for (uint32_t i = 0; i < poly_len; ++i) {
          pv[i] = in_mont<F>(repr, round_polys[(size_t)k * poly_len + i]);
          s = zk::fe_add<F>(s, pv[i]);
        }
        if (!zk::fe_eq<F>(s, expected)) {  // :66-68
          *out_verified = 0;
          return;
        }
        require(poly_len >= 2, "index out of bounds: poly.evaluation[1]");
        absorb<F>(&tr, pv.data(), poly_len);
        const Fe r = challenge<F>(&tr);
        expected = zk::fe_add<F>(pv[0], zk::fe_mul<F>(r, zk::fe_sub<F>(pv[1], pv[0])));  // :73-74
        require(tables_left > 0, "partial_evaluate of a 0-variable polynomial (pair_points underflow panics)");
        --tables_left;
        chal.push_back(r);
      }
      require(chal.size() == nvars, "Invalid number of values");  // evaluate() :80-82
      const Fe v = mle_evaluate_device<F>(c, c->input.fe(), nvars, chal);
      *out_verified = zk::fe_eq<F>(expected, v) ? 1 : 0;
    });
  });
}

int zk_gkr_sumcheck_prove(zk_ctx* c, zk_field field, zk_repr repr, const zk_fe* const tables[4], uint32_t nvars,
                          const zk_fe* claimed_sum, zk_transcript* transcript, zk_fe* out_coeffs,
                          uint8_t* out_ncoeffs, zk_fe* out_challenges, zk_fe* out_claimed_sum) {
  return guarded([&] {
    require(c && tables && claimed_sum && transcript && out_claimed_sum, "null argument");
    require(nvars == 0 || (out_coeffs && out_ncoeffs && out_challenges), "null output");
    for (int t = 0; t < 4; ++t) require(tables[t] != nullptr, "null table");
    require(pow2_ok(nvars), "table too large");
    bind(c);
    dispatch(field, [&](auto f) {
      using F = decltype(f);
      const Fe cs = in_mont<F>(repr, *claimed_sum);
      const uint64_t N = (uint64_t)1 << nvars;
      c->input.ensure(4 * N * 32);
      const Fe* dT[4];
      for (int t = 0; t < 4; ++t) {
        upload<F>(c, repr, tables[t], N, c->input.fe(t * N));
        dT[t] = c->input.fe(t * N);
      }
      GkrOut g;
      gkr_prove_device<F>(c, dT, nvars, false, transcript, g);
      emit_gkr<F>(repr, g, nvars, out_coeffs, out_ncoeffs, out_challenges);
      *out_claimed_sum = out_repr<F>(repr, cs);  // carried through (:110-114)
    });
  });
}

int zk_gkr_sumcheck_verify(zk_field field, zk_repr repr, const zk_fe* coeffs, const uint8_t* ncoeffs,
                           uint32_t nrounds, const zk_fe* claimed_sum, zk_transcript* transcript, int* out_verified,
                           zk_fe* out_final_claimed_sum, zk_fe* out_challenges) {
  return guarded([&] {
    require(claimed_sum && transcript && out_verified && out_final_claimed_sum && out_challenges, "null argument");
    require(nrounds == 0 || (coeffs && ncoeffs), "null argument");
    dispatch(field, [&](auto f) {
      using F = decltype(f);
      using namespace zk;
      Fe claim = in_mont<F>(repr, *claimed_sum);
      const Fe zero = fe_zero<F>(), one = fe_one<F>();
      for (uint32_t k = 0; k < nrounds; ++k) {
        require(ncoeffs[k] <= 3, "round polynomial has more than 3 coefficients");
        Fe cf[3];
        const int m = ncoeffs[k];
        for (int i = 0; i < m; ++i) cf[i] = in_mont<F>(repr, coeffs[3 * k + i]);
        // UnivariatePoly::evaluate (univariate_polynomial_dense.rs:20-26)
        auto eval = [&](const Fe& x) {
          Fe s = zero, xp = one;
          for (int i = 0; i < m; ++i) {
            s = fe_add<F>(s, fe_mul<F>(cf[i], xp));
            xp = fe_mul<F>(xp, x);
          }
          return s;
        };
        if (!fe_eq<F>(fe_add<F>(eval(zero), eval(one)), claim)) {  // :128-134
          *out_verified = 0;
          *out_final_claimed_sum = out_repr<F>(repr, zero);
          out_challenges[0] = out_repr<F>(repr, zero);
          return;
        }
        absorb<F>(transcript, cf, (size_t)m);
        const Fe r = challenge<F>(transcript);
        out_challenges[k] = out_repr<F>(repr, r);
        claim = eval(r);
      }
      *out_verified = 1;
      *out_final_claimed_sum = out_repr<F>(repr, claim);
    });
  });
}

// ---- GKR over a layered circuit ----
int zk_gkr_circuit_rounds(uint32_t nlayers, const uint32_t* gates, uint32_t* out_total_rounds) {
  return guarded([&] {
    require(gates && out_total_rounds, "null argument");
    check_shape(nlayers, gates);
    *out_total_rounds = circuit_rounds(nlayers, gates);
  });
}

int zk_gkr_circuit_prove(zk_ctx* c, zk_field field, zk_repr repr, uint32_t nlayers, const uint32_t* gates,
                         const uint8_t* ops, const zk_fe* inputs, uint32_t ninputs, zk_fe* out_output_poly,
                         zk_fe* out_coeffs, uint8_t* out_ncoeffs, zk_fe* out_challenges, zk_fe* out_claims,
                         zk_fe* out_input_evals) {
  return guarded([&] {
    require(c && inputs && out_output_poly && out_coeffs && out_ncoeffs && out_challenges && out_input_evals,
            "null argument");
    check_circuit(nlayers, gates, ops, ninputs);
    require(nlayers == 1 || out_claims, "null argument");
    bind(c);
    dispatch(field, [&](auto f) {
      using F = decltype(f);
      CircuitOut o;
      gkr_circuit_prove_device<F>(c, repr, nlayers, gates, ops, inputs, ninputs, o);
      for (int i = 0; i < 2; ++i) out_output_poly[i] = out_repr<F>(repr, o.out_poly[i]);
      emit_gkr<F>(repr, o.sc, (uint32_t)o.sc.ncoeffs.size(), out_coeffs, out_ncoeffs, out_challenges);
      for (size_t i = 0; i < o.claims.size(); ++i) out_claims[i] = out_repr<F>(repr, o.claims[i]);
      for (int i = 0; i < 2; ++i) out_input_evals[i] = out_repr<F>(repr, o.in_eval[i]);
    });
  });
}

int zk_gkr_circuit_verify(zk_field field, zk_repr repr, uint32_t nlayers, const uint32_t* gates, const uint8_t* ops,
                          const zk_fe* inputs, uint32_t ninputs, const zk_fe* output_poly, const zk_fe* coeffs,
                          const uint8_t* ncoeffs, const zk_fe* claims, const zk_fe* input_evals, int* out_verified) {
  return guarded([&] {
    require(output_poly && coeffs && ncoeffs && input_evals && out_verified, "null argument");
    check_circuit(nlayers, gates, ops, ninputs);
    require(nlayers == 1 || claims, "null argument");
    dispatch(field, [&](auto f) {
      using F = decltype(f);
      *out_verified = gkr_circuit_verify_host<F>(repr, nlayers, gates, ops, inputs, ninputs, output_poly, coeffs,
                                                 ncoeffs, claims, input_evals)
                          ? 1
                          : 0;
    });
  });
}

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
    k->bases.resize(nvars + 1);
    const uint64_t N = (uint64_t)1 << nvars;
    const G1A* table = g1_fixed_table(c);
    DevBuf& tb = c->msm[14];
    tb.ensure(nvars * 32);
    upload<Fr381>(c, repr, taus, nvars, reinterpret_cast<Fe*>(tb.p));
    DevBuf& sc = c->msm[15];
    sc.ensure(N * 32);
    launch(c, ZK_K_MSM, 32.0 * N, (double)N * nvars, zk::k_eq_scalars<Fr381>, grid_for(c, N, zk::k_eq_scalars<Fr381>),
           (const Fe*)tb.p, nvars, N, reinterpret_cast<Fe*>(sc.p));
    DevBuf& jac = c->msm[13];
    jac.ensure(N * sizeof(G1J));
    launch(c, ZK_K_MSM, 176.0 * N, 0, zk::k_fixed_base, grid_for(c, N, zk::k_fixed_base), table,
           (const Fe*)sc.p, N, dptr<G1J>(jac));
    for (uint32_t v = nvars + 1; v-- > 0;) {
      const uint64_t n = (uint64_t)1 << v;
      if (v < nvars)
        launch(c, ZK_K_MSM, 336.0 * n, 0, zk::k_pair_sum, grid_for(c, n, zk::k_pair_sum),
               (const G1A*)k->bases[v + 1].p, n, dptr<G1J>(jac));
      k->bases[v].ensure(n * sizeof(G1A));
      launch(c, ZK_K_MSM, 240.0 * n, 0, zk::k_batch_normalize, blocks_for((n + zk::kBatchNorm - 1) / zk::kBatchNorm),
             (const G1J*)dptr<G1J>(jac), n, dptr<G1A>(k->bases[v]));
    }
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
    HIPCK(hipMemcpyAsync(a.data(), k->bases[nvars_suffix].p, n * sizeof(G1A), hipMemcpyDeviceToHost, c->stream));
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
    for (uint32_t i = 0; i < k->nv; ++i) out[i] = g1_out(q[i]);
  });
}

int zk_msm_g1(zk_ctx* c, zk_repr repr, const zk_g1* bases, const zk_fe* scalars, size_t n, zk_g1* out) {
  return guarded([&] {
    require(c && out && (n == 0 || (bases && scalars)), "null argument");
    bind(c);
    std::vector<G1A> b(n);
    for (size_t i = 0; i < n; ++i) {
      Fq x, y;
      memcpy(x.v, bases[i].x, 48);
      memcpy(y.v, bases[i].y, 48);
      require(zk::fq_is_canonical(x) && zk::fq_is_canonical(y), "point coordinate >= modulus");
      if (zk::fq_is_zero(x) && zk::fq_is_zero(y)) {
        b[i] = {zk::fq_zero(), zk::fq_zero()};
      } else {
        b[i] = {zk::fq_to_mont(x), zk::fq_to_mont(y)};
        const Fq lhs = zk::fq_sqr(b[i].y);
        Fq four = zk::fq_zero();
        four.v[0] = 4;
        const Fq rhs = zk::fq_add(zk::fq_mul(zk::fq_sqr(b[i].x), b[i].x), zk::fq_to_mont(four));
        require(zk::fq_eq(lhs, rhs), "point not on the curve");
      }
    }
    DevBuf& db = c->msm[9];
    db.ensure(std::max<size_t>(1, n) * sizeof(G1A));
    if (n) HIPCK(hipMemcpyAsync(db.p, b.data(), n * sizeof(G1A), hipMemcpyHostToDevice, c->stream));
    c->input.ensure(std::max<size_t>(1, n) * 32);
    upload_fr_canonical(c, repr, scalars, n, c->input.fe());
    *out = g1_out(msm_g1_device(c, dptr<G1A>(db), c->input.fe(), n));
  });
}

// ---- proof blobs ----
// Layout (include/zk_sumcheck.h "Proof blob"): "ZKSP", version 1, kind,
// field, 0, nrounds (u32 LE), claimed_sum (32 B), then per round m (u8) and
// m canonical 32-byte LE coefficients — for a GKR proof exactly the bytes the
// transcript absorbs in that round (fq_vec_to_bytes of the trimmed poly).
extern "C++" {
namespace {
constexpr uint8_t kBlobVersion = 1;

struct BlobWriter {
  uint8_t* out;
  size_t cap, len = 0;
  void put(const void* p, size_t n) {
    if (out && len + n <= cap) memcpy(out + len, p, n);
    len += n;
  }
  void u8(uint8_t v) { put(&v, 1); }
  void u32(uint32_t v) { put(&v, 4); }  // little-endian host
};

template <class F>
void blob_fe(BlobWriter& w, zk_repr repr, const zk_fe& x) {
  uint8_t b[32];
  canon_bytes<F>(in_mont<F>(repr, x), b);
  w.put(b, 32);
}

void blob_header(BlobWriter& w, int kind, zk_field field, uint32_t nrounds) {
  w.put("ZKSP", 4);
  w.u8(kBlobVersion);
  w.u8((uint8_t)kind);
  w.u8((uint8_t)field);
  w.u8(0);
  w.u32(nrounds);
}

struct BlobReader {
  const uint8_t* p;
  size_t len, off = 0;
  const uint8_t* take(size_t n) {
    require(off + n <= len, "proof blob truncated");
    const uint8_t* q = p + off;
    off += n;
    return q;
  }
};

// parse the header; returns kind
int blob_open(BlobReader& r, zk_field* field, uint32_t* nrounds) {
  const uint8_t* h = r.take(12);
  require(memcmp(h, "ZKSP", 4) == 0, "not a proof blob");
  require(h[4] == kBlobVersion, "unsupported proof blob version");
  require(h[5] == ZK_BLOB_GKR || h[5] == ZK_BLOB_SUMCHECK, "unknown proof blob kind");
  require(h[6] <= ZK_BLS12_381_FR && h[7] == 0, "bad proof blob header");
  *field = (zk_field)h[6];
  memcpy(nrounds, h + 8, 4);
  return h[5];
}

template <class F>
zk_fe blob_read_fe(BlobReader& r, zk_repr repr) {  // canonical bytes -> repr, rejects >= p
  zk_fe x;
  memcpy(x.limb, r.take(32), 32);
  const Fe c = from_zk(x);
  require(zk::fe_is_canonical<F>(c), "proof blob element >= modulus");
  return repr == ZK_REPR_MONTGOMERY ? to_zk(zk::fe_to_mont<F>(c)) : x;
}
}  // namespace
}  // extern "C++"

int zk_gkr_proof_to_blob(zk_field field, zk_repr repr, const zk_fe* coeffs, const uint8_t* ncoeffs, uint32_t nrounds,
                         const zk_fe* claimed_sum, uint8_t* out, size_t cap, size_t* out_len) {
  return guarded([&] {
    require(claimed_sum && out_len && (nrounds == 0 || (coeffs && ncoeffs)), "null argument");
    dispatch(field, [&](auto f) {
      using F = decltype(f);
      BlobWriter w{out, cap};
      blob_header(w, ZK_BLOB_GKR, field, nrounds);
      blob_fe<F>(w, repr, *claimed_sum);
      for (uint32_t k = 0; k < nrounds; ++k) {
        require(ncoeffs[k] <= 3, "round polynomial has more than 3 coefficients");
        w.u8(ncoeffs[k]);
        for (int i = 0; i < ncoeffs[k]; ++i) blob_fe<F>(w, repr, coeffs[3 * (size_t)k + i]);
      }
      *out_len = w.len;
      if (out) require(w.len <= cap, "output buffer too small");
    });
  });
}

int zk_sumcheck_proof_to_blob(zk_field field, zk_repr repr, const zk_fe* round_polys, uint32_t nrounds,
                              uint32_t poly_len, const zk_fe* claimed_sum, uint8_t* out, size_t cap, size_t* out_len) {
  return guarded([&] {
    require(claimed_sum && out_len && (nrounds == 0 || round_polys), "null argument");
    require(poly_len <= 255, "round polynomial too long for the blob format");
    dispatch(field, [&](auto f) {
      using F = decltype(f);
      BlobWriter w{out, cap};
      blob_header(w, ZK_BLOB_SUMCHECK, field, nrounds);
      blob_fe<F>(w, repr, *claimed_sum);
      for (uint32_t k = 0; k < nrounds; ++k) {
        w.u8((uint8_t)poly_len);
        for (uint32_t i = 0; i < poly_len; ++i) blob_fe<F>(w, repr, round_polys[(size_t)k * poly_len + i]);
      }
      *out_len = w.len;
      if (out) require(w.len <= cap, "output buffer too small");
    });
  });
}

int zk_proof_blob_info(const uint8_t* blob, size_t len, int* out_kind, zk_field* out_field, uint32_t* out_nrounds) {
  return guarded([&] {
    require(blob && out_kind && out_field && out_nrounds, "null argument");
    BlobReader r{blob, len};
    *out_kind = blob_open(r, out_field, out_nrounds);
  });
}

int zk_gkr_proof_from_blob(const uint8_t* blob, size_t len, zk_repr repr, zk_fe* out_coeffs, uint8_t* out_ncoeffs,
                           uint32_t cap_rounds, zk_fe* out_claimed_sum) {
  return guarded([&] {
    require(blob && out_claimed_sum, "null argument");
    BlobReader r{blob, len};
    zk_field field;
    uint32_t n;
    require(blob_open(r, &field, &n) == ZK_BLOB_GKR, "not a GKR sum-check proof blob");
    require(n <= cap_rounds && (n == 0 || (out_coeffs && out_ncoeffs)), "output buffer too small");
    dispatch(field, [&](auto f) {
      using F = decltype(f);
      *out_claimed_sum = blob_read_fe<F>(r, repr);
      for (uint32_t k = 0; k < n; ++k) {
        const uint8_t m = *r.take(1);
        require(m <= 3, "round polynomial has more than 3 coefficients");
        out_ncoeffs[k] = m;
        for (int i = 0; i < 3; ++i) out_coeffs[3 * (size_t)k + i] = i < m ? blob_read_fe<F>(r, repr) : zk_fe{};
      }
      require(r.off == len, "trailing bytes after the proof");
    });
  });
}

int zk_sumcheck_proof_from_blob(const uint8_t* blob, size_t len, zk_repr repr, zk_fe* out_round_polys,
                                size_t cap_elems, uint32_t* out_poly_len, zk_fe* out_claimed_sum) {
  return guarded([&] {
    require(blob && out_poly_len && out_claimed_sum, "null argument");
    BlobReader r{blob, len};
    zk_field field;
    uint32_t n;
    require(blob_open(r, &field, &n) == ZK_BLOB_SUMCHECK, "not a sum-check proof blob");
    dispatch(field, [&](auto f) {
      using F = decltype(f);
      *out_claimed_sum = blob_read_fe<F>(r, repr);
      uint32_t plen = 0;
      for (uint32_t k = 0; k < n; ++k) {
        const uint8_t m = *r.take(1);
        require(k == 0 || m == plen, "round polynomials of different lengths");
        plen = m;
        require((size_t)(k + 1) * m <= cap_elems && out_round_polys, "output buffer too small");
        for (uint32_t i = 0; i < m; ++i) out_round_polys[(size_t)k * m + i] = blob_read_fe<F>(r, repr);
      }
      *out_poly_len = plen;
      require(r.off == len, "trailing bytes after the proof");
    });
  });
}

int zk_gkr_verify_blob(const uint8_t* blob, size_t len, zk_transcript* transcript, int* out_verified,
                       zk_fe* out_final_claimed_sum, zk_fe* out_challenges, uint32_t cap_rounds) {
  int rc = ZK_OK;
  const int g = guarded([&] {
    require(blob && transcript && out_verified && out_final_claimed_sum, "null argument");
    BlobReader r{blob, len};
    zk_field field;
    uint32_t n;
    require(blob_open(r, &field, &n) == ZK_BLOB_GKR, "not a GKR sum-check proof blob");
    require(n <= cap_rounds && (n == 0 || out_challenges), "output buffer too small");
    std::vector<zk_fe> cf(3 * (size_t)std::max<uint32_t>(n, 1));
    std::vector<uint8_t> nc(std::max<uint32_t>(n, 1));
    zk_fe cs;
    if (zk_gkr_proof_from_blob(blob, len, ZK_REPR_CANONICAL, cf.data(), nc.data(), n, &cs) != ZK_OK)
      fail(ZK_EINVAL, g_last_error);
    zk_fe dummy;
    rc = zk_gkr_sumcheck_verify(field, ZK_REPR_CANONICAL, cf.data(), nc.data(), n, &cs, transcript, out_verified,
                                out_final_claimed_sum, n ? out_challenges : &dummy);
    if (rc != ZK_OK) fail(rc, g_last_error);
  });
  return g;
}

int zk_keccak256(const uint8_t* data, size_t len, uint8_t out[32]) {
  return guarded([&] {
    require(out && (data || len == 0), "null argument");
    zk::Keccak256 h;
    h.update(data, len);
    h.finalize_reset(out);
  });
}

// ---- device-resident API ----
int zk_dev_alloc(zk_ctx* c, size_t bytes, void** out) {
  return guarded([&] {
    require(c && out, "null argument");
    bind(c);
    *out = nullptr;
    if (hipMalloc(out, bytes ? bytes : 1) != hipSuccess) {
      (void)hipGetLastError();
      *out = nullptr;
      fail(ZK_ENOMEM, "hipMalloc failed");
    }
  });
}
int zk_dev_free(zk_ctx* c, void* p) {
  return guarded([&] {
    require(c, "null ctx");
    bind(c);
    if (p) HIPCK(hipFree(p));
  });
}
int zk_dev_upload(zk_ctx* c, zk_field field, zk_repr repr, const zk_fe* host, size_t n, void* dev) {
  return guarded([&] {
    require(c && (n == 0 || (host && dev)), "null argument");
    bind(c);
    dispatch(field, [&](auto f) {
      using F = decltype(f);
      upload<F>(c, repr, host, n, reinterpret_cast<Fe*>(dev));
    });
  });
}
int zk_dev_download(zk_ctx* c, zk_field field, zk_repr repr, const void* dev, size_t n, zk_fe* host) {
  return guarded([&] {
    require(c && (n == 0 || (host && dev)), "null argument");
    bind(c);
    dispatch(field, [&](auto f) {
      using F = decltype(f);
      download<F>(c, repr, reinterpret_cast<const Fe*>(dev), n, host);
    });
  });
}
int zk_dev_synth_fill(zk_ctx* c, zk_field field, void* dev, uint64_t count, uint64_t seed, uint32_t table,
                      uint64_t index0, uint64_t stride) {
  return guarded([&] {
    require(c && (dev || count == 0), "null argument");
    bind(c);
    dispatch(field, [&](auto f) {
      using F = decltype(f);
      const uint64_t key = zk::splitmix64(zk::splitmix64(seed) + table);
      const uint32_t grid = grid_for(c, count, zk::k_synth<F>);
      launch(c, ZK_K_SYNTH, 32.0 * count, (double)count, zk::k_synth<F>, grid, reinterpret_cast<Fe*>(dev), count, key, index0, stride);
      sync(c);
    });
  });
}
int zk_dev_mle_partial_evaluate(zk_ctx* c, zk_field field, const void* d_in, uint32_t nvars, uint32_t bit,
                                zk_repr repr, const zk_fe* value, void* d_out) {
  return guarded([&] {
    require(c && d_in && d_out && value, "null argument");
    require(nvars >= 1 && bit < nvars, "pair_points underflow panics");
    require(d_in != d_out, "d_out may not alias d_in");
    bind(c);
    dispatch(field, [&](auto f) {
      using F = decltype(f);
      const Fe r = in_mont<F>(repr, *value);
      const uint64_t half = (uint64_t)1 << (nvars - 1);
      const uint32_t grid = grid_for(c, half, zk::k_fold<F>);
      const uint32_t s = nvars - 1 - bit;
      launch(c, ZK_K_FOLD, 96.0 * half, (double)half, zk::k_fold<F>, grid, reinterpret_cast<const Fe*>(d_in), reinterpret_cast<Fe*>(d_out), half, s, r);
      sync(c);
    });
  });
}
int zk_dev_gkr_sumcheck_prove(zk_ctx* c, zk_field field, const void* const d_tables[4], uint32_t nvars,
                              zk_repr repr, const zk_fe* claimed_sum, zk_transcript* transcript, zk_fe* out_coeffs,
                              uint8_t* out_ncoeffs, zk_fe* out_challenges) {
  return guarded([&] {
    require(c && d_tables && transcript && claimed_sum, "null argument");
    require(nvars == 0 || (out_coeffs && out_ncoeffs && out_challenges), "null output");
    for (int t = 0; t < 4; ++t) require(d_tables[t] != nullptr, "null table");
    require(pow2_ok(nvars), "table too large");
    bind(c);
    dispatch(field, [&](auto f) {
      using F = decltype(f);
      (void)in_mont<F>(repr, *claimed_sum);
      const Fe* dT[4];
      for (int t = 0; t < 4; ++t) dT[t] = reinterpret_cast<const Fe*>(d_tables[t]);
      GkrOut g;
      gkr_prove_device<F>(c, dT, nvars, false, transcript, g);
      emit_gkr<F>(repr, g, nvars, out_coeffs, out_ncoeffs, out_challenges);
    });
  });
}

// ---- multi-GPU ----
int zk_ctx_attach_host_comm(zk_ctx* c, int rank, int world, zk_allreduce_u64_fn allreduce, void* user) {
  return guarded([&] {
    require(c && allreduce, "null argument");
    require(world >= 1 && (world & (world - 1)) == 0, "world must be a power of two");
    require(rank >= 0 && rank < world, "rank out of range");
    if (c->nccl) {
      (void)ncclCommDestroy(c->nccl);
      c->nccl = nullptr;
    }
    c->rank = rank;
    c->world = world;
    c->comm = COMM_HOST;
    c->ar = allreduce;
    c->user = user;
  });
}
int zk_comm_get_unique_id(uint8_t out[128]) {
  return guarded([&] {
    require(out, "null argument");
    static_assert(sizeof(ncclUniqueId) == 128, "ncclUniqueId size");
    ncclUniqueId id;
    NCCLCK(ncclGetUniqueId(&id));
    memcpy(out, &id, 128);
  });
}
int zk_ctx_attach_rccl(zk_ctx* c, int rank, int world, const uint8_t unique_id[128]) {
  return guarded([&] {
    require(c && unique_id, "null argument");
    require(world >= 1 && (world & (world - 1)) == 0, "world must be a power of two");
    require(rank >= 0 && rank < world, "rank out of range");
    bind(c);
    if (c->nccl) {
      (void)ncclCommDestroy(c->nccl);
      c->nccl = nullptr;
    }
    ncclUniqueId id;
    memcpy(&id, unique_id, 128);
    NCCLCK(ncclCommInitRank(&c->nccl, world, id, rank));
    c->rank = rank;
    c->world = world;
    c->comm = COMM_RCCL;
  });
}
int zk_ctx_detach_comm(zk_ctx* c) {
  return guarded([&] {
    require(c, "null ctx");
    if (c->nccl) (void)ncclCommDestroy(c->nccl);
    c->nccl = nullptr;
    c->rank = 0;
    c->world = 1;
    c->comm = COMM_NONE;
  });
}
int zk_dev_gkr_sumcheck_prove_sharded(zk_ctx* c, zk_field field, const void* const d_local_tables[4],
                                      uint32_t nvars_local, zk_repr repr, const zk_fe* claimed_sum,
                                      zk_transcript* transcript, zk_fe* out_coeffs, uint8_t* out_ncoeffs,
                                      zk_fe* out_challenges) {
  return guarded([&] {
    require(c && d_local_tables && transcript && claimed_sum && out_coeffs && out_ncoeffs && out_challenges,
            "null argument");
    for (int t = 0; t < 4; ++t) require(d_local_tables[t] != nullptr, "null table");
    require(pow2_ok(nvars_local), "table too large");
    require(c->world == 1 || c->comm != COMM_NONE, "no communicator attached");
    require(c->world <= 256, "world too large for the gather buffers");
    bind(c);
    dispatch(field, [&](auto f) {
      using F = decltype(f);
      (void)in_mont<F>(repr, *claimed_sum);
      const Fe* dT[4];
      for (int t = 0; t < 4; ++t) dT[t] = reinterpret_cast<const Fe*>(d_local_tables[t]);
      GkrOut g;
      gkr_prove_device<F>(c, dT, nvars_local, true, transcript, g);
      uint32_t lg = 0;
      while ((1 << lg) < c->world) ++lg;
      emit_gkr<F>(repr, g, nvars_local + lg, out_coeffs, out_ncoeffs, out_challenges);
    });
  });
}

}  // extern "C"
