// Host-side core shared by the library's translation units (zk_sumcheck.hip,
// gkr_circuit.hip, kzg.hip, blob.hip): errors and the C-ABI guard, field
// dispatch and representation conversion, the transcript, the device context
// (zk_ctx), kernel launch / timing, and the sum-check / GKR round drivers.
#pragma once
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
#include "mfma.hpp"
#include "hfield.hpp"

using zk::Fe;

// ===========================================================================
// errors
// ===========================================================================
namespace zkh {
inline thread_local std::string g_last_error;

struct ZkError {
  int code;
  std::string msg;
};
[[noreturn]] inline void fail(int code, const std::string& msg) { throw ZkError{code, msg}; }

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

inline void require(bool cond, const char* msg) {
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
  const Fe c = zk::hfe_from_mont<F>(m);
  memcpy(out, c.v, 32);
}

}  // namespace zkh
using namespace zkh;

// ===========================================================================
// transcript (fiat_shamir_transcript.rs:5-37)
// ===========================================================================
struct zk_transcript {
  zk::Keccak256 h;
};

namespace zkh {
// get_random_challenge: d = finalize_reset(); append(d); from_le_bytes_mod_order(d)
template <class F>
Fe challenge(zk_transcript* t) {
  uint8_t d[32];
  t->h.finalize_reset(d);
  t->h.update(d, 32);
  Fe x;
  memcpy(x.v, d, 32);
  return zk::hfe_to_mont<F>(x);  // LE integer mod p (2^256 < 6p), Montgomery image
}
template <class F>
void absorb(zk_transcript* t, const Fe* m, size_t n) {  // append(fq_vec_to_bytes(v))
  uint8_t b[32];
  for (size_t i = 0; i < n; ++i) {
    canon_bytes<F>(m[i], b);
    t->h.update(b, 32);
  }
}
}  // namespace zkh
using namespace zkh;

// ===========================================================================
// context
// ===========================================================================
namespace zkh {
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
// a temporary device buffer, freed when it goes out of scope (error paths too)
struct ScopedBuf {
  DevBuf b;
  ScopedBuf() = default;
  ScopedBuf(const ScopedBuf&) = delete;
  ScopedBuf& operator=(const ScopedBuf&) = delete;
  ~ScopedBuf() { b.release(); }
};

enum CommKind { COMM_NONE = 0, COMM_HOST = 1, COMM_RCCL = 2 };
}  // namespace zkh
using namespace zkh;

struct zk_ctx {
  int device = 0;
  int num_cus = 256;
  hipStream_t stream = nullptr;
  DevBuf work[2];  // ping-pong fold workspaces: 4 tables each
  DevBuf input;    // host-API staging (4 tables)
  DevBuf partials;
  DevBuf tailbuf;  // k_gkr_tail: 64 relay slots, then the fresh per-round table regions
  DevBuf small;    // round totals (<= 64 u64) + flag + gather buffers
  uint64_t* h_red = nullptr;  // pinned, device-mapped page (kHostPage): round totals, flag, challenge slots
  uint32_t tag = 0;           // last round tag handed to a kernel
  uint64_t lanes_max_pairs = 1u << 15;  // rounds with <= this many pairs use 8 lanes per pair
  std::chrono::steady_clock::time_point work_t0;  // when the last round result was seen
  bool work_open = false;
  uint32_t timing = 0;  // bit k: time launches of kernel kind k
  zk_stats stats{};
  struct Pending {
    int kind;
    hipEvent_t a, b;
    double bytes;
  };
  std::vector<zk_launch> launch_log;  // event-timed launches since the last stats reset
  std::vector<std::pair<hipEvent_t, hipEvent_t>> ev_free;
  std::vector<Pending> pending;
  // communicator
  int rank = 0, world = 1;
  CommKind comm = COMM_NONE;
  zk_allreduce_u64_fn ar = nullptr;
  bool force_coll = false;  // debug: run the collective path even at world 1 (ZK_FORCE_COLLECTIVES)
  bool prelaunch = true;    // pre-enqueue round kernels (ZK_PRELAUNCH=0 launches each after its challenge)
  bool host_prelaunch = false;  // ... also under a host communicator (ZK_HOST_PRELAUNCH; ranks on distinct devices only)
  bool dround = true;       // two rounds per kernel from round 2 on (ZK_DROUND=0: one round per kernel)
  int d0 = 3;              // (dround, even variable count below 11 or ZK_D0T=0) rounds 0 and 1 from the inputs in one kernel, k_gkr_d0m (ZK_D0; 0 off)
  bool d0t = true;          // nv >= 11: rounds 0-2 in one pass, then steps that fold by three (ZK_D0T)
  bool dm = true;           // double steps with two pending challenges on the matrix cores (k_gkr_dm; ZK_DM=0: k_gkr_dround)
  uint64_t dm_min_quads = 1u << 17;  // ... when they have at least this many quads (ZK_DM_MIN_QUADS; smaller steps are latency-bound: k_gkr_dround)
  bool dtail = true;        // the small double rounds in one persistent kernel (ZK_DTAIL=0: one launch each)
  uint64_t dtail_max_quads = 1u << 10;  // it starts at the first double step with <= this many quads (ZK_DTAIL_MAX_QUADS)
  uint32_t dtail_blocks = 64;           // at most this many blocks (<= 64: atomic fan-in) (ZK_DTAIL_BLOCKS)
  uint32_t gather_vars = 10;  // sharded: gather the tables once <= this many local rounds remain, finish locally (ZK_GATHER_VARS; 0: at the end)
  DevBuf gbuf;                // sharded gather: fold scratch, the one-hot buffer, the interleaved global tables
  bool t33_pipe = true;  // ZK_T33_PIPE (0: off): the 64-octant k_gkr_t33 with a double-buffered image, products interleaved
  // ZK_LC_LOADS: lane-contiguous non-temporal input loads (mfma.hpp ld_half_nt) —
  // bit 0 k_gkr_d0t, bit 1 the first k_gkr_t33 (over the input tables), bit 2 the later 64-octant ones
  uint32_t lc_loads = 7;
  uint32_t mall_order = 0;  // ZK_MALL_ORDER: k_gkr_d0t reads the first k_gkr_t33's chunks grouped, that t33 walks them in reverse; 2: the groups permuted for the second t33 too (mfma.hpp)
  uint32_t t33_oct64_min = 1;  // k_gkr_t33 takes 64-octant chunks from this many chunks per CU (ZK_T33_OCT64_MIN; fewer: 32-octant chunks, twice the chunks; round 6: 4 -> 1, the second pass 2 us faster, profiles/r6_knob_ab.txt)
  uint32_t host_rounds = 4;  // the last <= this many rounds (even) on the host, from tables the persistent tail hands over (ZK_HOST_ROUNDS; 0 off)
  uint64_t* h_tab = nullptr; // pinned, device-mapped: the 4 tables handed to the host rounds
  bool device_fs = false;    // the persistent tail draws its own challenges (ZK_DEVICE_FS; dfs.hpp)
  zk::FsLog* h_fslog = nullptr;  // pinned, device-mapped: 64 records of device-drawn rounds
  size_t h_tab_bytes = 0;
  bool tail = true;         // (ZK_DROUND=0 only) pre-enqueued small rounds in one persistent kernel (ZK_TAIL=0: one launch each)
  bool circuit_dense = false;  // circuit GKR: dense L^2 layer tables instead of the two-phase prover (ZK_CIRCUIT_DENSE)
  uint32_t circuit_host_lgl = 9;  // circuit GKR: layers with tables of <= 2^this entries run on the host (ZK_CIRCUIT_HOST_LGL)
  uint64_t tail_max_pairs = 1u << 15;  // the tail starts at the first round with <= this many pairs (ZK_TAIL_MAX_PAIRS)
  uint64_t* tail_trace = nullptr;      // ZK_DEBUG_TAIL: pinned per-round stamps of the tail kernel, printed per proof
  uint64_t* block_trace = nullptr;     // ZK_DEBUG_BLOCKS=<step>: pinned per-block stamps of that step (needs ZK_DEBUG_TAIL)
  int block_trace_step = -1;
  uint32_t grid_cap = 0;         // ZK_GRID_CAP: at most this many blocks for the grid-striding matrix-core steps (0: resident grid)
  uint32_t atomic_fanin = 1024;  // ZK_ATOMIC_FANIN: grids up to this many blocks fan in through u64 atomics
  uint32_t rtag = 0;        // last tag handed to a pre-enqueued round kernel
  void* user = nullptr;
  ncclComm_t nccl = nullptr;
  // peer reduction (zk_ctx_attach_peer_reduce): the sharded steps' sums meet
  // in the ranks' IPC-mapped receive buffers instead of an RCCL all-reduce
  bool peer = false;
  uint64_t* peer_buf = nullptr;       // our receive buffer (uncached device memory)
  uint64_t* peer_gbuf = nullptr;      // our early-gather receive buffer (uncached): [world][4 x 2^12 Fe], world tags
  std::vector<void*> peer_open;       // the peers' buffers, opened from their IPC handles
  zk::PeerSlots* d_peer = nullptr;    // device copy of the slot table
  uint64_t peer_seq = 0;              // last reduction's sequence tag (the same on every rank)
  // KZG / MSM scratch (grow-only) and the cached fixed-base table of G1
  DevBuf msm[19];
  bool msm_balanced = true;  // ZK_MSM_BALANCED: bucket sums in equal tasks across bucket boundaries (kzg.hip)
  uint32_t msm_win_task = 4;  // ZK_MSM_WIN_TASK: points per task in the window sums' segmented reduction
  DevBuf scan_tmp[4];
  DevBuf g1_table;
  DevBuf g1_table16;  // 16-bit windows (100 MB), built on the device from g1_table
  // (the 20-bit signed-window table, 654 MB, is cached per device for the process: kzg.hip FixedBaseCache)
};


namespace zkh {
// small device area: [0,2048) round sums (<= 256 u64), [2048] input check
// flag, [2560,3712) fan-in counters (9 x 128 B), [4096,6144) limb accumulator
// (<= 256 u64), [6144,6656) single-round relay slots (8 x 64 B), [6656,7168)
// the double-round relay slot, [8192, +64 KiB) all-reduce bounce buffer
// (<= 256 ranks x 256 B), then the tail's 4 local elements and the gathered
// 4 x world tables
constexpr size_t kSmallBytes = 160 * 1024;
constexpr size_t kBlockTraceMax = 8192;  // ZK_DEBUG_BLOCKS: blocks traced
inline uint64_t* d_red(zk_ctx* c) { return reinterpret_cast<uint64_t*>(c->small.p); }
inline uint32_t* d_flag(zk_ctx* c) { return reinterpret_cast<uint32_t*>(reinterpret_cast<char*>(c->small.p) + 2048); }
inline uint32_t* d_counter(zk_ctx* c) { return reinterpret_cast<uint32_t*>(reinterpret_cast<char*>(c->small.p) + 2560); }
inline uint64_t* d_accum(zk_ctx* c) { return reinterpret_cast<uint64_t*>(reinterpret_cast<char*>(c->small.p) + 4096); }
inline char* d_gather(zk_ctx* c) { return reinterpret_cast<char*>(c->small.p) + 8192; }
// pinned, device-mapped host page (8 KiB): [0,2048) round totals, [2048] the
// result flag, [4096,4160) the single-round challenge slot, [4160] the error
// word, [6144,6400) the double-round challenge words
constexpr size_t kHostPage = 8192;
inline uint32_t* h_flag(zk_ctx* c) { return reinterpret_cast<uint32_t*>(reinterpret_cast<char*>(c->h_red) + 2048); }
inline zk::RWait* h_rin(zk_ctx* c) { return reinterpret_cast<zk::RWait*>(reinterpret_cast<char*>(c->h_red) + 4096); }
inline uint32_t* h_err(zk_ctx* c) { return reinterpret_cast<uint32_t*>(reinterpret_cast<char*>(c->h_red) + 4160); }
inline zk::RPost* h_rpost(zk_ctx* c) { return reinterpret_cast<zk::RPost*>(reinterpret_cast<char*>(c->h_red) + 6144); }
inline zk::RWait* d_relay(zk_ctx* c) { return reinterpret_cast<zk::RWait*>(reinterpret_cast<char*>(c->small.p) + 6144); }
inline zk::RPost* d_rpost(zk_ctx* c) { return reinterpret_cast<zk::RPost*>(reinterpret_cast<char*>(c->small.p) + 6656); }
static_assert(6656 + sizeof(zk::RPost) <= 8192 && 6144 + sizeof(zk::RPost) <= kHostPage, "relay slot overlaps");

inline void bind(zk_ctx* c) { HIPCK(hipSetDevice(c->device)); }

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

// Grid of a grid-striding matrix-core step: the resident grid `res`, capped
// by ZK_GRID_CAP (tests: several chunks per block at oracle-checkable sizes),
// but never below `min_blocks`, the count that keeps every block within its
// int32 tile bound (k*ChunksMax in mfma.hpp).
// The grid must fit the partial-sum buffer (ensure_partials): checked here,
// before anything is launched with it.
inline uint32_t step_grid(zk_ctx* c, uint32_t res, uint64_t min_blocks) {
  uint64_t g = res;
  if (c->grid_cap > 0 && g > c->grid_cap) g = c->grid_cap;
  g = std::max<uint64_t>({g, min_blocks, 1});
  if ((g + 8) * zk::kSlotU64 * 8 > c->partials.bytes) fail(ZK_EINVAL, "internal: step grid exceeds the partial-sum buffer");
  return (uint32_t)g;
}

// Launch wrapper: counts algorithmic bytes / multiplications per kernel kind
// and, when timing is on, has the dispatch packet itself record start/stop
// events on c->stream (hipExtLaunchKernelGGL: no extra API calls per launch).
template <class Kern, class... Args>
void launch(zk_ctx* c, int kind, double bytes, double muls, Kern kernel, uint32_t grid, Args... args) {
  zk_ctx::Pending p{kind, nullptr, nullptr, bytes};
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
constexpr size_t kLaunchLogMax = 1 << 16;  // launch_log entries kept (bounded)
// after a stream sync: fold event timings into the stats
inline void flush_timing(zk_ctx* c) {
  static const bool dbg = getenv("ZK_DEBUG_EVENTS") != nullptr;
  for (auto& p : c->pending) {
    float ms = 0.f;
    HIPCK(hipEventElapsedTime(&ms, p.a, p.b));
    if (dbg) fprintf(stderr, "zk: kind %d %.1f us\n", p.kind, ms * 1e3);
    c->stats.kernel_ms[p.kind] += ms;
    if (c->launch_log.size() >= kLaunchLogMax)  // a context timed for a long time keeps the newest launches
      c->launch_log.erase(c->launch_log.begin(), c->launch_log.begin() + kLaunchLogMax / 2);
    c->launch_log.push_back(zk_launch{p.kind, (double)ms, p.bytes});
    c->ev_free.push_back({p.a, p.b});
  }
  c->pending.clear();
}
inline void sync(zk_ctx* c) {
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
inline bool multi_rank(zk_ctx* c) { return (c->world > 1 || c->force_coll) && c->comm != COMM_NONE; }

// Collective timing (ZK_K_COLL): an RCCL collective on the stream is bracketed
// by events when that kind is timed (its duration then joins the launch log
// like a kernel's); a host communicator's callback is host wall time, counted
// under the same condition. `bytes` = what this rank sends.
struct CollTimer {
  zk_ctx* c;
  double bytes;
  zk_ctx::Pending p{ZK_K_COLL, nullptr, nullptr, 0.0};
  std::chrono::steady_clock::time_point t0;
  CollTimer(zk_ctx* cc, double b) : c(cc), bytes(b) {
    p.bytes = b;
    if (c->comm == COMM_RCCL && ((c->timing >> ZK_K_COLL) & 1u)) {
      if (c->ev_free.empty()) {
        hipEvent_t a, e;
        HIPCK(hipEventCreate(&a));
        HIPCK(hipEventCreate(&e));
        c->ev_free.push_back({a, e});
      }
      p.a = c->ev_free.back().first;
      p.b = c->ev_free.back().second;
      c->ev_free.pop_back();
      HIPCK(hipEventRecord(p.a, c->stream));
    }
    t0 = std::chrono::steady_clock::now();
  }
  ~CollTimer() {
    if (p.a) {
      (void)hipEventRecord(p.b, c->stream);
      c->pending.push_back(p);
    } else if (c->comm == COMM_HOST && ((c->timing >> ZK_K_COLL) & 1u)) {  // timed like a kernel kind
      const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
      c->stats.kernel_ms[ZK_K_COLL] += ms;
      if (c->launch_log.size() < kLaunchLogMax) c->launch_log.push_back(zk_launch{ZK_K_COLL, ms, bytes});
    }
    c->stats.launches[ZK_K_COLL] += 1;
    c->stats.alg_bytes[ZK_K_COLL] += bytes;
  }
};

// In-place SUM of n u64 over all ranks (host memory in/out). RCCL runs on the
// ctx stream through a device bounce buffer; a host communicator runs its callback.
inline void allreduce_host(zk_ctx* c, uint64_t* w, size_t n) {
  if (c->comm == COMM_RCCL) {
    uint64_t* d = reinterpret_cast<uint64_t*>(d_gather(c));
    HIPCK(hipMemcpyAsync(d, w, n * 8, hipMemcpyHostToDevice, c->stream));
    {
      CollTimer ct(c, 8.0 * n);
      NCCLCK(ncclAllReduce(d, d, n, ncclUint64, ncclSum, c->nccl, c->stream));
    }
    HIPCK(hipMemcpyAsync(w, d, n * 8, hipMemcpyDeviceToHost, c->stream));
    sync(c);
  } else if (c->comm == COMM_HOST) {
    CollTimer ct(c, 8.0 * n);
    if (c->ar(c->user, w, n) != 0) fail(ZK_ECOMM, "host all-reduce callback failed");
  } else {
    fail(ZK_ECOMM, "no communicator attached");
  }
  c->stats.collectives += 1;
}

// Peer reduction set-up / tear-down (zk_ctx_attach_peer_reduce).
inline void peer_release(zk_ctx* c) {
  if (c->stream) (void)hipStreamSynchronize(c->stream);
  for (void* p : c->peer_open) (void)hipIpcCloseMemHandle(p);
  c->peer_open.clear();
  if (c->d_peer) (void)hipFree(c->d_peer);
  if (c->peer_buf) (void)hipFree(c->peer_buf);
  if (c->peer_gbuf) (void)hipFree(c->peer_gbuf);
  c->d_peer = nullptr;
  c->peer_buf = nullptr;
  c->peer_gbuf = nullptr;
  c->peer = false;
  c->peer_seq = 0;
}

// One reduction of known values (rank g contributes (g + 1)(t + 1) in word t)
// through the same device path as the steps; the host checks the world's sum.
static __global__ void k_peer_check(zk::RoundSink sk) {
  __shared__ zk::LimbScratch<16> sc;
  const uint32_t t = threadIdx.x;
  if (t < 16) sc.tot[t] = (uint64_t)(sk.peer->rank + 1) * (t + 1);
  __syncthreads();
  zk::publish_limbs<16>(sc, sk);
}

// The early gather through the peers: one block copies this rank's slot (n
// u64) into every rank's gather buffer at [rank] with system-scope stores,
// drains, raises its tag there, then waits until every rank's tag has arrived
// in its own buffer (k_interleave then reads it like the communicator's).
static __global__ __launch_bounds__(1024) void k_peer_gather(const zk::PeerSlots* __restrict__ ps, const uint64_t* __restrict__ src,
                                                      uint64_t n, uint64_t seq, uint32_t* err) {
  const uint32_t t = threadIdx.x, W = ps->world, me = ps->rank;
  const uint64_t cap = (uint64_t)4 * (1u << zk::kPeerGatherMaxT) * 4;  // u64 per rank slot
  for (uint32_t r = 0; r < W; ++r) {
    uint64_t* dst = ps->gather[r] + me * cap;
    for (uint64_t i = t; i < n; i += blockDim.x) __hip_atomic_store(dst + i, src[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (t == 0)
    for (uint32_t r = 0; r < W; ++r)
      __hip_atomic_store(ps->gather[r] + W * cap + me, seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  if (t < W) {
    const uint64_t* tag = ps->gather[me] + W * cap + t;
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    while (__hip_atomic_load(tag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != seq) {
      __builtin_amdgcn_s_sleep(1);
      if (__builtin_amdgcn_s_memrealtime() - t0 > zk::kPeerWaitTicks) {
        __hip_atomic_store(err, 2u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        break;
      }
    }
  }
}

// (launched through this non-template wrapper: every unit that includes the kernel uses it)
inline void launch_peer_gather(zk_ctx* c, const void* src, uint64_t n) {
  k_peer_gather<<<1, 1024, 0, c->stream>>>(c->d_peer, reinterpret_cast<const uint64_t*>(src), n, ++c->peer_seq, h_err(c));
  HIPCK(hipGetLastError());
}
inline size_t peer_gather_bytes(int world) {
  return ((size_t)world * 4 * ((size_t)1 << zk::kPeerGatherMaxT) * 4 + zk::kPeerMax) * sizeof(uint64_t);
}
// One attach phase's outcome agreed over the world: true only if
// every rank passed. Every rank calls it at the same points of peer_attach,
// whatever its own outcome, so no rank keeps peer mode (or waits in a peer
// kernel, or in the communicator) while another has dropped out.
inline bool peer_consensus(zk_ctx* c, bool ok) {
  uint64_t bad = ok ? 0 : 1;
  allreduce_host(c, &bad, 1);
  return bad == 0;
}
inline void peer_attach(zk_ctx* c) {
  const size_t bytes = 2 * (size_t)c->world * zk::kPeerSlotU64 * sizeof(uint64_t), gbytes = peer_gather_bytes(c->world);
  constexpr size_t HW = (2 * sizeof(hipIpcMemHandle_t) + 7) / 8;
  std::vector<uint64_t> w(HW * c->world, 0);
  std::string why;
  // phase 1: our buffers and their handles (a rank that fails here still takes
  // part in the exchange, with zero handles, and in the consensus below)
  try {
    HIPCK(hipExtMallocWithFlags(reinterpret_cast<void**>(&c->peer_buf), bytes, hipDeviceMallocUncached));
    HIPCK(hipExtMallocWithFlags(reinterpret_cast<void**>(&c->peer_gbuf), gbytes, hipDeviceMallocUncached));
    HIPCK(hipMemset(c->peer_buf, 0, bytes));
    HIPCK(hipMemset(c->peer_gbuf, 0, gbytes));
    HIPCK(hipDeviceSynchronize());
    hipIpcMemHandle_t h[2];
    HIPCK(hipIpcGetMemHandle(&h[0], c->peer_buf));
    HIPCK(hipIpcGetMemHandle(&h[1], c->peer_gbuf));
    memcpy(&w[HW * c->rank], h, sizeof h);
  } catch (const ZkError& e) {
    why = e.msg;
  }
  allreduce_host(c, w.data(), w.size());  // disjoint slots: the sum is the gather
  zk::PeerSlots ps{};
  ps.world = (uint32_t)c->world;
  ps.rank = (uint32_t)c->rank;
  // phase 2: the peers' buffers
  for (int r = 0; r < c->world && why.empty(); ++r) {
    if (r == c->rank) {
      ps.slot[r] = c->peer_buf;
      ps.gather[r] = c->peer_gbuf;
      continue;
    }
    hipIpcMemHandle_t hr[2];
    memcpy(hr, &w[HW * r], sizeof hr);
    for (int b = 0; b < 2 && why.empty(); ++b) {
      void* p = nullptr;
      const hipError_t e = hipIpcOpenMemHandle(&p, hr[b], hipIpcMemLazyEnablePeerAccess);
      if (e != hipSuccess) {
        (void)hipGetLastError();
        why = std::string("peer reduction: opening rank ") + std::to_string(r) + "'s buffer: " + hipGetErrorString(e);
        break;
      }
      c->peer_open.push_back(p);
      (b == 0 ? ps.slot[r] : ps.gather[r]) = reinterpret_cast<uint64_t*>(p);
    }
  }
  if (why.empty() && (hipMalloc(reinterpret_cast<void**>(&c->d_peer), sizeof ps) != hipSuccess ||
                      hipMemcpy(c->d_peer, &ps, sizeof ps, hipMemcpyHostToDevice) != hipSuccess)) {
    (void)hipGetLastError();
    why = "peer reduction: device slot table";
  }
  if (!peer_consensus(c, why.empty())) {
    peer_release(c);
    fail(ZK_ECOMM, why.empty() ? "peer reduction: another rank could not set up its buffers" : why);
  }
  c->peer = true;
  c->peer_seq = 0;
  // phase 3, the check: the same publish path, a reduction every rank takes part in
  zk::RoundSink sk{};
  sk.host_out = c->h_red;
  sk.host_flag = h_flag(c);
  sk.tag = ++c->tag;
  sk.peer = c->d_peer;
  sk.peer_seq = ++c->peer_seq;
  sk.err = h_err(c);
  __atomic_store_n(h_err(c), 0u, __ATOMIC_RELAXED);
  k_peer_check<<<1, zk::kBlock, 0, c->stream>>>(sk);
  bool ok = hipGetLastError() == hipSuccess && hipStreamSynchronize(c->stream) == hipSuccess;
  const uint32_t err = __atomic_load_n(h_err(c), __ATOMIC_ACQUIRE);
  ok = ok && err == 0 && __atomic_load_n(h_flag(c), __ATOMIC_ACQUIRE) == sk.tag;
  const uint64_t tri = (uint64_t)c->world * (c->world + 1) / 2;
  for (uint64_t t = 0; t < 16 && ok; ++t) ok = __atomic_load_n(c->h_red + t, __ATOMIC_RELAXED) == tri * (t + 1);
  // (tests: ZK_PEER_CHECK_FAIL_RANK=r makes rank r report a failed check, so
  // the world's consensus path runs: every rank must drop peer mode)
  if (const char* fr = getenv("ZK_PEER_CHECK_FAIL_RANK"))
    if (atoi(fr) == c->rank) ok = false;
  if (!peer_consensus(c, ok)) {
    __atomic_store_n(h_err(c), 0u, __ATOMIC_RELAXED);
    peer_release(c);
    fail(ZK_ECOMM, ok ? "peer reduction check: failed on another rank"
                      : (err ? "peer reduction check: a peer never arrived" : "peer reduction check: wrong sums"));
  }
}

inline zk::RoundSink make_sink(zk_ctx* c, bool across_ranks) {
  zk::RoundSink s;
  s.trace = c->tail_trace ? c->tail_trace + 512 : nullptr;  // ZK_DEBUG_TAIL: per-step stamps
  s.btrace = nullptr;
  s.atomic_max = c->atomic_fanin;
  s.partials = reinterpret_cast<uint64_t*>(c->partials.p);
  s.counter = d_counter(c);
  s.accum = d_accum(c);
  s.tag = ++c->tag;
  const bool via_peer = across_ranks && multi_rank(c) && c->peer;
  const bool via_rccl = across_ranks && multi_rank(c) && c->comm == COMM_RCCL && !via_peer;
  s.dev_out = via_rccl ? d_red(c) : nullptr;
  s.host_out = via_rccl ? nullptr : c->h_red;
  s.host_flag = via_rccl ? nullptr : h_flag(c);
  s.peer = via_peer ? c->d_peer : nullptr;
  s.peer_seq = via_peer ? ++c->peer_seq : 0;
  s.err = h_err(c);
  if (via_peer) c->stats.collectives += 1;
  return s;
}

inline void wait_flag(zk_ctx* c, uint32_t tag) {
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
// (Round 6 measured leaving the publish to the next pre-enqueued step kernel's
// block 0 instead of k_publish — one kernel and one boundary fewer per step —
// and removed it: that block's copy then waits behind the step's first loads,
// which every other block issues at entry, and the forced-RCCL proof at world 1
// got 5-8 us slower, profiles/r6_rccl_publish_ab.txt.)
inline void enqueue_reduce(zk_ctx* c, const zk::RoundSink& sk, bool across_ranks, int n) {
  if (across_ranks && multi_rank(c) && c->comm == COMM_RCCL && !c->peer) {
    {
      CollTimer ct(c, 8.0 * n);
      NCCLCK(ncclAllReduce(d_red(c), d_red(c), n, ncclUint64, ncclSum, c->nccl, c->stream));
    }
    c->stats.collectives += 1;
    zk::k_publish<<<1, 256, 0, c->stream>>>(d_red(c), n, c->h_red, h_flag(c), sk.tag);
    HIPCK(hipGetLastError());
  }
}

// product: the limb sums are sums of products of two Montgomery images (R^2
// scale: REDC once); 17-word sums always are, 8-word sums are element sums
// unless the kernel reduced product sums mod p in the block (k_gkr_d0t).
template <class F, int K>
void collect_sums(zk_ctx* c, const zk::RoundSink& sk, bool across_ranks, int L, Fe (&out)[K], bool product = false) {
  const bool multi = across_ranks && multi_rank(c);
  const int n = K * L;
  wait_flag(c, sk.tag);
  if (const uint32_t e = __atomic_load_n(h_err(c), __ATOMIC_ACQUIRE))
    fail(ZK_EDEVICE, e == 2u ? "a peer's sums never arrived (peer reduction, 10 s)"
                             : "a pre-enqueued round kernel waited more than 1 s for its challenge");
  uint64_t w[K * 17 > 17 ? K * 17 : 17];
  for (int i = 0; i < n; i += 8) __builtin_prefetch(c->h_red + i);  // the device wrote these lines: misses in flight together
  for (int i = 0; i < n; ++i) w[i] = __atomic_load_n(c->h_red + i, __ATOMIC_RELAXED);
  if (multi && c->comm == COMM_HOST && !c->peer) {
    CollTimer ct(c, 8.0 * n);
    if (c->ar(c->user, w, n) != 0) fail(ZK_ECOMM, "host all-reduce callback failed");
    c->stats.collectives += 1;
  }
  for (int k = 0; k < K; ++k) out[k] = zk::hlimbs_to_fe<F>(w + L * k, L, L == 17 || product);
}

// Partial-sum slots (one kSlotU64 slot per block; above atomic_fanin the
// grid also writes the 8 shard slots after its last block). Sized, before a
// phase enqueues anything, for the largest grid a step over tables of 2^nv
// elements can launch: a resident grid (<= 8 blocks of 256 threads per CU) or
// the int32-tile minimum of the matrix-core steps (k_gkr_d0t: 2 ceil(2^nv /
// 2^17) blocks; k_gkr_t33, k_gkr_dm3, k_gkr_dm and k_gkr_d0m need fewer).
inline uint64_t max_step_grid(zk_ctx* c, uint32_t nv) {
  const uint64_t tile = nv > 17 ? (uint64_t)2 << (nv - 17) : 2;
  return std::max<uint64_t>((uint64_t)c->num_cus * 8, tile);
}
inline void ensure_partials(zk_ctx* c, uint32_t nv) {
  c->partials.ensure((size_t)(max_step_grid(c, nv) + 8) * zk::kSlotU64 * 8);
}

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
  c[2] = hfe_half<F>(hfe_add<F>(hfe_sub<F>(e0, hfe_add<F>(e1, e1)), e2));
  c[1] = hfe_sub<F>(hfe_sub<F>(e1, e0), c[2]);
  int m = 3;
  while (m > 0 && fe_is_zero<F>(c[m - 1])) --m;
  absorb<F>(tr, c, (size_t)m);
  out.ncoeffs[k] = (uint8_t)m;
  for (int i = 0; i < 3; ++i) out.coeffs[3 * k + i] = i < m ? c[i] : fe_zero<F>();
  r = challenge<F>(tr);
  out.challenges[k] = r;
  // UnivariatePoly::evaluate(r) (:20-26) via Horner — same field value
  return hfe_add<F>(c[0], hfe_mul<F>(r, hfe_add<F>(c[1], hfe_mul<F>(r, c[2]))));
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
  void note() {  // ZK_DEBUG_TAIL: host time from the last result flag to this post
    if (c->tail_trace)
      fprintf(stderr, "zk host: flag -> post %.2f us\n",
              std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - c->work_t0).count());
  }
  void post(const Fe& r, uint32_t tag) {
    note();
    zk::RWait* s = h_rin(c);
    for (int i = 0; i < 8; ++i) __atomic_store_n(&s->r.v[i], r.v[i], __ATOMIC_RELAXED);
    __atomic_store_n(&s->tag, tag, __ATOMIC_RELEASE);
  }
  // the double-round slot: 24 self-tagged words (tag << 32 | limb), any order
  void post2(const Fe& ra, const Fe& rb, const Fe& rab, uint32_t tag) {
    note();
    zk::RPost* s = h_rpost(c);
    const uint64_t t = (uint64_t)tag << 32;
    for (int i = 0; i < 8; ++i) {
      __atomic_store_n(&s->w[i], t | ra.v[i], __ATOMIC_RELAXED);
      __atomic_store_n(&s->w[8 + i], t | rb.v[i], __ATOMIC_RELAXED);
      __atomic_store_n(&s->w[16 + i], t | rab.v[i], __ATOMIC_RELAXED);
    }
  }
  // a fold by three (k_gkr_t33, k_gkr_dm3): the eight eq weights (kernels.hpp block_get_eq8)
  void post8(const Fe (&e)[8], uint32_t tag) {
    note();
    zk::RPost* s = h_rpost(c);
    const uint64_t t = (uint64_t)tag << 32;
    for (int k = 0; k < 8; ++k)
      for (int i = 0; i < 8; ++i) __atomic_store_n(&s->w[8 * k + i], t | e[k].v[i], __ATOMIC_RELAXED);
  }
  // the device-FS tail's first step: also the transcript digest and the claim (dfs.hpp kFsWords)
  void post5(const Fe& ra, const Fe& rb, const Fe& rab, const uint32_t (&dig)[8], const Fe& claim, uint32_t tag) {
    zk::RPost* s = h_rpost(c);
    const uint64_t t = (uint64_t)tag << 32;
    for (int i = 0; i < 8; ++i) {
      __atomic_store_n(&s->w[24 + i], t | dig[i], __ATOMIC_RELAXED);
      __atomic_store_n(&s->w[32 + i], t | claim.v[i], __ATOMIC_RELAXED);
    }
    post2(ra, rb, rab, tag);
  }
  ~PostR() {
    if (done || last == 0) return;
    post(zk::fe_zero<zk::Bn254Fr>(), last);
    Fe z[8];
    for (auto& x : z) x = zk::fe_zero<zk::Bn254Fr>();
    post8(z, last);  // every word of the slot (any step's reader)
    (void)hipStreamSynchronize(c->stream);
  }
};

// Pre-enqueue the rounds of a phase (ZK_PRELAUNCH, default on)? Never with a
// host all-reduce callback (zk_ctx_attach_host_comm): the callback's latency is
// unbounded (a lagging rank would trip the kernels' 1 s challenge guard), and
// ranks that share one device would starve each other — a pre-enqueued step
// spinning on its challenge holds the CUs the other rank's producing kernel
// needs. Each step then launches after its challenge (same proof).
// ZK_HOST_PRELAUNCH=1 keeps pre-enqueue under a host communicator: for callers
// whose ranks each own a device and whose callback answers well inside the
// kernels' 1 s challenge guard (the library cannot see either from here).
inline bool prelaunch(zk_ctx* c, uint32_t nv) {
  return c->prelaunch && nv > 1 && (c->comm != COMM_HOST || c->host_prelaunch);
}

// Run `nv` rounds over 4 device tables of 2^nv elements starting at global
// round k0, as a sequence of steps:
//   round 0        k_gkr_round0: e0, e1, e2 on the input tables;
//   single round i k_gkr_round / k_gkr_round_lanes: fold by r_{i-1}, e0, e2;
//   double (i,i+1) k_gkr_dround: apply the pending challenges, rounds i and
//                  i+1 from one pass (default from round 2 on; an odd count
//                  of remaining rounds puts one single round first);
//   tail           (ZK_DROUND=0) k_gkr_tail: the small rounds in one kernel.
// e1 of every round after the first is derived on the host as
// s_{k-1}(r_{k-1}) - e0, exact because A*S + M*P has degree 2 per variable.
// Pre-enqueued (default): every step (and, across ranks over RCCL, its
// all-reduce + publish) is enqueued before round 0's sums are read; each
// waits in-kernel for the challenges the host posts. On return `cur` holds
// tables of 2^pend elements with the last `pend` challenges not yet applied.
// Small rounds in one persistent kernel (k_gkr_tail, ZK_DROUND=0 only)?
// Pre-enqueued only, and not when each round's sums take an RCCL all-reduce
// on the stream (the kernel would hold the stream).
// (Nor with peer reduction: its steps keep the RCCL schedule.)
inline bool use_tail(zk_ctx* c, bool across_ranks) {
  return c->tail && !(across_ranks && multi_rank(c) && (c->comm == COMM_RCCL || c->peer));
}
constexpr size_t kTailRelayBytes = 64 * sizeof(zk::RPost);  // 64 relay slots (k_gkr_tail: RWait, k_gkr_dtail: RPost)
inline size_t tail_bytes(uint64_t h0) { return kTailRelayBytes + 16 * h0 * sizeof(Fe); }

struct GStep {
  int kind;        // GS_*
  uint32_t i;      // first round (local)
  int np;          // double / dtail: pending challenges at entry (1 or 2)
  uint32_t nd = 0; // dtail: double steps it runs
  bool dfs = false;  // dtail: device-side Fiat-Shamir between its steps (ZK_DEVICE_FS)
};
enum {
  GS_ROUND0 = 0, GS_SINGLE = 1, GS_DOUBLE = 2, GS_TAIL = 3, GS_DTAIL = 4, GS_D0 = 5, GS_D0T = 6, GS_T32 = 7, GS_T33 = 8,
  GS_HOST = 11   // the last rounds on the host, from the tables the persistent tail's last step hands over
};

// Host rounds (ZK_HOST_ROUNDS, default 4; only where the caller does not
// need the final tables, host_ok): a double step on a few-element table is
// one wave's dependent chain of 256-bit multiplies (~7 us) plus a hand-off
// (~5 us), while the host does the same round in about a microsecond. So
// the persistent tail's last device step stores its output tables (4 x
// 2^(H+2) elements, 8 KiB at H = 4) to pinned host memory, and the host folds
// them by that step's two challenges and runs the last H rounds itself — the
// reference's own arithmetic (gkr_prove's loop, sum_check_protocol.rs:86-115,
// with get_round_partial_polynomial_proof_gkr :152-166 and partial_evaluate
// multilinear_polynomial_evaluation.rs:52-63), same field values.
template <class F>
void host_fold(std::vector<Fe> (&T)[4], const Fe& r) {
  for (auto& t : T) {
    const size_t h = t.size() / 2;
    for (size_t j = 0; j < h; ++j) t[j] = zk::hfe_add<F>(t[j], zk::hfe_mul<F>(r, zk::hfe_sub<F>(t[j + h], t[j])));
    t.resize(h);
  }
}
// e0 = sum [A S + M P](lo), e2 = sum [A S + M P](2 hi - lo) over the pairs of the current tables
// (products summed unreduced, one reduction per value)
template <class F>
void host_round_sums(const std::vector<Fe> (&T)[4], Fe& e0, Fe& e2) {
  using namespace zk;
  const size_t h = T[0].size() / 2;
  uint64_t a0[9] = {0}, a2[9] = {0};
  for (size_t j = 0; j < h; ++j) {
    h64::V x2[4];
    for (int t = 0; t < 4; ++t) x2[t] = h64::of(hfe_sub<F>(hfe_add<F>(T[t][j + h], T[t][j + h]), T[t][j]));
    h64::mac_wide(a0, h64::of(T[0][j]), h64::of(T[1][j]));
    h64::mac_wide(a0, h64::of(T[2][j]), h64::of(T[3][j]));
    h64::mac_wide(a2, x2[0], x2[1]);
    h64::mac_wide(a2, x2[2], x2[3]);
  }
  e0 = wide_to_fe<F>(a0);
  e2 = wide_to_fe<F>(a2);
}

// The four tables folded by every challenge of a phase (the multilinear
// extensions at the phase's point), when its last rounds ran on the host.
struct FinalVals {
  Fe v[4];
  bool ok = false;
};

// gather_max > 0 (sharded phases): stop after the first step boundary b with
// nv - b <= gather_max; *stop = b (nv when the phase runs to its end).
// fin: filled (fin->ok) when the phase ends in host rounds — one more host
// fold of the last two entries by the last challenge.
template <class F>
void gkr_phase(zk_ctx* c, const Fe* cur[4], uint32_t nv, uint32_t k0, bool across_ranks, zk_transcript* tr,
               GkrOut& out, Fe& claim, Fe& r, uint32_t& pend, bool host_ok = false, uint32_t gather_max = 0,
               uint32_t* stop = nullptr, FinalVals* fin = nullptr) {
  if (fin) fin->ok = false;
  const uint64_t L = (uint64_t)1 << nv;
  const bool pre = prelaunch(c, nv);
  std::vector<GStep> steps;
  // rounds 0 and 1 in one pass over the inputs (default; same-box A/B at n = 24:
  // BN254 Fr 1.72-1.74 vs 1.82-1.85 ms, BLS12-381 Fr 1.76 vs 1.83 ms)
  // Three rounds per pass (ZK_D0T, nv >= 11): rounds 0-2 over the inputs
  // (k_gkr_d0t), then nt triple steps that fold by the three pending
  // challenges and run three rounds (k_gkr_t33), one two-round step that
  // folds by three (k_gkr_dm3), and double steps (the small ones in the
  // persistent k_gkr_dtail). nt: the largest count leaving an even number
  // R >= 12 of rounds after the triples, else the smallest leaving an even
  // R >= 8 (every matrix-core step needs >= 64 quads / 32 octants).
  // (Measured and removed: triple steps to the end in a persistent MFMA
  // kernel, and rounds 0-3 in the input pass with a fold by four)
  const bool d0t = c->dround && c->d0t && nv >= 11;
  int nt = -1;
  if (d0t)
    for (int k = 0; 3 + 3 * k + 8 <= (int)nv; ++k) {
      const int R = (int)nv - 3 - 3 * k;
      if (R % 2 == 0 && (R >= 12 || nt < 0)) nt = k;
    }
  const bool d0t_doubles = d0t && nt >= 0;
  const bool d0 = !d0t_doubles && c->dround && c->d0 > 0 && nv >= 2 && nv % 2 == 0;
  if (nv >= 1) steps.push_back({d0t_doubles ? GS_D0T : (d0 ? GS_D0 : GS_ROUND0), 0, 0});
  if (d0t_doubles) {
    for (int k = 0; k < nt; ++k) steps.push_back({GS_T33, 3u + 3u * k, 3});
    steps.push_back({GS_T32, 3u + 3u * nt, 3});
  }
  if (c->dround) {
    uint32_t i = d0t_doubles ? 5u + 3u * nt : (d0 ? 2 : 1);
    int np = d0t_doubles || d0 ? 2 : 1;  // challenges pending at the first double step
    if (!d0 && !d0t_doubles) {
      if (nv >= 2) steps.push_back({GS_SINGLE, i++, 0});
      if (nv >= 3 && (nv - 2) % 2 == 1) steps.push_back({GS_SINGLE, i++, 0});
    }
    for (; i + 1 < nv; i += 2, np = 2) steps.push_back({GS_DOUBLE, i, np});
    // host rounds: the last H rounds, if they are whole double steps and the
    // persistent tail keeps >= 2 device steps before them
    // (H = ZK_HOST_ROUNDS, or fewer when that leaves the tail < 2 steps: odd
    // round counts at n = 9, 11 take H = 2)
    uint32_t hostH = 0;
    if (host_ok && pre && c->dtail && use_tail(c, across_ranks) && !(across_ranks && multi_rank(c)) && c->host_rounds >= 2) {
      for (uint32_t H = c->host_rounds & ~1u; H >= 2 && hostH == 0; H -= 2) {
        size_t k = steps.size();
        uint32_t got = 0;
        while (got < H && k > 0 && steps[k - 1].kind == GS_DOUBLE && steps[k - 1].np == 2) {
          --k;
          got += 2;
        }
        size_t smalls = 0;  // device double steps left for the persistent tail
        for (size_t q = 0; q < k; ++q)
          if (steps[q].kind == GS_DOUBLE && (L >> steps[q].i) / 4 <= c->dtail_max_quads) ++smalls;
        if (got == H && smalls >= 2 && k == steps.size() - H / 2) {
          steps.resize(k);
          hostH = H;
        }
      }
    }
    // the small doubles (>= 2 of them) in one persistent kernel
    if (pre && c->dtail && use_tail(c, across_ranks)) {
      size_t d0 = 0;
      while (d0 < steps.size() && !(steps[d0].kind == GS_DOUBLE && (L >> steps[d0].i) / 4 <= c->dtail_max_quads)) ++d0;
      const size_t nd = steps.size() - d0;
      if (d0 < steps.size() && nd >= 2 && nd <= 64) {
        const GStep first = steps[d0];
        steps.resize(d0);
        // device-side Fiat-Shamir between the tail's steps: one rank's sums only
        // (a sharded tail's sums are all-reduced on the host between steps)
        const bool dfs = c->device_fs && !(across_ranks && multi_rank(c));
        steps.push_back({GS_DTAIL, first.i, first.np, (uint32_t)nd, dfs});
        if (dfs && !c->h_fslog) {
          HIPCK(hipHostMalloc(reinterpret_cast<void**>(&c->h_fslog), 64 * sizeof(zk::FsLog),
                              hipHostMallocMapped | hipHostMallocCoherent));
          memset(c->h_fslog, 0, 64 * sizeof(zk::FsLog));
        }
        const uint64_t Q0 = (L >> first.i) / 4;
        const size_t had = c->tailbuf.bytes;
        c->tailbuf.ensure(kTailRelayBytes + zk::dtail_region(Q0, (uint32_t)nd) * sizeof(Fe));
        if (c->tailbuf.bytes != had) HIPCK(hipMemset(c->tailbuf.p, 0, kTailRelayBytes));  // relay tags at rest
      }
    }
    if (hostH > 0) {
      if (steps.empty() || steps.back().kind != GS_DTAIL) fail(ZK_EINVAL, "internal: host rounds need the persistent tail");
      const size_t need = (size_t)4 * ((size_t)1 << (hostH + 2)) * sizeof(Fe);
      if (c->h_tab_bytes < need) {
        if (c->h_tab) HIPCK(hipHostFree(c->h_tab));
        c->h_tab = nullptr;
        c->h_tab_bytes = 0;
        HIPCK(hipHostMalloc(reinterpret_cast<void**>(&c->h_tab), need, hipHostMallocMapped | hipHostMallocCoherent));
        c->h_tab_bytes = need;
      }
      steps.push_back({GS_HOST, nv - hostH, 2});
    }
  } else {
    // first round >= 1 with <= tail_max_pairs pairs, if at least two rounds remain
    uint32_t tail0 = nv;
    if (pre && use_tail(c, across_ranks)) {
      uint32_t i = 1;
      while (i < nv && (L >> i) / 2 > c->tail_max_pairs) ++i;
      if (i + 2 <= nv && nv - i <= 64) {
        tail0 = i;
        const size_t had = c->tailbuf.bytes;
        c->tailbuf.ensure(tail_bytes((L >> i) / 2));  // before anything of this phase is enqueued
        if (c->tailbuf.bytes != had) HIPCK(hipMemset(c->tailbuf.p, 0, kTailRelayBytes));  // relay tags at rest
      }
    }
    for (uint32_t i = 1; i < nv; ++i) {
      if (i == tail0) {
        steps.push_back({GS_TAIL, i, 0});
        break;
      }
      steps.push_back({GS_SINGLE, i, 0});
    }
  }
  auto rounds_of = [&](const GStep& st) -> uint32_t {
    switch (st.kind) {
      case GS_DOUBLE: case GS_D0: case GS_T32: return 2;
      case GS_D0T: case GS_T33: return 3;
      case GS_DTAIL: return 2 * st.nd;
      case GS_TAIL: case GS_HOST: return nv - st.i;
      default: return 1;
    }
  };
  uint32_t end = nv;  // rounds this phase runs
  if (gather_max > 0) {  // sharded: stop at the first boundary leaving <= gather_max rounds (host.hpp gkr_prove_device)
    for (size_t s = 0; s < steps.size(); ++s) {
      const uint32_t b = steps[s].i + rounds_of(steps[s]);
      const int k = steps[s].kind;
      if (k == GS_TAIL || k == GS_DTAIL || k == GS_HOST) break;  // (persistent steps are not cut)
      if (b < nv && nv - b <= gather_max) {
        steps.resize(s + 1);
        end = b;
        break;
      }
    }
  }
  if (stop) *stop = end;
  const size_t ns = steps.size();
  {  // the schedule covers rounds 0 .. end-1 exactly once, in order (checked before anything launches)
    uint32_t next = 0;
    for (const GStep& st : steps) {
      if (st.i != next) fail(ZK_EINVAL, "internal: step schedule out of order");
      next += rounds_of(st);
    }
    if (next != end) fail(ZK_EINVAL, "internal: step schedule does not cover every round");
  }
  // ZK_MALL_ORDER: the input pass groups its chunks by the first 64-octant
  // k_gkr_t33's (16 of its 32-octant chunks per t33 chunk), that t33 takes them
  // in reverse (mfma.hpp k_gkr_d0t / k_gkr_t33 `order`); needs both steps at
  // these positions and the input pass's chunk count a multiple of 16
  const bool oct64_3 = (L >> 6) / 64 >= (uint64_t)c->num_cus * c->t33_oct64_min;   // first t33: 64-octant
  const bool oct64_6 = (L >> 9) / 64 >= (uint64_t)c->num_cus * c->t33_oct64_min;   // second t33: 64-octant
  uint32_t d0t_order = c->mall_order && ns >= 2 && steps[0].kind == GS_D0T && steps[1].kind == GS_T33 &&
                               ((L >> 3) / 32) % 16 == 0 && oct64_3 ? 1u : 0u;
  if (d0t_order && c->mall_order >= 2 && ns >= 3 && steps[2].kind == GS_T33 && oct64_6 && ((L >> 6) / 64) % 8 == 0)
    d0t_order = 2;
  std::vector<zk::RoundSink> sinks(nv);  // per round (a double uses its first round's, a tail one per round)
  std::vector<uint32_t> rtags(ns, 0);    // per step: the (first) challenge tag it waits for
  int inbuf = -1;                        // work buffer holding cur (-1: the input tables)
  Fe rz = zk::fe_zero<F>(), ra = rz, rb = rz;  // last three challenges (oldest first)
  auto out_tables = [&](uint64_t size, Fe* nx[4]) {
    const int ob = inbuf == 0 ? 1 : 0;
    Fe* w = c->work[ob].fe();
    for (int t = 0; t < 4; ++t) nx[t] = w + (uint64_t)t * size;
    inbuf = ob;
  };
  auto enqueue = [&](size_t si) {
    const GStep& st = steps[si];
    if (st.kind == GS_HOST) return;  // no kernel: the host runs these rounds
    const uint32_t i = st.i;
    const uint64_t size = L >> i;  // table length in round i
    const uint64_t h = size / 2;   // pairs
    sinks[i] = make_sink(c, across_ranks);
    if (c->block_trace && (int)si == c->block_trace_step) sinks[i].btrace = c->block_trace;
    const zk::RoundSink& sk = sinks[i];
    if (st.kind == GS_ROUND0) {
      const uint32_t grid = grid_for(c, 2 * h, zk::k_gkr_round0<F>);
      launch(c, ZK_K_GKR_ROUND0, 256.0 * h, 6.0 * h, zk::k_gkr_round0<F>, grid, cur[0], cur[1], cur[2], cur[3], h, sk);
      enqueue_reduce(c, sk, across_ranks, 3 * 17);
      return;
    }
    if (st.kind == GS_D0) {  // rounds 0 and 1 over the input tables (size 4Q), nothing written
      const uint64_t Q = size / 4;
      // products on the matrix cores (k_gkr_d0m, mfma.hpp)
      const uint64_t nch = (Q + 31) / 32;
      const uint32_t res = grid_for(c, nch * zk::kBlock, zk::k_gkr_d0m<F>);
      const uint32_t grid = step_grid(c, res, (nch + 2 * zk::kD0MChunksMax - 1) / (2 * zk::kD0MChunksMax));
      launch(c, ZK_K_GKR_D0, 128.0 * size, 4.5 * size, zk::k_gkr_d0m<F>, grid, cur[0], cur[1], cur[2], cur[3], Q, sk);
      enqueue_reduce(c, sk, across_ranks, zk::kD0Limbs);
      return;
    }
    if (st.kind == GS_D0T) {  // rounds 0, 1, 2 over the input tables (size 8 O), nothing written
      const uint64_t O = size / 8, nch = O / 32;
      const uint32_t res = ((c->lc_loads & 1u) ? grid_for(c, 2 * nch * zk::kBlock, zk::k_gkr_d0t<F, true>)
                                                : grid_for(c, 2 * nch * zk::kBlock, zk::k_gkr_d0t<F>)) & ~1u;
      const uint32_t grid = step_grid(c, res, std::max<uint64_t>(2, 2 * ((nch + zk::kD0TChunksMax - 1) / zk::kD0TChunksMax))) & ~1u;
      const uint32_t order = d0t_order;
      if (c->lc_loads & 1u)
        launch(c, ZK_K_GKR_D0, 128.0 * size, 8.0 * size, zk::k_gkr_d0t<F, true>, grid, cur[0], cur[1], cur[2], cur[3], O, order, sk);
      else
        launch(c, ZK_K_GKR_D0, 128.0 * size, 8.0 * size, zk::k_gkr_d0t<F>, grid, cur[0], cur[1], cur[2], cur[3], O, order, sk);
      enqueue_reduce(c, sk, across_ranks, zk::kD0TLimbs);
      return;
    }
    if (st.kind == GS_T32 || st.kind == GS_T33) {  // fold level i-3 by three challenges to level i
      const uint64_t Q = size / 4;
      Fe* nx[4];
      out_tables(size, nx);
      zk::DIn din{};
      if (pre) {
        din.host = h_rpost(c);
        din.relay = d_rpost(c);
        din.err = h_err(c);
        din.tag = rtags[si] = ++c->rtag;
      } else {
        din.ra = rz;
        din.rb = ra;
        din.rab = rb;  // carries r_{i-1} for this step
      }
      if (st.kind == GS_T33) {  // rounds i .. i+2 over level i's octants: 27 moment sums
        const uint64_t O = size / 8;
        // 64-octant chunks while they still give every CU a chunk, else 32 (twice the blocks)
        if (O / 64 >= (uint64_t)c->num_cus * c->t33_oct64_min) {
          const uint64_t nch = O / 64;
          const uint32_t res = grid_for(c, nch * zk::kBlock, zk::k_gkr_t33<F, 64>);
          const uint32_t grid = step_grid(c, res, (nch + zk::kT33ChunksMax<64> - 1) / zk::kT33ChunksMax<64>);
          const uint32_t order = si == 1 ? d0t_order : 0u;  // (the pass right after an ordered k_gkr_d0t)
          const bool lc = c->t33_pipe && (c->lc_loads & (si == 1 ? 2u : 4u));
          if (lc)
            launch(c, ZK_K_GKR_T33, 9216.0 * O, 96.0 * O, zk::k_gkr_t33<F, 64, true, true>, grid, cur[0], cur[1], cur[2],
                   cur[3], nx[0], nx[1], nx[2], nx[3], O, order, din, sk);
          else if (c->t33_pipe)
            launch(c, ZK_K_GKR_T33, 9216.0 * O, 96.0 * O, zk::k_gkr_t33<F, 64, true>, grid, cur[0], cur[1], cur[2],
                   cur[3], nx[0], nx[1], nx[2], nx[3], O, order, din, sk);
          else
            launch(c, ZK_K_GKR_T33, 9216.0 * O, 96.0 * O, zk::k_gkr_t33<F, 64>, grid, cur[0], cur[1], cur[2], cur[3],
                   nx[0], nx[1], nx[2], nx[3], O, order, din, sk);
        } else {
          const uint64_t nch = O / 32;
          const uint32_t res = grid_for(c, nch * zk::kBlock, zk::k_gkr_t33<F, 32>);
          const uint32_t grid = step_grid(c, res, (nch + zk::kT33ChunksMax<32> - 1) / zk::kT33ChunksMax<32>);
          launch(c, ZK_K_GKR_T33, 9216.0 * O, 96.0 * O, zk::k_gkr_t33<F, 32>, grid, cur[0], cur[1], cur[2], cur[3],
                 nx[0], nx[1], nx[2], nx[3], O, 0u, din, sk);
        }
        for (int t = 0; t < 4; ++t) cur[t] = nx[t];
        enqueue_reduce(c, sk, across_ranks, zk::kD0TLimbs);
        return;
      }
      const uint64_t nch = Q / zk::kDMQuads;
      const uint32_t res = grid_for(c, nch * zk::kBlock, zk::k_gkr_dm3<F>);
      const uint32_t grid = step_grid(c, res, (nch + zk::kDMChunksMax - 1) / zk::kDMChunksMax);
      launch(c, ZK_K_GKR_DM, 4608.0 * Q, 48.0 * Q, zk::k_gkr_dm3<F>, grid, cur[0], cur[1], cur[2], cur[3], nx[0],
             nx[1], nx[2], nx[3], Q, din, sk);
      for (int t = 0; t < 4; ++t) cur[t] = nx[t];
      enqueue_reduce(c, sk, across_ranks, zk::kDLimbs);
      return;
    }
    if (st.kind == GS_TAIL) {
      // rounds i .. nv-1: consecutive sink and challenge tags, fresh table
      // regions in tailbuf (round m: 4 tables of 2 (h >> m) elements)
      const uint32_t nr = nv - i;
      for (uint32_t m = 1; m < nr; ++m) sinks[i + m] = make_sink(c, across_ranks);
      zk::TailArgs a{};
      for (int t = 0; t < 4; ++t) a.in[t] = cur[t];
      a.relay = reinterpret_cast<zk::RWait*>(c->tailbuf.p);
      a.out = reinterpret_cast<Fe*>(reinterpret_cast<char*>(c->tailbuf.p) + kTailRelayBytes);
      a.h0 = h;
      a.nrounds = nr;
      a.host = h_rin(c);
      a.err = h_err(c);
      rtags[si] = c->rtag + 1;
      c->rtag += nr;
      a.rtag0 = rtags[si];
      if (c->tail_trace) a.trace = reinterpret_cast<uint64_t*>(c->tail_trace);
      const uint64_t want = (8 * h + zk::kBlock - 1) / zk::kBlock;
      const uint32_t grid = (uint32_t)std::min<uint64_t>(want, (uint64_t)c->num_cus);  // one block per CU: co-resident
      const double pairs = (double)(2 * h - (h >> (nr - 1)));
      launch(c, ZK_K_GKR_TAIL, 768.0 * pairs, 12.0 * pairs, zk::k_gkr_tail<F>, grid, a, sk);
      const uint64_t hl = h >> (nr - 1);  // pairs of the last round
      Fe* last = a.out + zk::tail_region(h, nr - 1);
      for (int t = 0; t < 4; ++t) cur[t] = last + (uint64_t)t * 2 * hl;
      return;
    }
    if (st.kind == GS_DTAIL) {
      const uint64_t Q0 = size / 4;
      for (uint32_t d = 1; d < st.nd; ++d) sinks[i + 2 * d] = make_sink(c, across_ranks);
      zk::DTailArgs a{};
      for (int t = 0; t < 4; ++t) a.in[t] = cur[t];
      a.relay = reinterpret_cast<zk::RPost*>(c->tailbuf.p);
      a.out = reinterpret_cast<Fe*>(reinterpret_cast<char*>(c->tailbuf.p) + kTailRelayBytes);
      a.Q0 = Q0;
      a.nsteps = st.nd;
      a.np0 = (uint32_t)st.np;
      a.host = h_rpost(c);
      a.err = h_err(c);
      rtags[si] = c->rtag + 1;
      c->rtag += st.nd;
      a.rtag0 = rtags[si];
      if (c->tail_trace) a.trace = c->tail_trace;
      if (si + 1 < ns && steps[si + 1].kind == GS_HOST) a.host_tab = c->h_tab;
      a.fslog = c->h_fslog;
      const uint32_t grid = (uint32_t)std::min<uint64_t>(
          {(Q0 + zk::kDQuads - 1) / zk::kDQuads, (uint64_t)std::min<uint32_t>(c->dtail_blocks, 64u), (uint64_t)c->num_cus});
      double bytes = 0, muls = 0;
      for (uint32_t d = 0; d < st.nd; ++d) {
        const bool two = d > 0 || st.np == 2;
        bytes += (two ? 2560.0 : 1536.0) * (Q0 >> (2 * d));
        muls += (two ? 40.0 : 24.0) * (Q0 >> (2 * d));
      }
      if (st.dfs)
        launch(c, ZK_K_GKR_DTAIL, bytes, muls, zk::k_gkr_dtail<F, true>, std::max<uint32_t>(grid, 1u), a, sk);
      else
        launch(c, ZK_K_GKR_DTAIL, bytes, muls, zk::k_gkr_dtail<F, false>, std::max<uint32_t>(grid, 1u), a, sk);
      const uint64_t Ql = Q0 >> (2 * (st.nd - 1));
      Fe* last = a.out + zk::dtail_region(Q0, st.nd - 1);
      for (int t = 0; t < 4; ++t) cur[t] = last + (uint64_t)t * 4 * Ql;
      return;
    }
    if (st.kind == GS_DOUBLE) {
      // input: level i - np (size << np), output Z: level i (size = 4Q)
      const uint64_t Q = size / 4;
      Fe* nx[4];
      out_tables(size, nx);
      zk::DIn din{};
      if (pre) {
        din.host = h_rpost(c);
        din.relay = d_rpost(c);
        din.err = h_err(c);
        din.tag = rtags[si] = ++c->rtag;
      } else if (st.np == 2) {
        din.ra = ra;
        din.rb = rb;
        din.rab = zk::fe_mul<F>(ra, rb);
      } else {
        din.rb = rb;
      }
      const double bytes = (st.np == 2 ? 2560.0 : 1536.0) * Q, muls = (st.np == 2 ? 40.0 : 24.0) * Q;
      if (st.np == 2 && c->dm && Q >= std::max<uint64_t>(c->dm_min_quads, zk::kDMQuads)) {  // matrix cores (mfma.hpp)
        const uint64_t nch = Q / zk::kDMQuads;
        const uint32_t res = grid_for(c, nch * zk::kBlock, zk::k_gkr_dm<F>);
        const uint32_t grid = step_grid(c, res, (nch + zk::kDMChunksMax - 1) / zk::kDMChunksMax);
        launch(c, ZK_K_GKR_DM, bytes, muls, zk::k_gkr_dm<F>, grid, cur[0], cur[1], cur[2], cur[3], nx[0], nx[1],
               nx[2], nx[3], Q, din, sk);
        for (int t = 0; t < 4; ++t) cur[t] = nx[t];
        enqueue_reduce(c, sk, across_ranks, zk::kDLimbs);
        return;
      }
      const uint32_t grid = st.np == 2 ? grid_for(c, zk::kDQuads * Q, zk::k_gkr_dround<F, 2>)
                                       : grid_for(c, zk::kDQuads * Q, zk::k_gkr_dround<F, 1>);
      if (st.np == 2)
        launch(c, ZK_K_GKR_DROUND, bytes, muls, zk::k_gkr_dround<F, 2>, grid, cur[0], cur[1], cur[2], cur[3], nx[0],
               nx[1], nx[2], nx[3], Q, din, sk);
      else
        launch(c, ZK_K_GKR_DROUND, bytes, muls, zk::k_gkr_dround<F, 1>, grid, cur[0], cur[1], cur[2], cur[3], nx[0],
               nx[1], nx[2], nx[3], Q, din, sk);
      for (int t = 0; t < 4; ++t) cur[t] = nx[t];
      enqueue_reduce(c, sk, across_ranks, zk::kDLimbs);
      return;
    }
    // single round i: fold the previous level (size 2*size) by r_{i-1} and evaluate
    Fe* nx[4];
    out_tables(size, nx);
    zk::RoundIn rin{};
    if (pre) {
      rin.host = h_rin(c);
      rin.relay = d_relay(c);
      rin.err = h_err(c);
      rin.tag = rtags[si] = ++c->rtag;
    } else {
      rin.r = rb;
    }
    if (h <= c->lanes_max_pairs) {  // latency-bound size: 8 lanes per pair
      const uint32_t g8 = grid_for(c, 8 * h, zk::k_gkr_round_lanes<F>);
      launch(c, ZK_K_GKR_LANES, 768.0 * h, 12.0 * h, zk::k_gkr_round_lanes<F>, g8, cur[0], cur[1], cur[2], cur[3], nx[0], nx[1], nx[2], nx[3], h, rin, sk);
    } else {
      const uint32_t grid = grid_for(c, 2 * h, zk::k_gkr_round<F>);
      launch(c, ZK_K_GKR_ROUND, 768.0 * h, 12.0 * h, zk::k_gkr_round<F>, grid, cur[0], cur[1], cur[2], cur[3], nx[0], nx[1], nx[2], nx[3], h, rin, sk);
    }
    for (int t = 0; t < 4; ++t) cur[t] = nx[t];
    enqueue_reduce(c, sk, across_ranks, 2 * 17);
  };
  // the highest challenge tag step si (and every step before it) waits for
  auto last_tag = [&](size_t si) {
    if (steps[si].kind == GS_TAIL) return rtags[si] + (nv - steps[si].i) - 1;
    if (steps[si].kind == GS_DTAIL) return rtags[si] + steps[si].nd - 1;
    return rtags[si];
  };
  PostR post{c};
  if (pre) {
    const auto t0 = std::chrono::steady_clock::now();
    for (size_t si = 0; si < ns; ++si) {
      enqueue(si);
      post.last = last_tag(si);  // from here on the guard releases what is enqueued
    }
    if (getenv("ZK_DEBUG_ENQUEUE"))
      fprintf(stderr, "zk: enqueued %zu steps (%u rounds) in %.1f us\n", ns, nv,
              std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count());
  }
  // hand the newest challenge(s) to step si + 1
  auto hand_on = [&](size_t si) {
    if (!pre || si + 1 >= ns) return;
    const GStep& nx = steps[si + 1];
    if (nx.kind == GS_HOST) return;
    if (nx.kind == GS_T32 || nx.kind == GS_T33) {
      // eq((rz, ra, rb), c), c = 4a + 2b + c0 (rz, the oldest, on the top bit): the
      // fold's eight weights, formed here instead of in every block of the step
      // (five products: ab = eq((rz, ra), (a, b)) from rz ra by differences,
      // then e(ab, c = 1) = ab rb and e(ab, c = 0) = ab - ab rb)
      const Fe one = zk::fe_one<F>();
      Fe ab[4];
      ab[3] = zk::hfe_mul<F>(rz, ra);
      ab[2] = zk::hfe_sub<F>(rz, ab[3]);                          // rz (1 - ra)
      ab[1] = zk::hfe_sub<F>(ra, ab[3]);                          // (1 - rz) ra
      ab[0] = zk::hfe_sub<F>(zk::hfe_sub<F>(one, rz), ab[1]);     // (1 - rz)(1 - ra)
      Fe e[8];
      for (int q = 0; q < 4; ++q) {
        e[2 * q + 1] = zk::hfe_mul<F>(ab[q], rb);
        e[2 * q] = zk::hfe_sub<F>(ab[q], e[2 * q + 1]);
      }
      post.post8(e, rtags[si + 1]);
    } else if (nx.kind == GS_DTAIL && nx.dfs) {
      // the sponge after a challenge is the zero state + its 32-byte digest
      // buffered (dfs.hpp): the device continues the transcript from there
      const zk::Keccak256& h = tr->h;
      bool fresh = h.fill == 32;
      for (int q = 0; q < 25; ++q) fresh = fresh && h.st[q] == 0;
      if (!fresh) fail(ZK_EINVAL, "internal: device Fiat-Shamir needs a transcript right after a challenge");
      uint32_t dig[8];
      memcpy(dig, h.buf, 32);
      const Fe rab = nx.np == 2 ? zk::hfe_mul<F>(ra, rb) : zk::fe_zero<F>();
      post.post5(nx.np == 2 ? ra : zk::fe_zero<F>(), rb, rab, dig, claim, rtags[si + 1]);
    } else if (nx.kind == GS_DOUBLE || nx.kind == GS_DTAIL) {
      if (nx.np == 2)
        post.post2(ra, rb, zk::hfe_mul<F>(ra, rb), rtags[si + 1]);
      else
        post.post2(zk::fe_zero<F>(), rb, zk::fe_zero<F>(), rtags[si + 1]);
    } else {
      post.post(rb, rtags[si + 1]);
    }
  };
  auto one_round = [&](uint32_t i, const Fe& e0, const Fe& e1, const Fe& e2) {
    claim = finish_round<F>(tr, e0, e1, e2, k0 + i, out, r);
    rz = ra;
    ra = rb;
    rb = r;
  };
  // rounds i0, i0 + 1, i0 + 2 from the 27 moment sums of k_gkr_d0t (tile id
  // 9 alpha + 3 beta + gamma per axis: 0 = X0 Y0, 1 = X1 Y1, 2 = X0 Y1 + X1 Y0);
  // X(t) Y(t) = (1-t)^2 m0 + t^2 m1 + t(1-t) ms, so at t = 2 the weights are (1, 4, -2)
  auto three_rounds = [&](uint32_t i0, bool first) {
    Fe T[zk::kD0TCats];
    collect_sums<F, zk::kD0TCats>(c, sinks[i0], across_ranks, 9, T, true);
    using namespace zk;
    const Fe one = fe_one<F>();
    auto at2w = [&](const Fe& m0, const Fe& m1, const Fe& ms) {  // value at t = 2: m0 + 4 m1 - 2 ms
      const Fe m1x2 = hfe_add<F>(m1, m1);
      return hfe_sub<F>(hfe_add<F>(m0, hfe_add<F>(m1x2, m1x2)), hfe_add<F>(ms, ms));
    };
    auto wts = [&](const Fe& t, Fe (&w)[3]) {  // (1-t)^2 = (1-t) - t(1-t), t(1-t) = t - t^2
      w[1] = hfe_mul<F>(t, t);
      w[2] = hfe_sub<F>(t, w[1]);
      w[0] = hfe_sub<F>(hfe_sub<F>(one, t), w[2]);
    };
    Fe U[3];  // round i0: U[alpha] = sum over beta, gamma in {0, 1}
    for (int a = 0; a < 3; ++a)
      U[a] = hfe_add<F>(hfe_add<F>(T[9 * a], T[9 * a + 1]), hfe_add<F>(T[9 * a + 3], T[9 * a + 4]));
    one_round(i0, U[0], first ? U[1] : hfe_sub<F>(claim, U[0]), at2w(U[0], U[1], U[2]));
    Fe wa[3];
    wts(r, wa);
    Fe V[3];  // round i0 + 1: V[beta] = sum_alpha w(ra, alpha) sum_{gamma in {0, 1}}
    for (int b = 0; b < 3; ++b) {
      V[b] = fe_zero<F>();
      for (int a = 0; a < 3; ++a)
        V[b] = hfe_add<F>(V[b], hfe_mul<F>(wa[a], hfe_add<F>(T[9 * a + 3 * b], T[9 * a + 3 * b + 1])));
    }
    one_round(i0 + 1, V[0], hfe_sub<F>(claim, V[0]), at2w(V[0], V[1], V[2]));
    Fe wb[3];
    wts(r, wb);
    Fe Z[3];  // round i0 + 2: Z[gamma] = sum_alpha w(ra, alpha) sum_beta w(rb, beta) T
    for (int g = 0; g < 3; ++g) {
      uint64_t acc[9] = {0};
      for (int a = 0; a < 3; ++a) {
        uint64_t in[9] = {0};
        for (int b = 0; b < 3; ++b) h64::mac_wide(in, h64::of(wb[b]), h64::of(T[9 * a + 3 * b + g]));
        h64::mac_wide(acc, h64::of(wa[a]), h64::of(wide_to_fe<F>(in)));
      }
      Z[g] = wide_to_fe<F>(acc);
    }
    one_round(i0 + 2, Z[0], hfe_sub<F>(claim, Z[0]), at2w(Z[0], Z[1], Z[2]));
  };
  // rounds i0 and i0 + 1 from a double step's eight product sums (the first
  // step of a phase, k_gkr_d0: nine, the ninth V11 for round 0's e1)
  auto two_rounds = [&](uint32_t i0, bool first = false) {
      Fe d[zk::kD0Cats];
      if (first)
        collect_sums<F, zk::kD0Cats>(c, sinks[i0], across_ranks, 17, d);
      else {
        Fe d8[zk::kDCats];
        collect_sums<F, zk::kDCats>(c, sinks[i0], across_ranks, 17, d8);
        std::copy(d8, d8 + zk::kDCats, d);
      }
      // categories: 0 V00, 1 V22, 2 V01, 3 V02, 4 V10, 5 V20, 6 V21, 7 V12, 8 V11 (kernels.hpp)
      // round i: e0 = V00 + V01, e1 = V10 + V11 (first) or s_{i-1}(r_{i-1}) - e0, e2 = V20 + V21
      const Fe e0 = zk::hfe_add<F>(d[0], d[2]);
      const Fe e1 = first ? zk::hfe_add<F>(d[4], d[8]) : zk::hfe_sub<F>(claim, e0);
      one_round(i0, e0, e1, zk::hfe_add<F>(d[5], d[6]));
      // round i + 1 at r = r_i: e0' through (V00, V10, V20), e2' through (V02, V12, V22) at r = 0, 1, 2
      const Fe one = zk::fe_one<F>(), two = zk::hfe_add<F>(one, one);
      const Fe rm1 = zk::hfe_sub<F>(r, one), rm2 = zk::hfe_sub<F>(r, two);
      const Fe L0 = zk::hfe_half<F>(zk::hfe_mul<F>(rm1, rm2));                   // (r-1)(r-2)/2
      const Fe L1 = zk::hfe_sub<F>(zk::fe_zero<F>(), zk::hfe_mul<F>(r, rm2));     // -r(r-2)
      const Fe L2 = zk::hfe_half<F>(zk::hfe_mul<F>(r, rm1));                     // r(r-1)/2
      auto lag = [&](const Fe& v0, const Fe& v1, const Fe& v2) {
        return zk::hfe_add<F>(zk::hfe_add<F>(zk::hfe_mul<F>(L0, v0), zk::hfe_mul<F>(L1, v1)), zk::hfe_mul<F>(L2, v2));
      };
      const Fe f0 = lag(d[0], d[4], d[5]), f2 = lag(d[3], d[7], d[1]);
      one_round(i0 + 1, f0, zk::hfe_sub<F>(claim, f0), f2);
  };
  for (size_t si = 0; si < ns; ++si) {
    const GStep& st = steps[si];
    if (!pre) enqueue(si);
    if (st.kind == GS_ROUND0) {
      Fe s3[3];
      collect_sums<F, 3>(c, sinks[0], across_ranks, 17, s3);
      one_round(0, s3[0], s3[1], s3[2]);
      pend = 1;
    } else if (st.kind == GS_D0) {
      two_rounds(0, true);
      pend = 2;
    } else if (st.kind == GS_D0T) {
      three_rounds(0, true);
      pend = 3;
    } else if (st.kind == GS_T32) {
      two_rounds(st.i);
      pend = 2;
    } else if (st.kind == GS_T33) {
      three_rounds(st.i, false);
      pend = 3;
    } else if (st.kind == GS_SINGLE) {
      Fe s2[2];
      collect_sums<F, 2>(c, sinks[st.i], across_ranks, 17, s2);
      one_round(st.i, s2[0], zk::hfe_sub<F>(claim, s2[0]), s2[1]);
      pend = 1;
    } else if (st.kind == GS_TAIL) {
      for (uint32_t i = st.i; i < nv; ++i) {
        Fe s2[2];
        collect_sums<F, 2>(c, sinks[i], across_ranks, 17, s2);
        one_round(i, s2[0], zk::hfe_sub<F>(claim, s2[0]), s2[1]);
        if (pre && i + 1 < nv) post.post(r, rtags[si] + (i + 1 - st.i));
      }
      pend = 1;
    } else if (st.kind == GS_DOUBLE) {
      two_rounds(st.i);
      pend = 2;
    } else if (st.kind == GS_HOST) {
      // the previous (persistent tail) step's output: level i - 2, 4 tables of
      // 2^(H+2) in h_tab, complete once its flag was seen; fold by r_{i-2}, r_{i-1}
      const auto t0 = std::chrono::steady_clock::now();
      const size_t len = (size_t)1 << (nv - st.i + 2);
      // one bulk copy first: the device wrote these lines, so every host read
      // misses; memcpy keeps many misses in flight, the unpack then hits L1
      std::vector<uint64_t> raw((size_t)16 * len);
      memcpy(raw.data(), c->h_tab, raw.size() * 8);
      const auto t1 = std::chrono::steady_clock::now();
      std::vector<Fe> T[4];
      for (int t = 0; t < 4; ++t) {  // word-major per table (kernels.hpp st_fe_sys)
        const uint64_t* w = raw.data() + (size_t)t * 4 * len;
        T[t].resize(len);
        for (size_t e = 0; e < len; ++e)
          for (int k = 0; k < 4; ++k) {
            const uint64_t x = w[k * len + e];
            T[t][e].v[2 * k] = (uint32_t)x;
            T[t][e].v[2 * k + 1] = (uint32_t)(x >> 32);
          }
      }
      host_fold<F>(T, ra);
      host_fold<F>(T, rb);
      for (uint32_t i = st.i; i < nv; ++i) {
        Fe e0, e2;
        host_round_sums<F>(T, e0, e2);
        one_round(i, e0, zk::hfe_sub<F>(claim, e0), e2);
        if (i + 1 < nv || fin) host_fold<F>(T, r);
      }
      if (fin) {
        for (int t = 0; t < 4; ++t) fin->v[t] = T[t][0];
        fin->ok = true;
      }
      if (c->tail_trace)
        fprintf(stderr, "zk host rounds %u..%u: %.2f us (table copy %.2f us)\n", st.i, nv - 1,
                std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count(),
                std::chrono::duration<double, std::micro>(t1 - t0).count());
      pend = 0;
    } else if (st.dfs) {  // GS_DTAIL, device Fiat-Shamir: steps 0 .. nd-2 drew their own challenges
      // their records are complete once the last step's flag is up (every
      // logging wave drained first, kernels.hpp k_gkr_dtail): replay them into
      // the host transcript — absorb the device's coefficients, draw the
      // challenge, check it against the device's — then finish the last step
      wait_flag(c, sinks[st.i + 2 * (st.nd - 1)].tag);
      for (uint32_t d = 0; d + 1 < st.nd; ++d) {
        const zk::FsLog& lg = c->h_fslog[d];
        if (__atomic_load_n(&lg.tag, __ATOMIC_ACQUIRE) != rtags[si] + d)
          fail(ZK_EDEVICE, "device Fiat-Shamir record missing");
        for (int j = 0; j < 2; ++j) {
          Fe cf[3], rd;
          for (int q = 0; q < 3; ++q) memcpy(cf[q].v, lg.c[j][q], 32);
          memcpy(rd.v, lg.r[j], 32);
          const uint32_t m = lg.m[j];
          if (m > 3) fail(ZK_EDEVICE, "device Fiat-Shamir record corrupt");
          for (uint32_t q = m; q < 3; ++q) cf[q] = zk::fe_zero<F>();
          // the device's interpolation, checked: s(0) + s(1) = 2 c0 + c1 + c2 must be
          // the running claim (a replayed hash alone proves only the replay)
          const Fe s01 = zk::hfe_add<F>(zk::hfe_add<F>(zk::hfe_add<F>(cf[0], cf[0]), cf[1]), cf[2]);
          if (memcmp(s01.v, claim.v, 32) != 0)
            fail(ZK_EDEVICE, "device Fiat-Shamir round polynomial does not match the running claim");
          const uint32_t k = k0 + st.i + 2 * d + j;
          absorb<F>(tr, cf, m);
          out.ncoeffs[k] = (uint8_t)m;
          for (uint32_t q = 0; q < 3; ++q) out.coeffs[3 * k + q] = q < m ? cf[q] : zk::fe_zero<F>();
          r = challenge<F>(tr);
          if (memcmp(r.v, rd.v, 32) != 0) fail(ZK_EDEVICE, "device Fiat-Shamir challenge differs from the host transcript");
          out.challenges[k] = r;
          claim = zk::hfe_add<F>(cf[0], zk::hfe_mul<F>(r, zk::hfe_add<F>(cf[1], zk::hfe_mul<F>(r, cf[2]))));
          c->stats.device_fs_rounds += 1;
          rz = ra;
          ra = rb;
          rb = r;
        }
      }
      two_rounds(st.i + 2 * (st.nd - 1));
      pend = 2;
    } else {  // GS_DTAIL
      for (uint32_t d = 0; d < st.nd; ++d) {
        two_rounds(st.i + 2 * d);
        if (d + 1 < st.nd) post.post2(ra, rb, zk::hfe_mul<F>(ra, rb), rtags[si] + d + 1);
      }
      pend = 2;
    }
    hand_on(si);
  }
  post.done = true;
  if (c->tail_trace) {  // ZK_DEBUG_TAIL: kernel entry, challenge received, publish per step (block 0 / last block)
    HIPCK(hipStreamSynchronize(c->stream));
    const uint64_t* T = c->tail_trace + 512;
    uint64_t prev_pub = 0;
    for (size_t si = 0; si < ns; ++si) {
      if (steps[si].kind == GS_TAIL || steps[si].kind == GS_DTAIL || steps[si].kind == GS_HOST) break;
      const uint64_t* row = T + (sinks[steps[si].i].tag & 63) * 4;
      const bool first = steps[si].kind == GS_ROUND0 || steps[si].kind == GS_D0 || steps[si].kind == GS_D0T;  // no challenge to wait for
      const uint64_t rr = first ? row[0] : row[1];
      fprintf(stderr, "zk step %zu (kind %d, round %u): publish->entry %7.2f us, entry->r %7.2f, r->publish %8.2f"
              " (r->block 0 loop end %8.2f, ->publish %6.2f)\n", si, steps[si].kind, steps[si].i,
              prev_pub ? (row[0] - prev_pub) * 0.01 : 0.0, first ? 0.0 : (row[1] - row[0]) * 0.01, (row[2] - rr) * 0.01,
              row[3] > rr ? (row[3] - rr) * 0.01 : 0.0, row[3] > rr ? ((int64_t)row[2] - (int64_t)row[3]) * 0.01 : 0.0);
      prev_pub = row[2];
      if (c->block_trace && (int)si == c->block_trace_step) {  // ZK_DEBUG_BLOCKS: per-block phases of this step
        std::vector<double> le, ep, ci, fl, wd;
        for (size_t b = 0; b < kBlockTraceMax; ++b) {
          const uint64_t* q = c->block_trace + 8 * b;
          if (!q[0] || !q[1] || !q[2]) continue;
          le.push_back((double)((int64_t)q[0] - (int64_t)rr) * 0.01);
          ep.push_back((double)((int64_t)q[1] - (int64_t)q[0]) * 0.01);
          ci.push_back((double)((int64_t)q[2] - (int64_t)q[1]) * 0.01);
          if (q[4] && q[5]) {
            fl.push_back((double)((int64_t)q[4] - (int64_t)q[0]) * 0.01);
            wd.push_back((double)((int64_t)q[5] - (int64_t)q[4]) * 0.01);
          }
        }
        auto pr = [](const char* what, std::vector<double> v) {
          if (v.empty()) return;
          std::sort(v.begin(), v.end());
          fprintf(stderr, "    %-22s min %8.2f  p10 %8.2f  med %8.2f  p90 %8.2f  max %8.2f us (%zu blocks)\n", what, v.front(),
                  v[v.size() / 10], v[v.size() / 2], v[v.size() * 9 / 10], v.back(), v.size());
        };
        if (const char* fn = getenv("ZK_DEBUG_BLOCKS_FILE")) {  // raw per-block stamps (us after r)
          if (FILE* f = fopen(fn, "w")) {
            fprintf(f, "block,loop_end,fanin_start,counted_in\n");
            for (size_t b = 0; b < kBlockTraceMax; ++b) {
              const uint64_t* q = c->block_trace + 8 * b;
              if (!q[0] || !q[1] || !q[2]) continue;
              fprintf(f, "%zu,%.2f,%.2f,%.2f\n", b, ((int64_t)q[0] - (int64_t)rr) * 0.01, ((int64_t)q[1] - (int64_t)rr) * 0.01,
                      ((int64_t)q[2] - (int64_t)rr) * 0.01);
            }
            fclose(f);
          }
        }
        pr("r -> loop end", le);
        pr("loop end -> epilogue", ep);
        pr("epilogue -> counted in", ci);
        pr("loop end -> flushed", fl);
        pr("flushed -> words", wd);
        memset(c->block_trace, 0, kBlockTraceMax * 64);
      }
    }
  }
  if (c->tail_trace && !steps.empty() && steps.back().kind == GS_TAIL) {  // ZK_DEBUG_TAIL
    HIPCK(hipStreamSynchronize(c->stream));
    const uint64_t* T = c->tail_trace;
    const uint32_t nr = nv - steps.back().i;
    for (uint32_t m = 0; m < nr; ++m)
      fprintf(stderr, "zk tail round %2u: wait r %6.2f us, fold+eval %6.2f, fan-in %6.2f, publish %6.2f, hand-off to next r %6.2f\n",
              m, (T[m * 8 + 1] - T[m * 8]) * 0.01, (T[m * 8 + 2] - T[m * 8 + 1]) * 0.01, (T[m * 8 + 3] - T[m * 8 + 2]) * 0.01,
              (T[m * 8 + 4] - T[m * 8 + 3]) * 0.01, m + 1 < nr ? (T[m * 8 + 9] - T[m * 8 + 4]) * 0.01 : 0.0);
  }
  const size_t sdt = !steps.empty() && steps.back().kind == GS_HOST ? steps.size() - 2 : steps.size() - 1;
  if (c->tail_trace && !steps.empty() && steps[sdt].kind == GS_DTAIL) {  // ZK_DEBUG_TAIL
    HIPCK(hipStreamSynchronize(c->stream));
    const uint64_t* T = c->tail_trace;
    const uint32_t nd = steps[sdt].nd;
    for (uint32_t m = 0; m < nd; ++m)
      fprintf(stderr, "zk dtail step %u: wait r %6.2f us, fold+eval %6.2f, limb sums %6.2f, fan-in %6.2f, publish %6.2f, hand-off to next r %6.2f\n",
              m, (T[m * 8 + 1] - T[m * 8]) * 0.01, (T[m * 8 + 2] - T[m * 8 + 1]) * 0.01, (T[m * 8 + 3] - T[m * 8 + 2]) * 0.01,
              (T[m * 8 + 4] - T[m * 8 + 3]) * 0.01, (T[m * 8 + 5] - T[m * 8 + 4]) * 0.01,
              m + 1 < nd ? (T[m * 8 + 9] - T[m * 8 + 5]) * 0.01 : 0.0);
    for (uint32_t m = 0; m < nd; ++m)  // block 0's fold+eval: constants, loop, store drain
      fprintf(stderr, "zk dtail step %u fold+eval: constants %6.2f us, loop %6.2f, store drain %6.2f\n", m,
              (T[m * 8 + 6] - T[m * 8 + 1]) * 0.01, (T[m * 8 + 7] - T[m * 8 + 6]) * 0.01, (T[m * 8 + 2] - T[m * 8 + 7]) * 0.01);
  }
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
  ensure_partials(c, nloc);
  __atomic_store_n(h_err(c), 0u, __ATOMIC_RELAXED);
  const uint64_t Lloc = (uint64_t)1 << nloc;
  const uint64_t wmax = std::max<uint64_t>(Lloc / 2, (uint64_t)G);
  c->work[0].ensure(4 * wmax * 32);
  c->work[1].ensure(4 * std::max<uint64_t>(wmax / 2, 1) * 32);
  const Fe* cur[4] = {dT[0], dT[1], dT[2], dT[3]};
  Fe claim = zk::fe_zero<F>(), r = zk::fe_zero<F>();
  uint32_t pend = 0;
  uint32_t stop = nloc;
  // the collective path: more than one rank, or (ZK_FORCE_COLLECTIVES with a
  // communicator) one rank through the same code, early gather included
  const bool coll = sharded && (lg > 0 || (c->force_coll && c->comm != COMM_NONE));
  gkr_phase<F>(c, cur, nloc, 0, sharded, tr, out, claim, r, pend, !coll,  // one rank: the final tables are not needed
               coll ? c->gather_vars : 0, &stop);
  if (!coll) {
    sync(c);  // settles event timings; the results are already on the host
    return;
  }
  if (stop < nloc) {
    // ---- early gather: T = nloc - stop local rounds remain. Every rank folds
    // its tables by the pending challenges (r_{stop-pend} .. r_{stop-1}) to 4 x
    // 2^T into its slot of a buffer [G][4][2^T]; ONE collective gathers every
    // rank's slot (RCCL: an in-place ncclAllGather, 4 x 2^T x 32 B sent per
    // rank, 128 KiB at T = 10; a host communicator only offers a SUM
    // all-reduce, so there the buffer is zeroed first and the all-reduce is
    // exact because every word has one nonzero contributor — G times the
    // bytes, a test / diagnostic path), k_interleave lays out the global
    // tables (index m G + g), and every rank runs the last T + lg rounds
    // locally, with no further collective: the small steps, whose latency an
    // all-reduce per step would dominate, run in the persistent tail and on
    // the host exactly as for one GPU. Same rounds, same transcript.
    const uint32_t T = nloc - stop;
    const uint64_t Tn = (uint64_t)1 << T;
    const uint64_t sz = (uint64_t)1 << (T + pend);  // current table length
    const size_t scratch = (size_t)4 * sz, onehot = (size_t)G * 4 * Tn, global = (size_t)4 * G * Tn;
    c->gbuf.ensure((scratch + onehot + global) * sizeof(Fe));
    Fe* sc = reinterpret_cast<Fe*>(c->gbuf.p);
    Fe* oh = sc + scratch;
    Fe* gl = oh + onehot;
    const bool via_peer = c->peer && T <= zk::kPeerGatherMaxT;
    if (c->comm != COMM_RCCL && !via_peer) HIPCK(hipMemsetAsync(oh, 0, onehot * sizeof(Fe), c->stream));
    Fe* slot = oh + (size_t)c->rank * 4 * Tn;
    if (pend == 0) {
      for (int t = 0; t < 4; ++t) HIPCK(hipMemcpyAsync(slot + t * Tn, cur[t], Tn * 32, hipMemcpyDeviceToDevice, c->stream));
    }
    for (uint32_t j = 0; j < pend; ++j) {
      const uint64_t half = sz >> (j + 1);
      Fe* dst = j + 1 == pend ? slot : sc + (j & 1 ? 2 * sz : 0);  // (scratch halves alternate; the last fold lands in the slot)
      const uint64_t dstride = j + 1 == pend ? Tn : half;
      const Fe& rj = out.challenges[stop - pend + j];
      launch(c, ZK_K_FOLD, 4 * half * 96.0, 4.0 * half, zk::k_fold4<F>, grid_for(c, half, zk::k_fold4<F>), cur[0], cur[1],
             cur[2], cur[3], dst, dst + dstride, dst + 2 * dstride, dst + 3 * dstride, half, rj);
      for (int t = 0; t < 4; ++t) cur[t] = dst + t * dstride;
    }
    const Fe* gsrc = oh;
    if (via_peer) {  // through the peers' gather buffers (k_peer_gather)
      const uint64_t cap = (uint64_t)4 * ((uint64_t)1 << zk::kPeerGatherMaxT);  // elements per rank slot
      launch_peer_gather(c, slot, 4 * Tn * 4);
      c->stats.collectives += 1;
      if (cap != 4 * Tn) {  // [G][cap] -> [G][4 Tn]: the layout k_interleave reads
        HIPCK(hipMemcpy2DAsync(oh, 4 * Tn * sizeof(Fe), c->peer_gbuf, cap * sizeof(Fe), 4 * Tn * sizeof(Fe), (size_t)G,
                               hipMemcpyDeviceToDevice, c->stream));
      } else {
        gsrc = reinterpret_cast<const Fe*>(c->peer_gbuf);
      }
    } else if (c->comm == COMM_RCCL) {  // in place: this rank's slot is its send buffer
      CollTimer ct(c, 4.0 * Tn * 32);
      NCCLCK(ncclAllGather(slot, oh, (size_t)4 * Tn * 4, ncclUint64, c->nccl, c->stream));
      c->stats.collectives += 1;
    } else {
      std::vector<uint64_t> w(onehot * 4);
      HIPCK(hipMemcpyAsync(w.data(), oh, onehot * sizeof(Fe), hipMemcpyDeviceToHost, c->stream));
      sync(c);
      allreduce_host(c, w.data(), w.size());
      HIPCK(hipMemcpyAsync(oh, w.data(), onehot * sizeof(Fe), hipMemcpyHostToDevice, c->stream));
      sync(c);  // w (pageable) is released at the end of this block
    }
    launch(c, ZK_K_FOLD, global * 64.0, 0.0, zk::k_interleave<F>, grid_for(c, global, zk::k_interleave<F>), gsrc, gl,
           Tn, (uint32_t)G);
    // (a peer gather slot that never arrives sets the error word: the next
    // step's collect_sums reports it)
    const Fe* gcur[4] = {gl, gl + G * Tn, gl + 2 * G * Tn, gl + 3 * G * Tn};
    gkr_phase<F>(c, gcur, T + lg, stop, false, tr, out, claim, r, pend, true);
    sync(c);
    return;
  }

  // ---- multi-GPU tail: every rank now holds 1 (folded) element per table ----
  // Gather the G x 4 elements with the same exact all-reduce as the rounds:
  // each rank fills only its own slot of a zeroed limb-split vector.
  Fe* send = reinterpret_cast<Fe*>(d_gather(c) + 65536);  // 4 elements, after the bounce buffer
  if (nloc > 0) {
    // the phase ended with pend challenges not applied (cur: 2^pend elements per
    // table): fold by r_{nloc-pend} .. r_{nloc-2} here, by r below
    for (uint32_t k = pend; k > 1; --k) {
      const uint64_t h = (uint64_t)1 << (k - 1);
      Fe* t2 = send + 4 + (k == 3 ? 0 : 16);  // scratch (the staging area below is written after a sync)
      launch(c, ZK_K_FOLD, 8 * h * 96.0, 8.0 * h, zk::k_fold4<F>, 1u, cur[0], cur[1], cur[2], cur[3], t2, t2 + h,
             t2 + 2 * h, t2 + 3 * h, h, out.challenges[nloc - k]);
      for (int t = 0; t < 4; ++t) cur[t] = t2 + h * t;
    }
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
  gkr_phase<F>(c, tcur, lg, nloc, false, tr, out, claim, r, pend);
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
  ensure_partials(c, n);
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
  enqueue(0);
  tr->h.update(table_bytes, nbytes);  // serial Keccak overlaps round 0 on the GPU
  // The later rounds are pre-enqueued only after the hash: a round kernel that
  // waited for its challenge across it would hit the device's 1 s wait guard
  // (the hash of a 24-variable table's 512 MiB takes longer than that).
  if (pre)
    for (uint32_t k = 1; k < n; ++k) {
      enqueue(k);
      post.last = rtags[k];
    }
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

inline bool pow2_ok(uint32_t nvars) { return nvars < 40; }

template <class F>
void emit_gkr(zk_repr repr, const GkrOut& g, uint32_t n, zk_fe* out_coeffs, uint8_t* out_ncoeffs,
              zk_fe* out_challenges) {
  for (uint32_t k = 0; k < n; ++k) {
    out_ncoeffs[k] = g.ncoeffs[k];
    for (int i = 0; i < 3; ++i) out_coeffs[3 * k + i] = out_repr<F>(repr, g.coeffs[3 * k + i]);
    out_challenges[k] = out_repr<F>(repr, g.challenges[k]);
  }
}
}  // namespace zkh
using namespace zkh;
