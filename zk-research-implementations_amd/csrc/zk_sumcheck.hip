// MI355X-native sum-check / GKR sum-check prover: the C ABI of
// include/zk_sumcheck.h for contexts, the transcript, MultilinearPoly, the
// plain and GKR sum-checks (host and device-resident), and multi-GPU.
//
// Round structure (drivers in host.hpp):
//   GKR  (sum_check_protocol.rs:86-115): round 0 = k_gkr_round0 (e0,e1,e2);
//        round k>=1 = k_gkr_round / k_gkr_round_lanes (fold by r_{k-1} + e0,e2),
//        every round kernel pre-enqueued and waiting in-kernel for its
//        challenge; the last block publishes the limb sums to pinned host
//        memory; host: e1 = s_{k-1}(r_{k-1}) - e0, closed-form interpolation +
//        trim, Keccak absorb, challenge r_k, posted to the next kernel.
//   plain (sum_check_protocol.rs:25-52): k_sc_round (fold + half sums).
// The host side holds only O(1)-per-round scalar work and the transcript;
// every table-sized operation runs on the GPU. Other units: gkr_circuit.hip
// (layered-circuit GKR), kzg.hip (KZG over BLS12-381 G1), blob.hip (proof bytes).
#include "host.hpp"

using namespace zkh;

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
    if (const char* e = getenv("ZK_HOST_PRELAUNCH")) c->host_prelaunch = atoi(e) != 0;
    if (const char* e = getenv("ZK_TAIL")) c->tail = atoi(e) != 0;
    if (const char* e = getenv("ZK_DROUND")) c->dround = atoi(e) != 0;
    if (const char* e = getenv("ZK_DTAIL")) c->dtail = atoi(e) != 0;
    if (const char* e = getenv("ZK_DM")) c->dm = atoi(e) != 0;
    if (const char* e = getenv("ZK_D0T")) c->d0t = atoi(e) != 0;
    if (const char* e = getenv("ZK_DM_MIN_QUADS")) c->dm_min_quads = strtoull(e, nullptr, 0);
    if (const char* e = getenv("ZK_D0")) c->d0 = atoi(e);
    if (const char* e = getenv("ZK_CIRCUIT_DENSE")) c->circuit_dense = atoi(e) != 0;
    if (const char* e = getenv("ZK_CIRCUIT_HOST_LGL")) c->circuit_host_lgl = (uint32_t)strtoul(e, nullptr, 0);
    if (const char* e = getenv("ZK_DTAIL_MAX_QUADS")) c->dtail_max_quads = strtoull(e, nullptr, 0);
    if (const char* e = getenv("ZK_GRID_CAP")) c->grid_cap = (uint32_t)strtoul(e, nullptr, 0);
    if (const char* e = getenv("ZK_ATOMIC_FANIN")) c->atomic_fanin = (uint32_t)strtoul(e, nullptr, 0);
    if (const char* e = getenv("ZK_DTAIL_BLOCKS")) c->dtail_blocks = (uint32_t)strtoul(e, nullptr, 0);
    if (const char* e = getenv("ZK_GATHER_VARS")) c->gather_vars = (uint32_t)strtoul(e, nullptr, 0);
    if (const char* e = getenv("ZK_T33_PIPE")) c->t33_pipe = atoi(e) != 0;
    if (const char* e = getenv("ZK_MSM_BALANCED")) c->msm_balanced = atoi(e) != 0;
    if (const char* e = getenv("ZK_MSM_WIN_TASK")) c->msm_win_task = std::max<uint32_t>(2u, (uint32_t)strtoul(e, nullptr, 0));
    if (const char* e = getenv("ZK_T33_OCT64_MIN")) c->t33_oct64_min = (uint32_t)strtoul(e, nullptr, 0);
    if (const char* e = getenv("ZK_LC_LOADS")) c->lc_loads = (uint32_t)strtoul(e, nullptr, 0) & 7u;
    if (const char* e = getenv("ZK_MALL_ORDER")) c->mall_order = std::min<uint32_t>((uint32_t)strtoul(e, nullptr, 0), 2u);
    if (const char* e = getenv("ZK_HOST_ROUNDS"))  // (<= 8: the tail hands over 4 x 2^(H+2) elements)
      c->host_rounds = std::min<uint32_t>((uint32_t)strtoul(e, nullptr, 0), 8u);
    if (const char* e = getenv("ZK_DEVICE_FS")) c->device_fs = atoi(e) != 0;
    if (const char* e = getenv("ZK_TAIL_MAX_PAIRS")) c->tail_max_pairs = strtoull(e, nullptr, 0);
    c->num_cus = prop.multiProcessorCount;
    try {
      bind(c);
      HIPCK(hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking));
      c->small.ensure(kSmallBytes);
      HIPCK(hipMemset(c->small.p, 0, kSmallBytes));
      HIPCK(hipHostMalloc(reinterpret_cast<void**>(&c->h_red), kHostPage, hipHostMallocMapped | hipHostMallocCoherent));
      memset(c->h_red, 0, kHostPage);
      if (getenv("ZK_DEBUG_TAIL")) {
        HIPCK(hipHostMalloc(reinterpret_cast<void**>(&c->tail_trace), 1024 * 8, hipHostMallocMapped | hipHostMallocCoherent));
        memset(c->tail_trace, 0, 1024 * 8);  // [0, 512): tail kernels, [512, 768): per-step stamps
        if (const char* b = getenv("ZK_DEBUG_BLOCKS")) {
          c->block_trace_step = atoi(b);
          HIPCK(hipHostMalloc(reinterpret_cast<void**>(&c->block_trace), zkh::kBlockTraceMax * 64,
                              hipHostMallocMapped | hipHostMallocCoherent));
          memset(c->block_trace, 0, zkh::kBlockTraceMax * 64);
        }
      }
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
  c->tailbuf.release();
  if (c->tail_trace) (void)hipHostFree(c->tail_trace);
  if (c->block_trace) (void)hipHostFree(c->block_trace);
  c->small.release();
  c->gbuf.release();
  for (auto& b : c->msm) b.release();
  for (auto& b : c->scan_tmp) b.release();
  c->g1_table.release();
  c->g1_table16.release();
  if (c->h_red) (void)hipHostFree(c->h_red);
  if (c->h_tab) (void)hipHostFree(c->h_tab);
  if (c->h_fslog) (void)hipHostFree(c->h_fslog);
  peer_release(c);
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
    c->launch_log.clear();
  });
}
int zk_ctx_get_launches(const zk_ctx* c, zk_launch* out, size_t cap, size_t* n) {
  return guarded([&] {
    require(c && n && (out || cap == 0), "null argument");
    *n = c->launch_log.size();
    for (size_t i = 0; i < cap && i < c->launch_log.size(); ++i) out[i] = c->launch_log[i];
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
int zk_transcript_serialize(const zk_transcript* t, uint8_t* out, size_t cap, size_t* out_len) {
  return guarded([&] {
    require(t && out_len, "null argument");
    *out_len = ZK_TRANSCRIPT_STATE_BYTES;
    require(out && cap >= ZK_TRANSCRIPT_STATE_BYTES, "output buffer smaller than ZK_TRANSCRIPT_STATE_BYTES");
    const uint32_t head[4] = {0x52544b5au /* "ZKTR" */, 1u, (uint32_t)t->h.fill, 0u};
    memcpy(out, head, 16);
    memcpy(out + 16, t->h.st, 200);  // little-endian host: lanes as u64 LE
    memset(out + 216, 0, zk::Keccak256::RATE);
    memcpy(out + 216, t->h.buf, t->h.fill);
  });
}
zk_transcript* zk_transcript_deserialize(const uint8_t* data, size_t len) {
  if (!data || len != ZK_TRANSCRIPT_STATE_BYTES) return nullptr;
  uint32_t head[4];
  memcpy(head, data, 16);
  if (head[0] != 0x52544b5au || head[1] != 1u || head[2] >= zk::Keccak256::RATE || head[3] != 0) return nullptr;
  for (size_t i = 216 + head[2]; i < ZK_TRANSCRIPT_STATE_BYTES; ++i)
    if (data[i]) return nullptr;
  zk_transcript* t = new (std::nothrow) zk_transcript();
  if (!t) return nullptr;
  memcpy(t->h.st, data + 16, 200);
  memcpy(t->h.buf, data + 216, head[2]);
  t->h.fill = head[2];
  return t;
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

// impl Add / Mul / Sub for MultilinearPoly (:113-151): zip -> the shorter table
int zk_mle_binop(zk_ctx* c, zk_field field, zk_repr repr, zk_mle_op op, const zk_fe* a, uint32_t nvars_a,
                 const zk_fe* b, uint32_t nvars_b, zk_fe* out) {
  return guarded([&] {
    require(c && a && b && out, "null argument");
    require(op == ZK_MLE_ADD || op == ZK_MLE_MUL || op == ZK_MLE_SUB, "unknown op");
    require(pow2_ok(nvars_a) && pow2_ok(nvars_b), "table too large");
    bind(c);
    dispatch(field, [&](auto f) {
      using F = decltype(f);
      const uint64_t na = (uint64_t)1 << nvars_a, nb = (uint64_t)1 << nvars_b, n = std::min(na, nb);
      c->input.ensure(2 * n * 32);
      c->work[0].ensure(n * 32);
      upload<F>(c, repr, a, n, c->input.fe());
      upload<F>(c, repr, b, n, c->input.fe() + n);
      const uint32_t grid = grid_for(c, n, zk::k_mle_map<F>);
      launch(c, ZK_K_CONVERT, 96.0 * n, op == ZK_MLE_MUL ? (double)n : 0.0, zk::k_mle_map<F>, grid,
             c->input.fe(), c->input.fe() + n, Fe{}, c->work[0].fe(), n, (uint32_t)op);
      download<F>(c, repr, c->work[0].fe(), n, out);
    });
  });
}

// scale(value) (:93-97)
int zk_mle_scale(zk_ctx* c, zk_field field, zk_repr repr, const zk_fe* evals, uint32_t nvars, const zk_fe* value,
                 zk_fe* out) {
  return guarded([&] {
    require(c && evals && value && out, "null argument");
    require(pow2_ok(nvars), "table too large");
    bind(c);
    dispatch(field, [&](auto f) {
      using F = decltype(f);
      const uint64_t n = (uint64_t)1 << nvars;
      const Fe s = in_mont<F>(repr, *value);
      c->input.ensure(n * 32);
      c->work[0].ensure(n * 32);
      upload<F>(c, repr, evals, n, c->input.fe());
      const uint32_t grid = grid_for(c, n, zk::k_mle_map<F>);
      launch(c, ZK_K_CONVERT, 64.0 * n, (double)n, zk::k_mle_map<F>, grid, c->input.fe(), (const Fe*)nullptr, s,
             c->work[0].fe(), n, (uint32_t)zk::MLE_MUL);
      download<F>(c, repr, c->work[0].fe(), n, out);
    });
  });
}

// tensor_add_mul_polynomials (:99-110); MultilinearPoly::new panics unless the
// product length is a power of two (so both lengths are)
static void check_tensor(zk_mle_op op, uint64_t na, uint64_t nb) {
  require(op == ZK_MLE_ADD || op == ZK_MLE_MUL, "tensor op must be Add or Mul (Operation)");
  require(na >= 1 && nb >= 1, "Invalid evaluations (empty tensor)");
  require((na & (na - 1)) == 0 && (nb & (nb - 1)) == 0, "Invalid evaluations (length not a power of two)");
  require(na <= ((uint64_t)1 << 39) / nb, "table too large");
}

int zk_mle_tensor(zk_ctx* c, zk_field field, zk_repr repr, zk_mle_op op, const zk_fe* a, uint64_t na,
                  const zk_fe* b, uint64_t nb, zk_fe* out) {
  return guarded([&] {
    require(c && a && b && out, "null argument");
    check_tensor(op, na, nb);
    bind(c);
    dispatch(field, [&](auto f) {
      using F = decltype(f);
      const uint64_t n = na * nb;
      c->input.ensure((na + nb) * 32);
      c->work[0].ensure(n * 32);
      upload<F>(c, repr, a, na, c->input.fe());
      upload<F>(c, repr, b, nb, c->input.fe() + na);
      const uint32_t lgb = (uint32_t)__builtin_ctzll(nb);
      const uint32_t grid = grid_for(c, n, zk::k_mle_tensor<F>);
      launch(c, ZK_K_CONVERT, 32.0 * n, op == ZK_MLE_MUL ? (double)n : 0.0, zk::k_mle_tensor<F>, grid,
             c->input.fe(), c->input.fe() + na, c->work[0].fe(), n, lgb, (uint32_t)op);
      download<F>(c, repr, c->work[0].fe(), n, out);
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
int zk_dev_mle_tensor(zk_ctx* c, zk_field field, zk_mle_op op, const void* d_a, uint64_t na, const void* d_b,
                      uint64_t nb, void* d_out) {
  return guarded([&] {
    require(c && d_a && d_b && d_out, "null argument");
    require(d_out != d_a && d_out != d_b, "d_out may not alias an input");
    check_tensor(op, na, nb);
    bind(c);
    dispatch(field, [&](auto f) {
      using F = decltype(f);
      const uint64_t n = na * nb;
      const uint32_t lgb = (uint32_t)__builtin_ctzll(nb);
      const uint32_t grid = grid_for(c, n, zk::k_mle_tensor<F>);
      launch(c, ZK_K_CONVERT, 32.0 * n, op == ZK_MLE_MUL ? (double)n : 0.0, zk::k_mle_tensor<F>, grid,
             reinterpret_cast<const Fe*>(d_a), reinterpret_cast<const Fe*>(d_b), reinterpret_cast<Fe*>(d_out), n,
             lgb, (uint32_t)op);
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
    peer_release(c);  // (a new communicator: the peer buffers are re-attached over it)
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
    peer_release(c);
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
    peer_release(c);
    if (c->nccl) (void)ncclCommDestroy(c->nccl);
    c->nccl = nullptr;
    c->rank = 0;
    c->world = 1;
    c->comm = COMM_NONE;
  });
}
int zk_ctx_comm_count(const zk_ctx* c, int* out_kind, int* out_rank, int* out_count) {
  return guarded([&] {
    require(c && out_kind && out_rank && out_count, "null argument");
    int n = c->world, r = c->rank;
    if (c->comm == COMM_RCCL) {  // what the communicator itself reports
      require(c->nccl != nullptr, "RCCL communicator missing");
      NCCLCK(ncclCommCount(c->nccl, &n));
      NCCLCK(ncclCommUserRank(c->nccl, &r));
    }
    *out_kind = static_cast<int>(c->comm);
    *out_rank = r;
    *out_count = n;
  });
}
int zk_ctx_attach_peer_reduce(zk_ctx* c, int enable, int* out_ok) {
  return guarded([&] {
    require(c, "null ctx");
    if (out_ok) *out_ok = 0;
    bind(c);
    peer_release(c);
    if (!enable) return;
    require(c->comm != COMM_NONE, "attach a communicator first");
    require(c->world <= (int)zk::kPeerMax, "peer reduction joins at most 8 ranks (one node)");
    try {
      peer_attach(c);
    } catch (...) {  // (e.g. the communicator failed mid-attach: nothing half-attached stays behind)
      peer_release(c);
      throw;
    }
    if (out_ok) *out_ok = 1;
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
