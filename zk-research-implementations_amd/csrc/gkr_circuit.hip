// GKR over a layered circuit: host driver and C ABI.
#include "host.hpp"

using namespace zkh;

namespace {
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

// One layer's sum-check (2 lgL rounds) in two phases over tables of L = 2^lgL
// entries (kernels.hpp k_phase1_tables / k_phase2_tables): the same round
// polynomials and challenges as gkr_prove over the dense L^2 tables, since
// every round value is the same field sum. Phase 1 binds b (rounds 0 .. lgL-1),
// phase 2 binds c; both phases run the device sum-check of the hot path
// (gkr_phase) on the shared transcript, their last rounds on the host.
// The layer's two evaluations come out of the folds: phase 1's W = w folded by
// r_b is w(r_b), and phase 2's S(c) = w(r_b) + w(c) folded by r_c is
// w(r_b) + w(r_c) (a multilinear extension plus a constant), so ev = {w(r_b),
// w(r_c)} (gkr_protocol.rs:75-76) without another pass over w — when a phase
// ends on the host (FinalVals); otherwise k_mle_eval2 evaluates w.
template <class F>
void gkr_layer_two_phase(zk_ctx* c, const Fe* w, const Fe* wt, const uint8_t* ops, uint32_t lgL, zk_transcript* tr,
                         GkrOut& out, Fe (&ev)[2]) {
  const uint32_t nv = 2 * lgL;
  const uint64_t L = (uint64_t)1 << lgL;
  out.coeffs.assign(3 * (size_t)nv, zk::fe_zero<F>());
  out.ncoeffs.assign(nv, 0);
  out.challenges.assign(nv, zk::fe_zero<F>());
  ensure_partials(c, lgL);
  __atomic_store_n(h_err(c), 0u, __ATOMIC_RELAXED);
  c->work[0].ensure(4 * std::max<uint64_t>(L / 2, 1) * 32);
  c->work[1].ensure(4 * std::max<uint64_t>(L / 4, 1) * 32);
  c->input.ensure(8 * L * 32);
  Fe* t1 = c->input.fe();
  Fe* t2 = t1 + 4 * L;
  const uint32_t blocks = (uint32_t)((L + zk::kBlock - 1) / zk::kBlock);
  launch(c, ZK_K_LAYER, 160.0 * L, 0.5 * L, zk::k_phase1_tables<F>, blocks, w, wt, ops, (uint32_t)L, t1, t1 + L,
         t1 + 2 * L, t1 + 3 * L);
  const Fe* cur[4] = {t1, t1 + L, t1 + 2 * L, t1 + 3 * L};
  Fe claim = zk::fe_zero<F>(), r = zk::fe_zero<F>();
  uint32_t pend = 0;
  FinalVals f1, f2;
  gkr_phase<F>(c, cur, lgL, 0, false, tr, out, claim, r, pend, true, 0, nullptr, &f1);  // rounds 0 .. lgL-1 (b)
  zk::LayerPts ep{};  // r_b, then r_c once phase 2 has drawn it
  for (uint32_t k = 0; k < lgL; ++k) ep.r[k] = ep.r[lgL + k] = out.challenges[k];
  auto eval2 = [&](Fe (&v)[2]) {  // w at ep.r[0..lgL) and ep.r[lgL..2 lgL) on the device
    const zk::RoundSink sk = make_sink(c, false);
    launch(c, ZK_K_LAYER, 32.0 * L, 4.0 * L, zk::k_mle_eval2<F>, grid_for(c, L, zk::k_mle_eval2<F>), w, lgL, ep, sk);
    collect_sums<F, 2>(c, sk, false, 17, v);
  };
  if (f1.ok) {
    ev[0] = f1.v[0];
  } else {
    Fe v[2];
    eval2(v);
    ev[0] = v[0];
  }
  launch(c, ZK_K_LAYER, 160.0 * L, (double)L * (lgL + 2), zk::k_phase2_tables<F>, blocks, w, wt, ops, lgL, ep, ev[0],
         t2, t2 + L, t2 + 2 * L, t2 + 3 * L);
  const Fe* cur2[4] = {t2, t2 + L, t2 + 2 * L, t2 + 3 * L};
  gkr_phase<F>(c, cur2, lgL, lgL, false, tr, out, claim, r, pend, true, 0, nullptr, &f2);  // rounds lgL .. 2 lgL-1 (c)
  if (f2.ok) {
    ev[1] = zk::hfe_sub<F>(f2.v[1], ev[0]);
  } else {
    for (uint32_t k = 0; k < lgL; ++k) ep.r[lgL + k] = out.challenges[lgL + k];
    Fe v[2];
    eval2(v);
    ev[1] = v[1];
  }
  sync(c);
}

// A small layer's sum-check entirely on the host (ZK_CIRCUIT_HOST_LGL): the
// same two phases over the same four tables of L entries as
// gkr_layer_two_phase, the same field values and transcript, with no device
// round trip — on tables of a few hundred entries one host pass per round
// takes microseconds, while each device step waits for a host hand-off. The
// reference's own arithmetic: gkr_prove (sum_check_protocol.rs:86-115) with
// get_round_partial_polynomial_proof_gkr (:152-166) and partial_evaluate
// (multilinear_polynomial_evaluation.rs:52-63); each round's three values are
// summed unreduced and reduced once.
template <class F>
void host_layer_phase(std::vector<Fe> (&T)[4], uint32_t n, uint32_t k0, zk_transcript* tr, GkrOut& out) {
  using namespace zk;
  Fe r;
  for (uint32_t i = 0; i < n; ++i) {
    const size_t h = T[0].size() / 2;
    uint64_t a0[9] = {0}, a1[9] = {0}, a2[9] = {0};
    for (size_t j = 0; j < h; ++j) {
      h64::V x2[4];
      for (int t = 0; t < 4; ++t) x2[t] = h64::of(hfe_sub<F>(hfe_add<F>(T[t][j + h], T[t][j + h]), T[t][j]));
      h64::mac_wide(a0, h64::of(T[0][j]), h64::of(T[1][j]));
      h64::mac_wide(a0, h64::of(T[2][j]), h64::of(T[3][j]));
      h64::mac_wide(a1, h64::of(T[0][j + h]), h64::of(T[1][j + h]));
      h64::mac_wide(a1, h64::of(T[2][j + h]), h64::of(T[3][j + h]));
      h64::mac_wide(a2, x2[0], x2[1]);
      h64::mac_wide(a2, x2[2], x2[3]);
    }
    finish_round<F>(tr, wide_to_fe<F>(a0), wide_to_fe<F>(a1), wide_to_fe<F>(a2), k0 + i, out, r);
    host_fold<F>(T, r);  // (after the last round: the tables at the phase's point, one entry each)
  }
}
// eq(pt, v) for every v < 2^n, bit n-1-k of v against pt[k] (MSB first):
// one product per entry (the table doubles once per coordinate)
template <class F>
std::vector<Fe> host_eq_table(const Fe* pt, uint32_t n) {
  std::vector<Fe> t(1, zk::fe_one<F>());
  for (uint32_t k = 0; k < n; ++k) {
    std::vector<Fe> u(2 * t.size());
    for (size_t j = 0; j < t.size(); ++j) {
      const Fe x = zk::hfe_mul<F>(t[j], pt[k]);
      u[2 * j] = zk::hfe_sub<F>(t[j], x);
      u[2 * j + 1] = x;
    }
    t.swap(u);
  }
  return t;
}
// w = the layer's L inputs, wt = its G gate weights (k_gate_weights), ops its gate ops
// (ev = {w(r_b), w(r_c)} from the folds, as in gkr_layer_two_phase)
template <class F>
void host_layer(const Fe* w, const std::vector<Fe>& wt, const uint8_t* ops, uint32_t lgL, zk_transcript* tr,
                GkrOut& out, Fe (&ev)[2]) {
  using namespace zk;
  const uint32_t nv = 2 * lgL;
  const size_t L = (size_t)1 << lgL;
  out.coeffs.assign(3 * (size_t)nv, fe_zero<F>());
  out.ncoeffs.assign(nv, 0);
  out.challenges.assign(nv, fe_zero<F>());
  std::vector<Fe> T[4];  // phase 1 (kernels.hpp k_phase1_tables): W = w, U, V, 1
  for (auto& t : T) t.assign(L, fe_zero<F>());
  for (size_t b = 0; b < L; ++b) {
    T[0][b] = w[b];
    T[3][b] = fe_one<F>();
    if ((b & 1) == 0) {
      const Fe x = wt[b >> 1], xw = hfe_mul<F>(x, w[b + 1]);
      if (ops[b >> 1]) {
        T[1][b] = xw;
      } else {
        T[1][b] = x;
        T[2][b] = xw;
      }
    }
  }
  host_layer_phase<F>(T, lgL, 0, tr, out);
  const Fe* rb = out.challenges.data();
  const Fe wrb = T[0][0];  // W = w folded by r_b
  for (auto& t : T) t.assign(L, fe_zero<F>());  // phase 2 (k_phase2_tables): A, S, M, P over c
  const std::vector<Fe> eqb = host_eq_table<F>(rb, lgL);
  for (size_t cc = 0; cc < L; ++cc) {
    if (cc & 1) {
      const size_t b = cc - 1;
      const Fe e = hfe_mul<F>(wt[b >> 1], eqb[b]);
      (ops[b >> 1] ? T[2] : T[0])[cc] = e;
    }
    T[1][cc] = hfe_add<F>(wrb, w[cc]);
    T[3][cc] = hfe_mul<F>(wrb, w[cc]);
  }
  host_layer_phase<F>(T, lgL, lgL, tr, out);
  ev[0] = wrb;
  ev[1] = hfe_sub<F>(T[1][0], wrb);  // S = w(r_b) + w(c) folded by r_c
}

template <class F>
void gkr_circuit_prove_device(zk_ctx* c, zk_repr repr, uint32_t nlayers, const uint32_t* gates, const uint8_t* ops,
                              const zk_fe* inputs, uint32_t ninputs, CircuitOut& o) {
  using namespace zk;
  struct Scoped {
    DevBuf b;
    ~Scoped() { b.release(); }
  } vals, dops, dwt;
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
  // layers with tables of <= 2^host_lgl entries run on the host (host_layer); their
  // inputs (the top of vals) come over in one copy
  const uint32_t host_lgl = c->circuit_host_lgl;
  std::vector<Fe> hvals;
  size_t hbase = nvals;
  for (uint32_t l = 0; l < nlayers; ++l)
    if (lg2u(2 * (uint64_t)gates[l]) <= host_lgl) {
      hbase = off[l];
      break;
    }
  if (hbase < nvals) {
    hvals.resize(nvals - hbase);
    HIPCK(hipMemcpyAsync(hvals.data(), vals.b.fe(hbase), hvals.size() * 32, hipMemcpyDeviceToHost, c->stream));
    sync(c);
  }
  static const bool dbg = getenv("ZK_DEBUG_CIRCUIT") != nullptr;
  using clk = std::chrono::steady_clock;
  auto us = [](clk::time_point a, clk::time_point b) { return std::chrono::duration<double, std::micro>(b - a).count(); };
  clk::time_point t0 = clk::now(), t1, t2;
  if (dbg) {
    sync(c);
    fprintf(stderr, "[circuit] evaluate+setup %.1f us\n", us(t0, clk::now()));
  }
  for (uint32_t idx = 0; idx < nlayers; ++idx) {
    if (dbg) t0 = clk::now();
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
    GkrOut g;
    const bool on_host = lgL <= host_lgl && off[l] >= hbase;
    Fe o1, o2, lev[2];
    bool have_ev = false;
    if (on_host) {  // gate weights, both phases and both evaluations on the host
      if (dbg) t1 = clk::now();
      std::vector<Fe> wt(G);
      const std::vector<Fe> eb = host_eq_table<F>(pts.data(), W);
      const std::vector<Fe> ec = has_c ? host_eq_table<F>(pts.data() + W, W) : std::vector<Fe>();
      for (uint32_t gi = 0; gi < G; ++gi) {  // k_gate_weights
        Fe wg = hfe_mul<F>(a, eb[gi]);
        if (has_c) wg = hfe_add<F>(wg, hfe_mul<F>(b, ec[gi]));
        wt[gi] = wg;
      }
      const Fe* hw = hvals.data() + (off[l] - hbase);
      host_layer<F>(hw, wt, ops + opoff[l], lgL, &tr, g, lev);
      if (dbg) t2 = clk::now();
      o1 = lev[0];
      o2 = lev[1];
    }
    LayerPts lp{};
    std::copy(pts.begin(), pts.end(), lp.r);
    if (!on_host)
      launch(c, ZK_K_LAYER, 32.0 * G, (double)G * (W + 2), k_gate_weights<F>, (G + kBlock - 1) / kBlock, lp, W, a, b,
             has_c, G, dwt.b.fe(0));
    if (on_host) {
    } else if (c->circuit_dense) {  // ZK_CIRCUIT_DENSE=1: the four L^2 tables, then the generic sum-check
      c->input.ensure(4 * T * 32);
      Fe* tab = c->input.fe();
      const uint32_t grid = grid_for(c, T, k_layer_tables<F>);
      launch(c, ZK_K_LAYER, 128.0 * T, (double)T, k_layer_tables<F>, grid, w, lgL, dwt.b.fe(0), dop + opoff[l], tab,
             tab + T, tab + 2 * T, tab + 3 * T);
      const Fe* dT[4] = {tab, tab + T, tab + 2 * T, tab + 3 * T};
      if (dbg) {
        sync(c);
        t1 = clk::now();
      }
      gkr_prove_device<F>(c, dT, nv, false, &tr, g);  // gkr_prove(claimed_sum, &fbc_poly, &mut transcript) (:68)
    } else {  // two phases over tables of size L (kernels.hpp k_phase1_tables / k_phase2_tables)
      if (dbg) t1 = clk::now();
      gkr_layer_two_phase<F>(c, w, dwt.b.fe(0), dop + opoff[l], lgL, &tr, g, lev);
      have_ev = true;
    }
    if (dbg) t2 = clk::now();
    for (uint32_t k = 0; k < nv; ++k) {
      for (int i = 0; i < 3; ++i) o.sc.coeffs[3 * (size_t)(k0 + k) + i] = g.coeffs[3 * (size_t)k + i];
      o.sc.ncoeffs[k0 + k] = g.ncoeffs[k];
      o.sc.challenges[k0 + k] = g.challenges[k];
    }
    k0 += nv;
    rb.assign(g.challenges.begin(), g.challenges.begin() + nv / 2);  // (:71-73)
    rc.assign(g.challenges.begin() + nv / 2, g.challenges.end());
    if (have_ev) {  // the two-phase prover's folds (gkr_layer_two_phase)
      o1 = lev[0];
      o2 = lev[1];
    } else if (!on_host) {  // o1 = w.evaluate(r_b), o2 = w.evaluate(r_c) (:75-76): one fused pass
      LayerPts ep{};
      std::copy(rb.begin(), rb.end(), ep.r);
      std::copy(rc.begin(), rc.end(), ep.r + lgL);
      const zk::RoundSink sk = make_sink(c, false);
      launch(c, ZK_K_LAYER, 32.0 * (2 * G), 4.0 * (2 * G), k_mle_eval2<F>, grid_for(c, 2 * (uint64_t)G, k_mle_eval2<F>),
             w, lgL, ep, sk);
      Fe ev[2];
      collect_sums<F, 2>(c, sk, false, 17, ev);
      o1 = ev[0];
      o2 = ev[1];
    }
    if (dbg)
      fprintf(stderr, "[circuit] layer %u nv %u: tables %.1f us, sum-check %.1f us (%.1f/round), evals %.1f us\n", idx,
              nv, us(t0, t1), us(t1, t2), us(t1, t2) / nv, us(t2, clk::now()));
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
                             const uint8_t* ncoeffs, const zk_fe* claims, const zk_fe* input_evals,
                             std::vector<Fe>* last_chal = nullptr) {
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
    if (idx + 1 == nlayers && last_chal) *last_chal = chal;
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

}  // namespace

extern "C" {

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

// ---- gkr::prove / gkr::verify with the input layer's KZG step (gkr_protocol.rs:92-118, :155-175) ----
// A composition of the entry points above: the circuit proof (GPU), then
// KZG::new over the caller's taus (GPU setup), commit (GPU MSM), the two
// openings KZG::open returns (= the input evaluations the circuit prover
// computed at r_b, r_c) and their get_proofs (GPU), and the G2 taus.
int zk_gkr_circuit_prove_kzg(zk_ctx* c, zk_repr repr, uint32_t nlayers, const uint32_t* gates, const uint8_t* ops,
                             const zk_fe* inputs, uint32_t ninputs, const zk_fe* taus, zk_fe* out_output_poly,
                             zk_fe* out_coeffs, uint8_t* out_ncoeffs, zk_fe* out_challenges, zk_fe* out_claims,
                             zk_fe* out_input_evals, zk_g1* out_commitment, zk_g1* out_proofs, zk_g2* out_g2_taus) {
  int rc = guarded([&] {
    require(c && inputs && taus && out_commitment && out_proofs && out_g2_taus && out_challenges, "null argument");
    check_circuit(nlayers, gates, ops, ninputs);
  });
  if (rc != ZK_OK) return rc;
  rc = zk_gkr_circuit_prove(c, ZK_BLS12_381_FR, repr, nlayers, gates, ops, inputs, ninputs, out_output_poly,
                            out_coeffs, out_ncoeffs, out_challenges, out_claims, out_input_evals);
  if (rc != ZK_OK) return rc;
  const uint32_t nin = lg2u(ninputs);
  const uint32_t total = circuit_rounds(nlayers, gates);
  const zk_fe* rb = out_challenges + (total - 2 * nin);  // the input layer's sum-check: (r_b, r_c) (:71-73)
  const zk_fe* rcp = rb + nin;
  zk_kzg* k = nullptr;
  rc = zk_kzg_setup(c, repr, taus, nin, &k);  // KZG::new(&input_poly, taus) (:105)
  if (rc == ZK_OK) rc = zk_kzg_commit(c, k, repr, inputs, out_commitment);  // :106
  if (rc == ZK_OK) rc = zk_kzg_get_proof(c, k, repr, inputs, &out_input_evals[0], rb, out_proofs);  // :108-110
  if (rc == ZK_OK) rc = zk_kzg_get_proof(c, k, repr, inputs, &out_input_evals[1], rcp, out_proofs + nin);  // :112-113
  if (rc == ZK_OK) rc = zk_kzg_g2_taus(k, out_g2_taus);
  zk_kzg_free(k);
  return rc;
}

int zk_gkr_circuit_verify_kzg(zk_repr repr, uint32_t nlayers, const uint32_t* gates, const uint8_t* ops,
                              const zk_fe* output_poly, const zk_fe* coeffs, const uint8_t* ncoeffs,
                              const zk_fe* claims, const zk_fe* opened_evals, const zk_g1* commitment,
                              const zk_g1* proofs, const zk_g2* g2_taus, int* out_verified) {
  std::vector<zk::Fe> chal;
  uint32_t ninputs = 0;
  int rc = guarded([&] {
    require(output_poly && coeffs && ncoeffs && opened_evals && commitment && proofs && g2_taus && out_verified,
            "null argument");
    require(nlayers >= 1 && gates, "null argument");
    ninputs = 2 * gates[0];
    check_circuit(nlayers, gates, ops, ninputs);
    require(nlayers == 1 || claims, "null argument");
    *out_verified = gkr_circuit_verify_host<zk::Bls12_381Fr>(repr, nlayers, gates, ops, nullptr, ninputs, output_poly,
                                                         coeffs, ncoeffs, claims, opened_evals, &chal)
                        ? 1
                        : 0;
  });
  if (rc != ZK_OK || !*out_verified) return rc;
  // KZG::verify of both openings at (r_b, r_c), the verifier's own challenges (:155-175)
  const uint32_t nin = lg2u(ninputs);
  if (chal.size() != 2 * (size_t)nin) {  // the sum-check failed before the input layer
    *out_verified = 0;
    return ZK_OK;
  }
  std::vector<zk_fe> pts(2 * (size_t)nin);
  for (size_t i = 0; i < pts.size(); ++i) pts[i] = out_repr<zk::Bls12_381Fr>(repr, chal[i]);
  int okb = 0, okc = 0;
  rc = zk_kzg_verify(repr, commitment, &opened_evals[0], proofs, nin, pts.data(), nin, g2_taus, &okb);
  if (rc == ZK_OK) rc = zk_kzg_verify(repr, commitment, &opened_evals[1], proofs + nin, nin, pts.data() + nin, nin,
                                      g2_taus, &okc);
  *out_verified = rc == ZK_OK && okb && okc;
  return rc;
}

}  // extern "C"
