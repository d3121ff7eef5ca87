/*
 * zk_sumcheck.h — C ABI of the MI355X-native sum-check / GKR sum-check prover.
 *
 * Drop-in boundary for the reference crates `sum_check`, `multilinear_polynomial`
 * and `fiat_shamir` (obah/zk-research-implementations). Each entry point names
 * the Rust item it replaces (paths relative to the reference root). The
 * reference is generic over `F: PrimeField`; here the field is a runtime
 * `zk_field` and elements are 32-byte little-endian 4 x u64 limbs, either
 * canonical (what `fq_vec_to_bytes` serialises) or Montgomery (ark-ff 0.5.0's
 * in-memory `Fp<MontBackend<_,4>,4>`, R = 2^256), selected per call by
 * `zk_repr` so a Rust shim can pass `Vec<F>` memory directly.
 *
 * Conventions
 *  - every function returns ZK_OK (0) or an error code; where the reference
 *    would `panic!` (non-power-of-two tables, mismatched sizes, wrong number of
 *    evaluation points) the call returns ZK_EINVAL and writes nothing else;
 *  - verification failures are NOT errors: they return ZK_OK with
 *    *out_verified = 0, exactly as the reference returns `false`;
 *  - host buffers are caller-owned; `zk_dev_*` calls take HIP device pointers
 *    holding Montgomery elements (32 B each, 16-B aligned);
 *  - a zk_ctx is bound to one HIP device and is not thread-safe: one per
 *    host thread. All calls are synchronous on return;
 *  - compute runs on the GPU only. A ctx cannot be created without a usable
 *    gfx950 device (ZK_EDEVICE); there is no CPU fallback.
 */
#ifndef ZK_SUMCHECK_H
#define ZK_SUMCHECK_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define ZK_ABI_VERSION 15u

typedef enum { ZK_BN254_FR = 0, ZK_BN254_FQ = 1, ZK_BLS12_381_FR = 2 } zk_field;
typedef enum { ZK_REPR_CANONICAL = 0, ZK_REPR_MONTGOMERY = 1 } zk_repr;

/* One field element: 4 x u64, little-endian limbs. */
typedef struct {
  uint64_t limb[4];
} zk_fe;

enum {
  ZK_OK = 0,
  ZK_EINVAL = 1,       /* reference would panic / bad argument */
  ZK_EDEVICE = 2,      /* HIP error or no usable device */
  ZK_ECOMM = 3,        /* collective failed */
  ZK_ENOMEM = 4,       /* device or host allocation failed */
  ZK_EUNSUPPORTED = 5  /* valid request outside what this build implements */
};

typedef struct zk_ctx zk_ctx;
typedef struct zk_transcript zk_transcript;

uint32_t zk_abi_version(void);
/* Message describing the last failing call on this host thread ("" if none). */
const char* zk_last_error(void);

/* ---------------------------------------------------------------------------
 * Context: HIP device + stream + device workspace (+ optional communicator).
 * ------------------------------------------------------------------------- */
int zk_ctx_create(int device, zk_ctx** out);
void zk_ctx_destroy(zk_ctx* ctx);

/* Per-kernel-kind counters; timing (HIP events around every launch on the
 * ctx stream) is collected only while enabled. */
enum {
  ZK_K_GKR_ROUND0 = 0, /* first GKR round: e0,e1,e2 over the input tables */
  ZK_K_GKR_ROUND = 1,  /* fused fold-by-r + next-round e0,e2 over 4 tables (k_gkr_round) */
  ZK_K_SC_ROUND = 2,   /* plain sum-check: (fold) + half sums */
  ZK_K_FOLD = 3,       /* MultilinearPoly::partial_evaluate */
  ZK_K_REDUCE = 4,     /* block partials -> limb-split sums */
  ZK_K_CONVERT = 5,    /* canonical <-> Montgomery */
  ZK_K_SYNTH = 6,      /* synthetic table generator */
  ZK_K_LAYER = 7,      /* GKR circuit: layer evaluation, gate weights, layer tables */
  ZK_K_MSM = 8,        /* KZG: bucket sort, bucket/window sums, fixed-base setup, normalisation */
  ZK_K_GKR_LANES = 9,  /* the same round for small tables, 8 lanes per pair (k_gkr_round_lanes) */
  ZK_K_GKR_TAIL = 10,  /* the small rounds of a proof in one persistent kernel (k_gkr_tail, ZK_DROUND=0) */
  ZK_K_GKR_DROUND = 11, /* two rounds per kernel: pending folds + round sums + next round's quadratics (k_gkr_dround) */
  ZK_K_GKR_DTAIL = 12, /* the small double rounds in one persistent kernel (k_gkr_dtail) */
  ZK_K_GKR_D0 = 13,    /* the input pass: rounds 0-2 (k_gkr_d0t) or rounds 0 and 1 (k_gkr_d0m), on the matrix cores */
  ZK_K_GKR_DM = 14,    /* two-round steps on the matrix cores that fold by two or three challenges (k_gkr_dm, k_gkr_dm3) */
  ZK_K_GKR_T33 = 15,   /* three-round steps on the matrix cores: fold by three + 27 moment sums (k_gkr_t33) */
  ZK_K_COLL = 16,      /* collectives of a sharded proof: RCCL all-reduce / all-gather (event-timed on the stream
                          when timing is on), or the host communicator's callback (host wall time, always) */
  ZK_K_KINDS = 17
};
typedef struct {
  uint64_t launches[ZK_K_KINDS];
  double kernel_ms[ZK_K_KINDS];  /* sum of event-timed durations */
  double alg_bytes[ZK_K_KINDS];  /* algorithmic HBM bytes */
  double field_muls[ZK_K_KINDS]; /* Montgomery multiplications issued */
  uint64_t host_syncs;           /* device->host round trips */
  uint64_t collectives;          /* all-reduce calls */
  double host_wait_us;           /* host time spent waiting for round results */
  double host_work_us;           /* host time from a round result to the next launch issued */
  uint64_t device_fs_rounds;     /* rounds whose challenge the device drew (ZK_DEVICE_FS), replayed by the host */
} zk_stats;
int zk_ctx_set_timing(zk_ctx* ctx, int enable);                /* all kinds on / off */
int zk_ctx_set_timing_mask(zk_ctx* ctx, uint32_t kind_mask);   /* bit k = time ZK_K_k launches */
int zk_ctx_get_stats(const zk_ctx* ctx, zk_stats* out);
int zk_ctx_reset_stats(zk_ctx* ctx);
/* The event-timed launches since the last zk_ctx_reset_stats, in launch order
 * (kind, duration, algorithmic bytes): *n gets the count, at most cap are copied. */
typedef struct {
  int kind;
  double ms;
  double alg_bytes;
} zk_launch;
int zk_ctx_get_launches(const zk_ctx* ctx, zk_launch* out, size_t cap, size_t* n);

/* ---------------------------------------------------------------------------
 * Fiat-Shamir transcript (host) — fiat_shamir/src/fiat_shamir_transcript.rs
 * ------------------------------------------------------------------------- */
zk_transcript* zk_transcript_new(void);                      /* Transcript::new        :12-17 */
zk_transcript* zk_transcript_clone(const zk_transcript* t);  /* #[derive(Clone)]       :5     */
void zk_transcript_free(zk_transcript* t);
int zk_transcript_append(zk_transcript* t, const uint8_t* data, size_t len); /* append :19-21 */
int zk_transcript_get_random_challenge(zk_transcript* t, zk_field field, zk_repr repr,
                                       zk_fe* out);          /* get_random_challenge   :23-29 */
/* Checkpoint / resume of a transcript mid-proof. The reference's
 * Transcript derives Clone (:5) but not serde; this is the byte image of that clone:
 *   "ZKTR" | u32 version (1) | u32 fill (< 136) | u32 0 | 25 x u64 LE Keccak lanes |
 *   136 bytes of the partial rate block (bytes >= fill are zero)
 * = ZK_TRANSCRIPT_STATE_BYTES. A deserialised transcript continues bit-exactly where the
 * serialised one stood (same challenges for the same appends). zk_transcript_deserialize
 * returns NULL on a bad magic / version / fill / non-zero padding or len != the size. */
#define ZK_TRANSCRIPT_STATE_BYTES 352
int zk_transcript_serialize(const zk_transcript* t, uint8_t* out, size_t cap, size_t* out_len);
zk_transcript* zk_transcript_deserialize(const uint8_t* data, size_t len);
/* fq_vec_to_bytes :32-37 — canonical LE, 32 bytes per element into out[32*n] */
int zk_fe_vec_to_bytes(zk_field field, zk_repr repr, const zk_fe* v, size_t n, uint8_t* out);

/* ---------------------------------------------------------------------------
 * MultilinearPoly — multilinear_polynomial/src/multilinear_polynomial_evaluation.rs
 * ------------------------------------------------------------------------- */
/* partial_evaluate(bit, value) :52-63; out has 2^(nvars-1) elements */
int zk_mle_partial_evaluate(zk_ctx* ctx, zk_field field, zk_repr repr, const zk_fe* evals, uint32_t nvars,
                            uint32_t bit, const zk_fe* value, zk_fe* out);
/* evaluate(values) :79-91; npoint must equal nvars (else ZK_EINVAL, the panic at :80-82) */
int zk_mle_evaluate(zk_ctx* ctx, zk_field field, zk_repr repr, const zk_fe* evals, uint32_t nvars,
                    const zk_fe* point, uint32_t npoint, zk_fe* out);

/* Table builders (multilinear_polynomial_evaluation.rs): op = ZK_MLE_ADD / MUL / SUB.
 *   zk_mle_binop   impl Add / Mul / Sub for MultilinearPoly :113-151 — element-wise over the
 *                  zip of a (2^nvars_a) and b (2^nvars_b): out has 2^min(nvars_a, nvars_b)
 *   zk_mle_scale   scale(value) :93-97 — out[i] = evals[i] * value, 2^nvars outputs
 *   zk_mle_tensor  tensor_add_mul_polynomials(a, b, op) :99-110 — out[i nb + j] = op(a[i], b[j]),
 *                  op ADD or MUL only (Operation :4-17); na * nb must be a nonzero power of
 *                  two (MultilinearPoly::new panics otherwise) — ZK_EINVAL */
typedef enum { ZK_MLE_ADD = 0, ZK_MLE_MUL = 1, ZK_MLE_SUB = 2 } zk_mle_op;
int zk_mle_binop(zk_ctx* ctx, zk_field field, zk_repr repr, zk_mle_op op, const zk_fe* a, uint32_t nvars_a,
                 const zk_fe* b, uint32_t nvars_b, zk_fe* out);
int zk_mle_scale(zk_ctx* ctx, zk_field field, zk_repr repr, const zk_fe* evals, uint32_t nvars,
                 const zk_fe* value, zk_fe* out);
int zk_mle_tensor(zk_ctx* ctx, zk_field field, zk_repr repr, zk_mle_op op, const zk_fe* a, uint64_t na,
                  const zk_fe* b, uint64_t nb, zk_fe* out);

/* ---------------------------------------------------------------------------
 * Sum-check — sum_check/src/sum_check_protocol.rs
 * ------------------------------------------------------------------------- */
/* prove :25-52 -> Proof{proof_polynomials: nvars x [s0, s1], claimed_sum} */
int zk_sumcheck_prove(zk_ctx* ctx, zk_field field, zk_repr repr, const zk_fe* evals, uint32_t nvars,
                      zk_fe* out_round_polys /* 2*nvars */, zk_fe* out_claimed_sum);
/* verify :54-84; round_polys = nrounds polys of poly_len elements each */
int zk_sumcheck_verify(zk_ctx* ctx, zk_field field, zk_repr repr, const zk_fe* evals, uint32_t nvars,
                       const zk_fe* round_polys, uint32_t nrounds, uint32_t poly_len, const zk_fe* claimed_sum,
                       int* out_verified);
/* gkr_prove :86-115 on SumPoly{[ProductPoly[t0,t1], ProductPoly[t2,t3]]}
 * (composed_polynomial.rs:88-103 — reduce uses exactly these four tables).
 * Mutates `transcript`; out_coeffs[3*k .. 3*k+ncoeffs[k]) are round k's trimmed
 * UnivariatePoly coefficients; claimed_sum is passed through (:110-114). */
int zk_gkr_sumcheck_prove(zk_ctx* ctx, zk_field field, zk_repr repr, const zk_fe* const tables[4], uint32_t nvars,
                          const zk_fe* claimed_sum, zk_transcript* transcript, zk_fe* out_coeffs /* 3*nvars */,
                          uint8_t* out_ncoeffs /* nvars */, zk_fe* out_challenges /* nvars */,
                          zk_fe* out_claimed_sum);
/* gkr_verify :117-150 (host-only, O(nrounds)). On failure *out_verified=0,
 * final claim 0 and a single zero challenge (:128-134). out_challenges needs
 * max(nrounds,1) slots. */
int zk_gkr_sumcheck_verify(zk_field field, zk_repr repr, const zk_fe* coeffs /* 3*nrounds */,
                           const uint8_t* ncoeffs, uint32_t nrounds, const zk_fe* claimed_sum,
                           zk_transcript* transcript, int* out_verified, zk_fe* out_final_claimed_sum,
                           zk_fe* out_challenges);

/* ---------------------------------------------------------------------------
 * GKR over a layered circuit (gkr_protocol.rs:31-227,
 * gkr_circuit.rs:1-144). Layers are given input -> output: gates[l] gates in
 * layer l, ops concatenated layer by layer (0 = Operation::Add, 1 = Mul), gate
 * g of layer l reading (in[2g], in[2g+1]). Supported shape (the one for which
 * the reference's table sizes agree; anything else is ZK_EINVAL): powers of
 * two, ninputs = 2 gates[0], gates[l+1] = gates[l] / 2, output layer of 1 or
 * 2 gates, 2 gates[0] <= 2^14.
 * The prover evaluates the circuit, builds every layer's four sum-check tables
 * (wiring folded at the verifier's points — sparse, instead of the reference's
 * dense 2^(3g+2) add_i / mul_i — and the tensor sum / product of w) and runs
 * the layer sum-checks on the GPU; the transcript is the reference's (fresh,
 * output poly absorbed first, alpha / beta per layer). The input layer's KZG
 * commitment (:92-118, row f3) is not made: the two input-MLE evaluations it
 * would open are returned instead, and the verifier recomputes them when
 * given the inputs.
 * Outputs (rounds in processing order: output layer first; layer l has
 * 2 log2(2 gates[l]) rounds, total from zk_gkr_circuit_rounds):
 *   out_output_poly[2], out_coeffs[3*total] + out_ncoeffs[total] (trimmed),
 *   out_challenges[total], out_claims[2*(nlayers-1)] = (o1, o2) per layer
 *   except the input layer, out_input_evals[2].
 * ------------------------------------------------------------------------- */
int zk_gkr_circuit_rounds(uint32_t nlayers, const uint32_t* gates, uint32_t* out_total_rounds);
int zk_gkr_circuit_prove(zk_ctx* ctx, zk_field field, zk_repr repr, uint32_t nlayers, const uint32_t* gates,
                         const uint8_t* ops, const zk_fe* inputs, uint32_t ninputs, zk_fe* out_output_poly,
                         zk_fe* out_coeffs, uint8_t* out_ncoeffs, zk_fe* out_challenges, zk_fe* out_claims,
                         zk_fe* out_input_evals);
/* gkr::verify (host). inputs may be NULL (then the input evaluations are not
 * re-derived, matching a verifier that trusts the commitment opening). */
int zk_gkr_circuit_verify(zk_field field, zk_repr repr, uint32_t nlayers, const uint32_t* gates, const uint8_t* ops,
                          const zk_fe* inputs, uint32_t ninputs, const zk_fe* output_poly, const zk_fe* coeffs,
                          const uint8_t* ncoeffs, const zk_fe* claims, const zk_fe* input_evals, int* out_verified);

/* ---------------------------------------------------------------------------
 * Multilinear KZG over BLS12-381 G1 (pcs/src/kzg_pcs/kzg.rs).
 * Scalars are BLS12-381 Fr (zk_fe, repr as elsewhere). Points are affine with
 * canonical little-endian 48-byte coordinates; (0, 0) is the point at infinity.
 *   zk_kzg_setup       KZG::new / run_trusted_setup's G1 half (:18-49): the
 *                      Lagrange basis eq(taus, i) * G for every i (MSB-first
 *                      hypercube, generate_bhc :171-181), plus the bases over
 *                      every suffix of taus used by get_proof, and (host)
 *                      the G2 taus tau_i * G2 used by KZG::verify (below).
 *   zk_kzg_commit      KZG::commit (:51-53) = sum_i evals[i] * L_i (Pippenger MSM)
 *   zk_kzg_get_proof   KZG::get_proof (:59-95): nvars quotient commitments
 *   zk_kzg_lagrange_basis  the basis over the last nvars_suffix taus
 *   zk_msm_g1          sum_i scalars[i] * bases[i] for caller bases (checked on the curve)
 * KZG::open is MultilinearPoly::evaluate: zk_mle_evaluate.
 * ------------------------------------------------------------------------- */
typedef struct {
  uint64_t x[6];
  uint64_t y[6];
} zk_g1;
typedef struct zk_kzg zk_kzg;
int zk_kzg_setup(zk_ctx* ctx, zk_repr repr, const zk_fe* taus, uint32_t nvars, zk_kzg** out);
void zk_kzg_free(zk_kzg* kzg);
int zk_kzg_lagrange_basis(zk_ctx* ctx, const zk_kzg* kzg, uint32_t nvars_suffix, zk_g1* out /* 2^nvars_suffix */);
int zk_kzg_commit(zk_ctx* ctx, const zk_kzg* kzg, zk_repr repr, const zk_fe* evals /* 2^nvars */, zk_g1* out);
int zk_dev_kzg_commit(zk_ctx* ctx, const zk_kzg* kzg, const void* dev_evals /* Montgomery Fr */, zk_g1* out);
int zk_kzg_get_proof(zk_ctx* ctx, const zk_kzg* kzg, zk_repr repr, const zk_fe* evals, const zk_fe* opened_value,
                     const zk_fe* point /* nvars */, zk_g1* out /* nvars */);
/* KZG::get_proof with the evaluations already on the device (Montgomery Fr,
 * 2^nvars, as zk_dev_kzg_commit takes them; read only): no host upload. repr
 * applies to opened_value and point. */
int zk_dev_kzg_get_proof(zk_ctx* ctx, const zk_kzg* kzg, zk_repr repr, const void* dev_evals, const zk_fe* opened_value,
                         const zk_fe* point /* nvars */, zk_g1* out /* nvars */);
/* Setups of >= 2^16 points use a fixed-base table of G1 (654 MB of device
 * memory) built once per device and shared by every context of the process.
 * This frees it for `device` (-1: every device); the next large setup rebuilds
 * it (~50 ms). ZK_EINVAL while a setup on that device is using it. */
int zk_kzg_release_fixed_base_cache(int device);
int zk_msm_g1(zk_ctx* ctx, zk_repr repr, const zk_g1* bases, const zk_fe* scalars, size_t n, zk_g1* out);

/* Verifier half (host, O(nvars) pairings; pcs/src/kzg_pcs/kzg.rs:35-49, :97-129).
 * G2 points are affine over Fq2 = Fq[u]/(u^2+1): x = x[0] + x[1] u, canonical
 * 48-byte LE coordinates, all zero = infinity; inputs are checked on the twist
 * y^2 = x^3 + 4(1+u).
 *   zk_kzg_g2_taus     KZG::g2_taus (pub field): tau_i * G2, nvars points
 *   zk_kzg_verify      KZG::verify: 1 / 0 in *out_verified; nproof != npoint is
 *                      ZK_EINVAL (the panic at :104-106); g2_taus holds npoint points
 *   zk_g2_mul_generator  scalars[i] * G2 (G2Projective::mul_bigint)
 *   zk_bls12_381_pairing Bls12_381::pairing(p, q) as 6 Fq2 = 72 u64: the
 *                      Fq12 = Fq6[w]/(w^2 - v), Fq6 = Fq2[v]/(v^3 - (1+u)) element
 *                      c0.c0, c0.c1, c0.c2, c1.c0, c1.c1, c1.c2, each Fq2 as (re, im)
 *                      canonical 6 x u64 (ark's field order)
 *   zk_bls12_381_pairing_check  *out_ok = prod_i e(p_i, q_i) == 1 */
typedef struct {
  uint64_t x[2][6];
  uint64_t y[2][6];
} zk_g2;
int zk_kzg_g2_taus(const zk_kzg* kzg, zk_g2* out /* nvars */);
int zk_kzg_verify(zk_repr repr, const zk_g1* commitment, const zk_fe* opened_value, const zk_g1* proof,
                  uint32_t nproof, const zk_fe* point, uint32_t npoint, const zk_g2* g2_taus, int* out_verified);
int zk_g2_mul_generator(zk_repr repr, const zk_fe* scalars, size_t n, zk_g2* out);
int zk_bls12_381_pairing(const zk_g1* p, const zk_g2* q, uint64_t out[72]);
int zk_bls12_381_pairing_check(const zk_g1* p, const zk_g2* q, size_t n, int* out_ok);

/* gkr::prove WITH the input layer's KZG step (gkr_protocol.rs:92-118), so the
 * proof is the reference's GkrProof including input_proof. BLS12-381 Fr only
 * (the reference's KZG is over BLS12-381, kzg.rs:3). The reference draws the
 * taus from StdRng::from_entropy (:97-103); here they are the caller's
 * taus[log2 ninputs] so proofs are reproducible. Writes everything
 * zk_gkr_circuit_prove writes (out_input_evals = the two values KZG::open
 * returns at r_b and r_c), plus the commitment (KZG::commit :106), the two
 * get_proof results out_proofs[2 log2 ninputs] (w_b's then w_c's, :108-113)
 * and the verifier's setup out_g2_taus[log2 ninputs] (KZG::g2_taus). */
int zk_gkr_circuit_prove_kzg(zk_ctx* ctx, zk_repr repr, uint32_t nlayers, const uint32_t* gates, const uint8_t* ops,
                             const zk_fe* inputs, uint32_t ninputs, const zk_fe* taus, zk_fe* out_output_poly,
                             zk_fe* out_coeffs, uint8_t* out_ncoeffs, zk_fe* out_challenges, zk_fe* out_claims,
                             zk_fe* out_input_evals, zk_g1* out_commitment, zk_g1* out_proofs, zk_g2* out_g2_taus);
/* gkr::verify (:128-227) with the two KZG::verify checks of the input layer
 * (:155-175) at the verifier's own (r_b, r_c): needs no inputs.
 * SOUNDNESS: g2_taus must come from a trusted setup the verifier holds, NOT
 * from the proof. The reference passes the prover's kzg_setup.g2_taus
 * (gkr_protocol.rs:167,175), and this entry point keeps that behaviour for
 * parity. A prover who picks its own setup can satisfy both pairings, so
 * this check is not sound against a malicious prover unless the caller
 * supplies g2_taus of its own (zk_kzg_g2_taus of a setup it trusts). */
int zk_gkr_circuit_verify_kzg(zk_repr repr, uint32_t nlayers, const uint32_t* gates, const uint8_t* ops,
                              const zk_fe* output_poly, const zk_fe* coeffs, const uint8_t* ncoeffs,
                              const zk_fe* claims, const zk_fe* opened_evals, const zk_g1* commitment,
                              const zk_g1* proofs, const zk_g2* g2_taus, int* out_verified);

/* ---------------------------------------------------------------------------
 * Proof blob: a canonical byte form of a proof, so a proof
 * produced on the CPU, on one GPU or on G GPUs can be compared as one digest
 * and shipped/verified elsewhere. The reference keeps proofs as in-memory
 * structs only (sum_check_protocol.rs:8-17); the blob holds exactly their
 * fields. All integers little-endian; field elements canonical 32-byte LE
 * (fq_vec_to_bytes, fiat_shamir_transcript.rs:32-37):
 *   [0,4)   "ZKSP"
 *   4       version = 1
 *   5       kind: ZK_BLOB_GKR (gkr_prove) or ZK_BLOB_SUMCHECK (prove)
 *   6       zk_field
 *   7       0
 *   [8,12)  nrounds (u32)
 *   [12,44) claimed_sum
 *   then per round: m (u8), m elements. For ZK_BLOB_GKR, m <= 3 is the trimmed
 *   coefficient count and the m elements are exactly the bytes the transcript
 *   absorbs that round; for ZK_BLOB_SUMCHECK they are the round's [s0, s1].
 * Parsing rejects (ZK_EINVAL) a bad magic/version/kind/field, truncation,
 * trailing bytes, m > 3 in a GKR blob, and elements >= p.
 * Serialisers return the size in *out_len; pass out = NULL to query it.
 * ------------------------------------------------------------------------- */
enum { ZK_BLOB_GKR = 1, ZK_BLOB_SUMCHECK = 2 };
int zk_gkr_proof_to_blob(zk_field field, zk_repr repr, const zk_fe* coeffs /* 3*nrounds */, const uint8_t* ncoeffs,
                         uint32_t nrounds, const zk_fe* claimed_sum, uint8_t* out, size_t cap, size_t* out_len);
int zk_sumcheck_proof_to_blob(zk_field field, zk_repr repr, const zk_fe* round_polys /* nrounds*poly_len */,
                              uint32_t nrounds, uint32_t poly_len, const zk_fe* claimed_sum, uint8_t* out,
                              size_t cap, size_t* out_len);
int zk_proof_blob_info(const uint8_t* blob, size_t len, int* out_kind, zk_field* out_field, uint32_t* out_nrounds);
int zk_gkr_proof_from_blob(const uint8_t* blob, size_t len, zk_repr repr, zk_fe* out_coeffs /* 3*cap_rounds */,
                           uint8_t* out_ncoeffs /* cap_rounds */, uint32_t cap_rounds, zk_fe* out_claimed_sum);
int zk_sumcheck_proof_from_blob(const uint8_t* blob, size_t len, zk_repr repr, zk_fe* out_round_polys,
                                size_t cap_elems, uint32_t* out_poly_len, zk_fe* out_claimed_sum);
/* gkr_verify of a GKR blob (claimed sum taken from the blob); outputs canonical. */
int zk_gkr_verify_blob(const uint8_t* blob, size_t len, zk_transcript* transcript, int* out_verified,
                       zk_fe* out_final_claimed_sum, zk_fe* out_challenges /* cap_rounds */, uint32_t cap_rounds);
/* Keccak-256 (the transcript's sponge: rate 136, pad 0x01..0x80) of a byte string */
int zk_keccak256(const uint8_t* data, size_t len, uint8_t out[32]);

/* ---------------------------------------------------------------------------
 * Device-resident API (tables already in HBM, Montgomery form)
 * ------------------------------------------------------------------------- */
int zk_dev_alloc(zk_ctx* ctx, size_t bytes, void** out);
int zk_dev_free(zk_ctx* ctx, void* p);
/* host (repr) -> device Montgomery, and back */
int zk_dev_upload(zk_ctx* ctx, zk_field field, zk_repr repr, const zk_fe* host, size_t n, void* dev);
int zk_dev_download(zk_ctx* ctx, zk_field field, zk_repr repr, const void* dev, size_t n, zk_fe* host);
/* synthetic table: dev[m] = synth(seed, table, index0 + m*stride) in Montgomery form */
int zk_dev_synth_fill(zk_ctx* ctx, zk_field field, void* dev, uint64_t count, uint64_t seed, uint32_t table,
                      uint64_t index0, uint64_t stride);
/* partial_evaluate on device buffers: d_out has 2^(nvars-1) elements (may not alias d_in) */
int zk_dev_mle_partial_evaluate(zk_ctx* ctx, zk_field field, const void* d_in, uint32_t nvars, uint32_t bit,
                                zk_repr repr, const zk_fe* value, void* d_out);
/* tensor_add_mul_polynomials on device buffers (Montgomery): d_out[i nb + j] = op(d_a[i], d_b[j]);
 * the GKR-shaped S = w (+) w and P = w (x) w tables built in HBM (d_out may not alias an input) */
int zk_dev_mle_tensor(zk_ctx* ctx, zk_field field, zk_mle_op op, const void* d_a, uint64_t na, const void* d_b,
                      uint64_t nb, void* d_out);
/* gkr_prove over device tables (read-only; the ctx workspace holds the folds) */
int zk_dev_gkr_sumcheck_prove(zk_ctx* ctx, zk_field field, const void* const d_tables[4], uint32_t nvars,
                              zk_repr repr, const zk_fe* claimed_sum, zk_transcript* transcript,
                              zk_fe* out_coeffs, uint8_t* out_ncoeffs, zk_fe* out_challenges);

/* ---------------------------------------------------------------------------
 * Multi-GPU: the hypercube is split over `world` ranks (one process or thread
 * per GPU, world a power of two). Rank g holds the sub-cube whose LOW
 * log2(world) index bits equal g: local m <-> global m*world + g. The first
 * nvars_local rounds fold purely locally; each round's partial sums are
 * combined with ONE all-reduce of at most 24 u64 (three elements split into
 * 32-bit limbs, so the u64 sum is exact); a last all-reduce of one-hot slots
 * gathers the 4 remaining elements of every rank so all ranks finish the last
 * log2(world) rounds identically. All-reduce (SUM, u64) is the only collective.
 * No broadcast is needed: every rank derives the same challenges from the
 * same transcript.
 * ------------------------------------------------------------------------- */
/* host-memory all-reduce supplied by the caller (e.g. torch.distributed/gloo).
 * With a host callback attached every step launches after its challenge
 * (pre-enqueue off): the callback's latency is unbounded and ranks may share
 * one device. */
typedef int (*zk_allreduce_u64_fn)(void* user, uint64_t* data, size_t count); /* in-place SUM, 0 = ok */
int zk_ctx_attach_host_comm(zk_ctx* ctx, int rank, int world, zk_allreduce_u64_fn allreduce, void* user);
/* RCCL over xGMI: rank 0 creates the id, every rank passes the same 128 bytes */
int zk_comm_get_unique_id(uint8_t out[128]);
int zk_ctx_attach_rccl(zk_ctx* ctx, int rank, int world, const uint8_t unique_id[128]);
int zk_ctx_detach_comm(zk_ctx* ctx);
/* The communicator the ctx holds: *out_kind = 0 none, 1 host callback, 2 RCCL;
 * *out_rank / *out_count = this rank and the number of ranks — for RCCL as the
 * communicator reports them (ncclCommUserRank / ncclCommCount), else the
 * attached rank / world (0 / 1 with none). */
int zk_ctx_comm_count(const zk_ctx* ctx, int* out_kind, int* out_rank, int* out_count);
/* Peer reduction (collective: every rank calls it, after attaching a
 * communicator; world <= 8, the ranks of one node). enable = 1: each rank
 * allocates an uncached receive buffer, the IPC handles are exchanged through
 * the attached communicator and opened, and one reduction of known values is
 * checked across the world. From then on each sharded step's sums are
 * summed by the step kernel itself — its publishing block writes them into
 * every rank's buffer and waits for the others' (replacing the step's
 * all-reduce of sum_check_protocol.rs:96-108's round sums; the early gather of
 * <= 4 x 2^12 elements per rank goes through a second such buffer).
 * enable = 0 releases it, as does attaching a communicator again. Proofs must
 * then run in the same order on every rank (the reductions carry a shared
 * sequence number); a proof that fails mid-way leaves the sequence unusable
 * until the next attach.
 * *out_ok (may be null) = 1 when enabled and the check passed. */
int zk_ctx_attach_peer_reduce(zk_ctx* ctx, int enable, int* out_ok);
/* gkr_prove over the global (nvars_local + log2(world))-variable SumPoly whose
 * local shard this rank holds; outputs are the global proof (identical on all
 * ranks). out arrays sized for nvars_local + log2(world) rounds. */
int zk_dev_gkr_sumcheck_prove_sharded(zk_ctx* ctx, zk_field field, const void* const d_local_tables[4],
                                      uint32_t nvars_local, zk_repr repr, const zk_fe* claimed_sum,
                                      zk_transcript* transcript, zk_fe* out_coeffs, uint8_t* out_ncoeffs,
                                      zk_fe* out_challenges);

#ifdef __cplusplus
}
#endif
#endif /* ZK_SUMCHECK_H */
