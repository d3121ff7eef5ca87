/*
 * ORACLE — TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement (plain C, single thread) of the reference's sum-check hot
 * path, used by tests/ as the parity checker and by bench.py as the
 * `cpu_baseline` ("port") leg. Nothing in the product library links, loads or
 * calls this code; the product path (zk-research-implementations_amd/) is
 * HIP-only and fails loudly without its extension.
 *
 * It follows the reference algorithm step by step, including its allocation
 * pattern (one fresh table per partial evaluation, reduce() clones, Lagrange
 * interpolation with trim), so its timing stands in for the Rust CPU prover
 * that cannot be built here (no cargo/rustc):
 *   sum_check/src/sum_check_protocol.rs:25-175
 *   multilinear_polynomial/src/multilinear_polynomial_evaluation.rs:26-164
 *   multilinear_polynomial/src/composed_polynomial.rs:15-103
 *   univariate_polynomial/src/univariate_polynomial_dense.rs:14-109
 *   fiat_shamir/src/fiat_shamir_transcript.rs:11-37
 * Field arithmetic restates ark-ff 0.5.0's `Fp<MontBackend<_,4>,4>` (4x64-bit
 * CIOS Montgomery, R = 2^256, u128 intermediates = ark's no-asm build); Keccak
 * restates sha3 0.10.8 / keccak 0.1.5 `Keccak256` (rate 136, pad 0x01..0x80).
 * Neither crate is vendored in /root/reference (Cargo.lock:89-92, 559-562,
 * 869-872); they are restated from their published algorithms.
 *
 * All field elements crossing this API are CANONICAL little-endian 4x u64.
 */
#ifndef ZK_ORACLE_H
#define ZK_ORACLE_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* field ids match include/zk_sumcheck.h */
enum { OR_BN254_FR = 0, OR_BN254_FQ = 1, OR_BLS12_381_FR = 2 };

typedef struct { uint64_t l[4]; } or_fe;

/* --- field (canonical in / canonical out) --- */
int or_fe_add(int field, const or_fe* a, const or_fe* b, or_fe* out);
int or_fe_mul(int field, const or_fe* a, const or_fe* b, or_fe* out);
int or_fe_to_mont(int field, const or_fe* a, or_fe* out);
int or_fe_from_le_bytes_mod_order(int field, const uint8_t* bytes, size_t n, or_fe* out);

/* --- Keccak-256 / transcript (fiat_shamir_transcript.rs:5-37) --- */
void or_keccak256(const uint8_t* data, size_t len, uint8_t out[32]);
void or_keccak_f1600(uint64_t st[25]);
typedef struct or_transcript or_transcript;
or_transcript* or_transcript_new(void);
void or_transcript_free(or_transcript* t);
void or_transcript_append(or_transcript* t, const uint8_t* data, size_t len);
int or_transcript_challenge(or_transcript* t, int field, or_fe* out);

/* --- multilinear (multilinear_polynomial_evaluation.rs) --- */
int or_mle_partial_evaluate(int field, const or_fe* evals, uint32_t nvars, uint32_t bit, const or_fe* r, or_fe* out);
int or_mle_evaluate(int field, const or_fe* evals, uint32_t nvars, const or_fe* point, or_fe* out);

/* --- univariate (univariate_polynomial_dense.rs:48-74) ---
 * interpolate npts points (x_i, y_i); writes trimmed coefficients, returns count */
int or_interpolate(int field, const or_fe* xs, const or_fe* ys, int npts, or_fe* coeffs_out);

/* --- sum-check (sum_check_protocol.rs) --- */
/* prove: out_round_polys[2*nvars], out_claimed_sum */
int or_sumcheck_prove(int field, const or_fe* evals, uint32_t nvars, or_fe* out_round_polys, or_fe* out_claimed_sum);
/* verify: round_polys is nrounds polys of poly_len elements each; returns 1/0, -1 = reference panics */
int or_sumcheck_verify(int field, const or_fe* evals, uint32_t nvars, const or_fe* round_polys, uint32_t nrounds,
                       uint32_t poly_len, const or_fe* claimed_sum);
/* gkr_prove on SumPoly{[ProductPoly[t0,t1], ProductPoly[t2,t3]]} (degree 2).
 * transcript is caller-owned and mutated; out_coeffs[3*nvars], out_ncoeffs[nvars], out_challenges[nvars] */
int or_gkr_prove(int field, const or_fe* const tables[4], uint32_t nvars, or_transcript* t, or_fe* out_coeffs,
                 uint8_t* out_ncoeffs, or_fe* out_challenges);
/* same outputs as or_gkr_prove: fused, in place, OpenMP over all threads (the fast CPU restatement) */
int or_gkr_prove_fast(int field, const or_fe* const tables[4], uint32_t nvars, or_transcript* t, or_fe* out_coeffs,
                      uint8_t* out_ncoeffs, or_fe* out_challenges);
int or_threads(void); /* OpenMP threads or_gkr_prove_fast uses */
/* gkr_verify: returns verified (1/0); out_final_claim, out_challenges[nrounds] (on failure: final 0, 1 challenge 0) */
int or_gkr_verify(int field, const or_fe* coeffs, const uint8_t* ncoeffs, uint32_t nrounds, const or_fe* claimed_sum,
                  or_transcript* t, or_fe* out_final_claim, or_fe* out_challenges);

/* --- synthetic inputs (identical to the device generator) --- */
void or_synth_fill(int field, uint64_t seed, uint32_t table, uint64_t index0, uint64_t count, or_fe* out);

#ifdef __cplusplus
}
#endif
#endif
