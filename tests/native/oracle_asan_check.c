/* Sanitizer driver for the C oracle (test infrastructure): built by
 * `make -C oracle asan` with -fsanitize=address,undefined and run by
 * tests/test_sanitizers_cpu.py. It runs every oracle entry point over small
 * sizes on the three fields — the reference-faithful and the fused OpenMP
 * GKR provers (which must agree), gkr_verify of their proofs, plain
 * prove/verify, folds, evaluation, interpolation, the transcript and Keccak
 * over every length around the rate — so ASan/UBSan see the oracle's own
 * allocation pattern (fresh tables per fold, clones, trims). Exit 0 and
 * "oracle_asan_check ok" on success. */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "zk_oracle.h"

static int failures = 0;
#define EXPECT(c)                                                                     \
  do {                                                                                \
    if (!(c)) {                                                                       \
      fprintf(stderr, "%s:%d: expectation failed: %s\n", __FILE__, __LINE__, #c);    \
      ++failures;                                                                     \
    }                                                                                 \
  } while (0)

static void gkr_checks(int field, uint32_t n) {
  const uint64_t N = 1ull << n;
  or_fe* t[4];
  for (int k = 0; k < 4; ++k) {
    t[k] = malloc(N * sizeof(or_fe));
    or_synth_fill(field, 7, (uint32_t)k, 0, N, t[k]);
  }
  const uint32_t m = n ? n : 1;
  or_fe* co = calloc(3 * m, sizeof(or_fe));
  or_fe* co2 = calloc(3 * m, sizeof(or_fe));
  or_fe* ch = calloc(m, sizeof(or_fe));
  or_fe* ch2 = calloc(m, sizeof(or_fe));
  uint8_t* nc = calloc(m, 1);
  uint8_t* nc2 = calloc(m, 1);
  or_transcript* a = or_transcript_new();
  or_transcript* b = or_transcript_new();
  EXPECT(or_gkr_prove(field, (const or_fe* const*)t, n, a, co, nc, ch) == 0);
  EXPECT(or_gkr_prove_fast(field, (const or_fe* const*)t, n, b, co2, nc2, ch2) == 0);
  EXPECT(memcmp(co, co2, 3 * m * sizeof(or_fe)) == 0 && memcmp(ch, ch2, m * sizeof(or_fe)) == 0);
  or_transcript_free(a);
  or_transcript_free(b);
  /* the claimed sum the verifier starts from: s_0(0) + s_0(1) */
  or_fe claim = {{0, 0, 0, 0}}, fin;
  if (n) {
    or_fe s1 = co[0];
    for (int i = 1; i < nc[0]; ++i) or_fe_add(field, &s1, &co[i], &s1);
    or_fe_add(field, &co[0], &s1, &claim);
  }
  or_transcript* v = or_transcript_new();
  const int ok = or_gkr_verify(field, co, nc, n, &claim, v, &fin, ch2);
  EXPECT(n == 0 || ok == 1);
  or_transcript_free(v);
  free(co), free(co2), free(ch), free(ch2), free(nc), free(nc2);
  for (int k = 0; k < 4; ++k) free(t[k]);
}

static void plain_checks(int field, uint32_t n) {
  const uint64_t N = 1ull << n;
  or_fe* e = malloc(N * sizeof(or_fe));
  or_synth_fill(field, 1, 0, 0, N, e);
  or_fe* rp = calloc(2 * (n ? n : 1), sizeof(or_fe));
  or_fe cs;
  EXPECT(or_sumcheck_prove(field, e, n, rp, &cs) == 0);
  EXPECT(or_sumcheck_verify(field, e, n, rp, n, 2, &cs) == 1);
  if (n) {
    or_fe* half = malloc(N / 2 * sizeof(or_fe));
    or_fe r = {{12345, 0, 0, 0}}, out;
    for (uint32_t bit = 0; bit < n; ++bit) EXPECT(or_mle_partial_evaluate(field, e, n, bit, &r, half) == 0);
    or_fe* pt = calloc(n, sizeof(or_fe));
    for (uint32_t i = 0; i < n; ++i) pt[i].l[0] = 3 + i;
    EXPECT(or_mle_evaluate(field, e, n, pt, &out) == 0);
    free(pt);
    free(half);
  }
  free(rp);
  free(e);
}

int main(void) {
  for (int field = 0; field < 3; ++field) {
    for (uint32_t n = 0; n <= 11; ++n) gkr_checks(field, n);
    for (uint32_t n = 0; n <= 10; ++n) plain_checks(field, n);
    or_fe xs[3] = {{{0}}, {{1}}, {{2}}}, ys[3] = {{{2}}, {{4}}, {{6}}}, c[8];
    EXPECT(or_interpolate(field, xs, ys, 3, c) == 2);  /* univariate_polynomial_dense.rs tests: [2, 2] */
    uint8_t bytes[64];
    for (int i = 0; i < 64; ++i) bytes[i] = (uint8_t)(0xa5 ^ i);
    or_fe x;
    EXPECT(or_fe_from_le_bytes_mod_order(field, bytes, 64, &x) == 0);
    EXPECT(or_fe_to_mont(field, &x, &x) == 0);
  }
  uint8_t data[700], d[32];
  for (int i = 0; i < 700; ++i) data[i] = (uint8_t)(i * 7);
  for (size_t len = 0; len <= sizeof data; ++len) or_keccak256(data, len, d);
  or_transcript* t = or_transcript_new();
  for (size_t len = 0; len < 300; len += 13) {
    or_fe ch;
    or_transcript_append(t, data, len);
    EXPECT(or_transcript_challenge(t, (int)(len % 3), &ch) == 0);
  }
  or_transcript_free(t);
  if (failures) {
    fprintf(stderr, "oracle_asan_check: %d failures\n", failures);
    return 1;
  }
  printf("oracle_asan_check ok\n");
  return 0;
}
