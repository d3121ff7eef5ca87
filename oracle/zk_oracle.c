/*
 * ORACLE — TEST INFRASTRUCTURE ONLY (see zk_oracle.h). Plain C restatement of
 * the reference sum-check path; every function cites the reference file:line
 * it follows. Used only by tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg.
 */
#include "zk_oracle.h"

#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

typedef unsigned __int128 u128;

/* ------------------------------------------------------------------------ */
/* Field: ark-ff 0.5.0 Fp<MontBackend<_,4>,4> restated (Montgomery, R=2^256) */
/* ------------------------------------------------------------------------ */
typedef struct {
  uint64_t p[4];
  uint64_t pinv; /* -p^-1 mod 2^64 */
  uint64_t r2[4];
} or_params;

static const or_params PARAMS[3] = {
    /* BN254 Fr (ark-bn254 0.5.0) */
    {{0x43e1f593f0000001ull, 0x2833e84879b97091ull, 0xb85045b68181585dull, 0x30644e72e131a029ull},
     0xc2e1f593efffffffull,
     {0x1bb8e645ae216da7ull, 0x53fe3ab1e35c59e3ull, 0x8c49833d53bb8085ull, 0x0216d0b17f4e44a5ull}},
    /* BN254 Fq */
    {{0x3c208c16d87cfd47ull, 0x97816a916871ca8dull, 0xb85045b68181585dull, 0x30644e72e131a029ull},
     0x87d20782e4866389ull,
     {0xf32cfc5b538afa89ull, 0xb5e71911d44501fbull, 0x47ab1eff0a417ff6ull, 0x06d89f71cab8351full}},
    /* BLS12-381 Fr (ark-bls12-381 0.5.0) */
    {{0xffffffff00000001ull, 0x53bda402fffe5bfeull, 0x3339d80809a1d805ull, 0x73eda753299d7d48ull},
     0xfffffffeffffffffull,
     {0xc999e990f3f29c6dull, 0x2b6cedcb87925c23ull, 0x05d314967254398full, 0x0748d9d99f59ff11ull}},
};

typedef struct { uint64_t l[4]; } mfe; /* Montgomery form */

static int geq_p(const uint64_t a[4], const uint64_t p[4]) {
  for (int i = 3; i >= 0; --i) {
    if (a[i] > p[i]) return 1;
    if (a[i] < p[i]) return 0;
  }
  return 1;
}
static void sub_p(uint64_t a[4], const uint64_t p[4]) {
  uint64_t borrow = 0;
  for (int i = 0; i < 4; ++i) {
    u128 d = (u128)a[i] - p[i] - borrow;
    a[i] = (uint64_t)d;
    borrow = (uint64_t)(d >> 64) & 1;
  }
}
/* CIOS Montgomery multiplication, 4x64 (ark-ff `mul_assign` without asm). */
static mfe m_mul(const or_params* P, mfe a, mfe b) {
  uint64_t t[6] = {0, 0, 0, 0, 0, 0};
  for (int i = 0; i < 4; ++i) {
    uint64_t c = 0;
    for (int j = 0; j < 4; ++j) {
      u128 x = (u128)a.l[j] * b.l[i] + t[j] + c;
      t[j] = (uint64_t)x;
      c = (uint64_t)(x >> 64);
    }
    u128 s = (u128)t[4] + c;
    t[4] = (uint64_t)s;
    t[5] = (uint64_t)(s >> 64);
    uint64_t m = t[0] * P->pinv;
    u128 x = (u128)m * P->p[0] + t[0];
    c = (uint64_t)(x >> 64);
    for (int j = 1; j < 4; ++j) {
      x = (u128)m * P->p[j] + t[j] + c;
      t[j - 1] = (uint64_t)x;
      c = (uint64_t)(x >> 64);
    }
    s = (u128)t[4] + c;
    t[3] = (uint64_t)s;
    t[4] = t[5] + (uint64_t)(s >> 64);
  }
  mfe r = {{t[0], t[1], t[2], t[3]}};
  if (t[4] || geq_p(r.l, P->p)) sub_p(r.l, P->p);
  return r;
}
static mfe m_add(const or_params* P, mfe a, mfe b) {
  mfe r;
  uint64_t c = 0;
  for (int i = 0; i < 4; ++i) {
    u128 s = (u128)a.l[i] + b.l[i] + c;
    r.l[i] = (uint64_t)s;
    c = (uint64_t)(s >> 64);
  }
  if (c || geq_p(r.l, P->p)) sub_p(r.l, P->p);
  return r;
}
static mfe m_sub(const or_params* P, mfe a, mfe b) {
  mfe r;
  uint64_t borrow = 0;
  for (int i = 0; i < 4; ++i) {
    u128 d = (u128)a.l[i] - b.l[i] - borrow;
    r.l[i] = (uint64_t)d;
    borrow = (uint64_t)(d >> 64) & 1;
  }
  if (borrow) {
    uint64_t c = 0;
    for (int i = 0; i < 4; ++i) {
      u128 s = (u128)r.l[i] + P->p[i] + c;
      r.l[i] = (uint64_t)s;
      c = (uint64_t)(s >> 64);
    }
  }
  return r;
}
static mfe m_neg(const or_params* P, mfe a) {
  mfe z = {{0, 0, 0, 0}};
  return m_sub(P, z, a);
}
static int m_is_zero(mfe a) { return (a.l[0] | a.l[1] | a.l[2] | a.l[3]) == 0; }
static int m_eq(mfe a, mfe b) { return !memcmp(a.l, b.l, 32); }
static mfe m_from_canon(const or_params* P, const or_fe* c) {
  mfe a, r2;
  memcpy(a.l, c->l, 32);
  memcpy(r2.l, P->r2, 32);
  return m_mul(P, a, r2);
}
static or_fe m_to_canon(const or_params* P, mfe a) {
  mfe one = {{1, 0, 0, 0}};
  mfe c = m_mul(P, a, one);
  or_fe r;
  memcpy(r.l, c.l, 32);
  return r;
}
static mfe m_from_u64(const or_params* P, uint64_t v) { /* F::from(u64) */
  or_fe c = {{v, 0, 0, 0}};
  return m_from_canon(P, &c);
}
static mfe m_zero(void) {
  mfe z = {{0, 0, 0, 0}};
  return z;
}
/* x.pow(&[e]) — square-and-multiply over the exponent's bits (ark Field::pow) */
static mfe m_pow(const or_params* P, mfe x, const uint64_t* e, int nlimbs) {
  mfe r = m_from_u64(P, 1);
  for (int i = nlimbs - 1; i >= 0; --i)
    for (int b = 63; b >= 0; --b) {
      r = m_mul(P, r, r);
      if ((e[i] >> b) & 1) r = m_mul(P, r, x);
    }
  return r;
}
static mfe m_inv(const or_params* P, mfe a) { /* a^(p-2); result identical to ark's inverse */
  uint64_t e[4];
  memcpy(e, P->p, 32);
  /* p - 2 (p odd, low limb >= 2 for all three moduli except BLS low limb == 1) */
  uint64_t borrow = 2;
  for (int i = 0; i < 4 && borrow; ++i) {
    uint64_t old = e[i];
    e[i] = old - borrow;
    borrow = old < borrow ? 1 : 0;
  }
  return m_pow(P, a, e, 4);
}

static const or_params* params(int field) {
  if (field < 0 || field > 2) return NULL;
  return &PARAMS[field];
}

int or_fe_add(int field, const or_fe* a, const or_fe* b, or_fe* out) {
  const or_params* P = params(field);
  if (!P) return -1;
  *out = m_to_canon(P, m_add(P, m_from_canon(P, a), m_from_canon(P, b)));
  return 0;
}
int or_fe_mul(int field, const or_fe* a, const or_fe* b, or_fe* out) {
  const or_params* P = params(field);
  if (!P) return -1;
  *out = m_to_canon(P, m_mul(P, m_from_canon(P, a), m_from_canon(P, b)));
  return 0;
}
int or_fe_to_mont(int field, const or_fe* a, or_fe* out) {
  const or_params* P = params(field);
  if (!P) return -1;
  mfe m = m_from_canon(P, a);
  memcpy(out->l, m.l, 32);
  return 0;
}

/* F::from_le_bytes_mod_order — ark-ff 0.5.0: leading (most significant)
 * num_modulus_bytes-1 bytes converted directly, then Horner over the rest:
 * res = res*256 + byte. The value is the LE integer mod p. */
static mfe m_from_le_bytes_mod_order(const or_params* P, const uint8_t* bytes, size_t n) {
  size_t direct = 31; /* (MODULUS_BIT_SIZE + 7)/8 - 1 for 254/255-bit moduli */
  if (direct > n) direct = n;
  or_fe hi = {{0, 0, 0, 0}};
  for (size_t k = 0; k < direct; ++k) { /* bytes[n-direct .. n) little-endian */
    size_t src = n - direct + k;
    hi.l[k / 8] |= (uint64_t)bytes[src] << (8 * (k % 8));
  }
  mfe res = m_from_canon(P, &hi);
  mfe w = m_from_u64(P, 256);
  for (size_t k = n - direct; k-- > 0;) {
    res = m_mul(P, res, w);
    res = m_add(P, res, m_from_u64(P, bytes[k]));
  }
  return res;
}
int or_fe_from_le_bytes_mod_order(int field, const uint8_t* bytes, size_t n, or_fe* out) {
  const or_params* P = params(field);
  if (!P) return -1;
  *out = m_to_canon(P, m_from_le_bytes_mod_order(P, bytes, n));
  return 0;
}

/* ------------------------------------------------------------------------ */
/* Keccak-256 (sha3 0.10.8 `Keccak256`: Keccak[c=512], pad 0x01 .. 0x80)     */
/* ------------------------------------------------------------------------ */
static const uint64_t KRC[24] = {
    0x0000000000000001ull, 0x0000000000008082ull, 0x800000000000808aull, 0x8000000080008000ull,
    0x000000000000808bull, 0x0000000080000001ull, 0x8000000080008081ull, 0x8000000000008009ull,
    0x000000000000008aull, 0x0000000000000088ull, 0x0000000080008009ull, 0x000000008000000aull,
    0x000000008000808bull, 0x800000000000008bull, 0x8000000000008089ull, 0x8000000000008003ull,
    0x8000000000008002ull, 0x8000000000000080ull, 0x000000000000800aull, 0x800000008000000aull,
    0x8000000080008081ull, 0x8000000000008080ull, 0x0000000080000001ull, 0x8000000080008008ull};
static const int KROT[25] = {0, 1, 62, 28, 27, 36, 44, 6, 55, 20, 3, 10, 43, 25, 39, 41, 45, 15, 21, 8, 18, 2, 61, 56, 14};

static uint64_t rotl(uint64_t x, int s) { return s ? (x << s) | (x >> (64 - s)) : x; }

void or_keccak_f1600(uint64_t A[25]) {
  for (int round = 0; round < 24; ++round) {
    uint64_t C[5], D[5], B[25];
    for (int x = 0; x < 5; ++x) C[x] = A[x] ^ A[x + 5] ^ A[x + 10] ^ A[x + 15] ^ A[x + 20];
    for (int x = 0; x < 5; ++x) D[x] = C[(x + 4) % 5] ^ rotl(C[(x + 1) % 5], 1);
    for (int i = 0; i < 25; ++i) A[i] ^= D[i % 5];
    /* rho + pi: B[y, 2x+3y] = rot(A[x,y], r[x,y]) */
    for (int x = 0; x < 5; ++x)
      for (int y = 0; y < 5; ++y) B[y + 5 * ((2 * x + 3 * y) % 5)] = rotl(A[x + 5 * y], KROT[x + 5 * y]);
    for (int x = 0; x < 5; ++x)
      for (int y = 0; y < 5; ++y) A[x + 5 * y] = B[x + 5 * y] ^ (~B[(x + 1) % 5 + 5 * y] & B[(x + 2) % 5 + 5 * y]);
    A[0] ^= KRC[round];
  }
}

#define RATE 136
struct or_transcript {
  uint64_t st[25];
  uint8_t buf[RATE];
  size_t fill;
};
static void k_absorb_block(uint64_t st[25], const uint8_t* blk) {
  for (int i = 0; i < RATE / 8; ++i) {
    uint64_t w = 0;
    for (int b = 0; b < 8; ++b) w |= (uint64_t)blk[8 * i + b] << (8 * b);
    st[i] ^= w;
  }
  or_keccak_f1600(st);
}
static void k_update(or_transcript* t, const uint8_t* data, size_t len) {
  while (len) {
    size_t take = RATE - t->fill;
    if (take > len) take = len;
    memcpy(t->buf + t->fill, data, take);
    t->fill += take;
    data += take;
    len -= take;
    if (t->fill == RATE) {
      k_absorb_block(t->st, t->buf);
      t->fill = 0;
    }
  }
}
static void k_finalize_reset(or_transcript* t, uint8_t out[32]) {
  memset(t->buf + t->fill, 0, RATE - t->fill);
  t->buf[t->fill] ^= 0x01;
  t->buf[RATE - 1] ^= 0x80;
  k_absorb_block(t->st, t->buf);
  for (int i = 0; i < 32; ++i) out[i] = (uint8_t)(t->st[i / 8] >> (8 * (i % 8)));
  memset(t->st, 0, sizeof t->st);
  t->fill = 0;
}
void or_keccak256(const uint8_t* data, size_t len, uint8_t out[32]) {
  or_transcript t;
  memset(&t, 0, sizeof t);
  k_update(&t, data, len);
  k_finalize_reset(&t, out);
}
or_transcript* or_transcript_new(void) { return (or_transcript*)calloc(1, sizeof(or_transcript)); }
void or_transcript_free(or_transcript* t) { free(t); }
/* Transcript::append (fiat_shamir_transcript.rs:19-21) */
void or_transcript_append(or_transcript* t, const uint8_t* data, size_t len) { k_update(t, data, len); }
/* Transcript::get_random_challenge (fiat_shamir_transcript.rs:23-29) */
static mfe tr_challenge(const or_params* P, or_transcript* t) {
  uint8_t d[32];
  k_finalize_reset(t, d);
  k_update(t, d, 32);
  return m_from_le_bytes_mod_order(P, d, 32);
}
int or_transcript_challenge(or_transcript* t, int field, or_fe* out) {
  const or_params* P = params(field);
  if (!P) return -1;
  *out = m_to_canon(P, tr_challenge(P, t));
  return 0;
}
/* fq_vec_to_bytes (fiat_shamir_transcript.rs:32-37): canonical LE 32 B each */
static void tr_append_fes(const or_params* P, or_transcript* t, const mfe* v, size_t n) {
  uint8_t b[32];
  for (size_t i = 0; i < n; ++i) {
    or_fe c = m_to_canon(P, v[i]);
    for (int k = 0; k < 32; ++k) b[k] = (uint8_t)(c.l[k / 8] >> (8 * (k % 8)));
    k_update(t, b, 32);
  }
}

/* ------------------------------------------------------------------------ */
/* MultilinearPoly (multilinear_polynomial_evaluation.rs:19-164)             */
/* ------------------------------------------------------------------------ */
typedef struct {
  mfe* ev;
  size_t len;
  uint32_t nvars;
} mle;

static mle mle_clone(const mle* a) {
  mle r = {(mfe*)malloc(a->len * sizeof(mfe)), a->len, a->nvars};
  memcpy(r.ev, a->ev, a->len * sizeof(mfe));
  return r;
}
static void mle_free(mle* a) {
  free(a->ev);
  a->ev = NULL;
}
/* insert_bit (:158-164) */
static size_t insert_bit(size_t value, uint32_t bit) {
  size_t high = value >> bit, mask = ((size_t)1 << bit) - 1, low = value & mask;
  return high << (bit + 1) | low;
}
/* partial_evaluate (:52-63) with pair_points (:39-50): allocates the pair
 * list, then pushes a + r(b - a) into a Vec grown without capacity. */
static mle mle_partial_evaluate(const or_params* P, const mle* a, uint32_t bit, mfe r) {
  size_t half = (size_t)1 << (a->nvars - 1);
  uint32_t inv = a->nvars - bit - 1;
  size_t* pairs = (size_t*)malloc(2 * half * sizeof(size_t));
  for (size_t v = 0; v < half; ++v) {
    size_t z = insert_bit(v, inv);
    pairs[2 * v] = z;
    pairs[2 * v + 1] = z | ((size_t)1 << inv);
  }
  size_t cap = 0, n = 0;
  mfe* out = NULL;
  for (size_t v = 0; v < half; ++v) {
    if (n == cap) {
      cap = cap ? 2 * cap : 4;
      out = (mfe*)realloc(out, cap * sizeof(mfe));
    }
    mfe x = a->ev[pairs[2 * v]], y = a->ev[pairs[2 * v + 1]];
    out[n++] = m_add(P, x, m_mul(P, r, m_sub(P, y, x)));
  }
  free(pairs);
  mle res = {out, half, a->nvars - 1};
  return res;
}
/* evaluate (:79-91) */
static mfe mle_evaluate(const or_params* P, const mle* a, const mfe* pt) {
  mle cur = mle_clone(a);
  for (uint32_t i = 0; i < a->nvars; ++i) {
    mle nx = mle_partial_evaluate(P, &cur, 0, pt[i]);
    mle_free(&cur);
    cur = nx;
  }
  mfe r = cur.ev[0];
  mle_free(&cur);
  return r;
}
static int is_pow2_len(size_t len) { return len && !(len & (len - 1)); }
static uint32_t ilog2(size_t len) {
  uint32_t k = 0;
  while (((size_t)1 << (k + 1)) <= len) ++k;
  return k;
}
static mle mle_from_canon(const or_params* P, const or_fe* evals, size_t len) {
  mle r = {(mfe*)malloc(len * sizeof(mfe)), len, ilog2(len)};
  for (size_t i = 0; i < len; ++i) r.ev[i] = m_from_canon(P, &evals[i]);
  return r;
}

int or_mle_partial_evaluate(int field, const or_fe* evals, uint32_t nvars, uint32_t bit, const or_fe* r, or_fe* out) {
  const or_params* P = params(field);
  if (!P || nvars == 0 || bit >= nvars) return -1;
  mle a = mle_from_canon(P, evals, (size_t)1 << nvars);
  mle b = mle_partial_evaluate(P, &a, bit, m_from_canon(P, r));
  for (size_t i = 0; i < b.len; ++i) out[i] = m_to_canon(P, b.ev[i]);
  mle_free(&a);
  mle_free(&b);
  return 0;
}
int or_mle_evaluate(int field, const or_fe* evals, uint32_t nvars, const or_fe* point, or_fe* out) {
  const or_params* P = params(field);
  if (!P) return -1;
  mle a = mle_from_canon(P, evals, (size_t)1 << nvars);
  mfe* pt = (mfe*)malloc((nvars + 1) * sizeof(mfe));
  for (uint32_t i = 0; i < nvars; ++i) pt[i] = m_from_canon(P, &point[i]);
  *out = m_to_canon(P, mle_evaluate(P, &a, pt));
  free(pt);
  mle_free(&a);
  return 0;
}

/* ------------------------------------------------------------------------ */
/* UnivariatePoly (univariate_polynomial_dense.rs:5-109)                     */
/* ------------------------------------------------------------------------ */
typedef struct {
  mfe c[16];
  int n;
} upoly;

static void up_trim(upoly* p) { /* :14-18 */
  while (p->n > 0 && m_is_zero(p->c[p->n - 1])) p->n--;
}
static upoly up_scalar_mul(const or_params* P, upoly p, mfe s) { /* :34-46 */
  for (int i = 0; i < p.n; ++i) p.c[i] = m_mul(P, p.c[i], s);
  up_trim(&p);
  return p;
}
static upoly up_add(const or_params* P, upoly a, upoly b) { /* :77-93 */
  upoly r;
  r.n = a.n > b.n ? a.n : b.n;
  for (int i = 0; i < r.n; ++i) r.c[i] = m_zero();
  for (int i = 0; i < a.n; ++i) r.c[i] = m_add(P, r.c[i], a.c[i]);
  for (int i = 0; i < b.n; ++i) r.c[i] = m_add(P, r.c[i], b.c[i]);
  return r;
}
static upoly up_mul(const or_params* P, upoly a, upoly b) { /* :95-109 (degree() trims both) */
  up_trim(&a);
  up_trim(&b);
  upoly r;
  r.n = (a.n - 1) + (b.n - 1) + 1;
  for (int i = 0; i < r.n; ++i) r.c[i] = m_zero();
  for (int i = 0; i < a.n; ++i)
    for (int j = 0; j < b.n; ++j) r.c[i + j] = m_add(P, r.c[i + j], m_mul(P, a.c[i], b.c[j]));
  return r;
}
static mfe up_evaluate(const or_params* P, const upoly* p, mfe x) { /* :20-26 */
  mfe s = m_zero();
  for (int i = 0; i < p->n; ++i) {
    uint64_t e = (uint64_t)i;
    s = m_add(P, s, m_mul(P, p->c[i], m_pow(P, x, &e, 1)));
  }
  return s;
}
static upoly up_interpolate(const or_params* P, const mfe* xs, const mfe* ys, int n) { /* :48-74 */
  upoly result;
  result.n = 1;
  result.c[0] = m_zero();
  for (int i = 0; i < n; ++i) {
    upoly li;
    li.n = 1;
    li.c[0] = m_from_u64(P, 1);
    for (int j = 0; j < n; ++j) {
      if (i == j) continue;
      upoly num;
      num.n = 2;
      num.c[0] = m_neg(P, xs[j]);
      num.c[1] = m_from_u64(P, 1);
      mfe den = m_sub(P, xs[i], xs[j]);
      li = up_mul(P, li, up_scalar_mul(P, num, m_inv(P, den)));
    }
    result = up_add(P, result, up_scalar_mul(P, li, ys[i]));
  }
  up_trim(&result);
  return result;
}
int or_interpolate(int field, const or_fe* xs, const or_fe* ys, int npts, or_fe* coeffs_out) {
  const or_params* P = params(field);
  if (!P || npts < 1 || npts > 8) return -1;
  mfe X[8], Y[8];
  for (int i = 0; i < npts; ++i) {
    X[i] = m_from_canon(P, &xs[i]);
    Y[i] = m_from_canon(P, &ys[i]);
  }
  upoly r = up_interpolate(P, X, Y, npts);
  for (int i = 0; i < r.n; ++i) coeffs_out[i] = m_to_canon(P, r.c[i]);
  return r.n;
}

/* ------------------------------------------------------------------------ */
/* sum-check (sum_check_protocol.rs)                                        */
/* ------------------------------------------------------------------------ */
static void tr_append_mle(const or_params* P, or_transcript* t, const mle* a) {
  tr_append_fes(P, t, a->ev, a->len);
}

/* prove (:25-52) + get_round_partial_polynomial_proof (:168-175) */
int or_sumcheck_prove(int field, const or_fe* evals, uint32_t nvars, or_fe* out_round_polys, or_fe* out_claimed_sum) {
  const or_params* P = params(field);
  if (!P) return -1;
  mle poly = mle_from_canon(P, evals, (size_t)1 << nvars);
  or_transcript* t = or_transcript_new();
  tr_append_mle(P, t, &poly);
  mfe claimed = m_zero();
  for (size_t i = 0; i < poly.len; ++i) claimed = m_add(P, claimed, poly.ev[i]);
  tr_append_fes(P, t, &claimed, 1);
  mle cur = mle_clone(&poly);
  for (uint32_t k = 0; k < nvars; ++k) {
    size_t mid = cur.len / 2;
    mfe rp[2] = {m_zero(), m_zero()};
    for (size_t i = 0; i < mid; ++i) rp[0] = m_add(P, rp[0], cur.ev[i]);
    for (size_t i = mid; i < cur.len; ++i) rp[1] = m_add(P, rp[1], cur.ev[i]);
    tr_append_fes(P, t, rp, 2);
    out_round_polys[2 * k] = m_to_canon(P, rp[0]);
    out_round_polys[2 * k + 1] = m_to_canon(P, rp[1]);
    mfe r = tr_challenge(P, t);
    mle nx = mle_partial_evaluate(P, &cur, 0, r);
    mle_free(&cur);
    cur = nx;
  }
  *out_claimed_sum = m_to_canon(P, claimed);
  mle_free(&cur);
  mle_free(&poly);
  or_transcript_free(t);
  return 0;
}

/* verify (:54-84) */
int or_sumcheck_verify(int field, const or_fe* evals, uint32_t nvars, const or_fe* round_polys, uint32_t nrounds,
                       uint32_t poly_len, const or_fe* claimed_sum) {
  const or_params* P = params(field);
  if (!P) return -2;
  if (nrounds > 0 && !is_pow2_len(poly_len)) return -1; /* MultilinearPoly::new panics */
  mle poly = mle_from_canon(P, evals, (size_t)1 << nvars);
  or_transcript* t = or_transcript_new();
  tr_append_mle(P, t, &poly);
  mfe expected = m_from_canon(P, claimed_sum);
  tr_append_fes(P, t, &expected, 1);
  mfe* chal = (mfe*)malloc((nrounds + 1) * sizeof(mfe));
  mfe* pv = (mfe*)malloc(poly_len * sizeof(mfe));
  mle cur = mle_clone(&poly);
  int result = 1;
  for (uint32_t k = 0; k < nrounds; ++k) {
    mfe s = m_zero();
    for (uint32_t i = 0; i < poly_len; ++i) {
      pv[i] = m_from_canon(P, &round_polys[(size_t)k * poly_len + i]);
      s = m_add(P, s, pv[i]);
    }
    if (!m_eq(s, expected)) {
      result = 0;
      goto done;
    }
    if (poly_len < 2) { /* poly.evaluation[1] out of bounds -> panic */
      result = -1;
      goto done;
    }
    tr_append_fes(P, t, pv, poly_len);
    mfe r = tr_challenge(P, t);
    expected = m_add(P, pv[0], m_mul(P, r, m_sub(P, pv[1], pv[0])));
    if (cur.nvars > 0) { /* redundant fold (:76); panics once the table is exhausted */
      mle nx = mle_partial_evaluate(P, &cur, 0, r);
      mle_free(&cur);
      cur = nx;
    } else {
      result = -1;
      goto done;
    }
    chal[k] = r;
  }
  if (nrounds != nvars) { /* evaluate() panics on a length mismatch (:80-82) */
    result = -1;
    goto done;
  }
  result = m_eq(expected, mle_evaluate(P, &poly, chal)) ? 1 : 0;
done:
  mle_free(&cur);
  mle_free(&poly);
  free(chal);
  free(pv);
  or_transcript_free(t);
  return result;
}

/* ProductPoly / SumPoly (composed_polynomial.rs:5-103), 2 products x 2 factors */
typedef struct {
  mle f[2][2];
} sumpoly;

static mle mle_copy_vec(const mle* a) { return mle_clone(a); } /* ProductPoly::new to_vec (:23-26) */

/* SumPoly::partial_evaluate (:78-86) -> ProductPoly::partial_evaluate (:38-50) */
static sumpoly sp_partial_evaluate(const or_params* P, const sumpoly* s, mfe v) {
  sumpoly r;
  for (int a = 0; a < 2; ++a)
    for (int b = 0; b < 2; ++b) {
      mle part = mle_partial_evaluate(P, &s->f[a][b], 0, v);
      r.f[a][b] = mle_copy_vec(&part); /* ProductPoly::new(partial_polys) copies again */
      mle_free(&part);
    }
  return r;
}
static void sp_free(sumpoly* s) {
  for (int a = 0; a < 2; ++a)
    for (int b = 0; b < 2; ++b) mle_free(&s->f[a][b]);
}
/* SumPoly::reduce (:88-99) with ProductPoly::reduce (:52-54), then .iter().sum() */
static mfe sp_reduce_sum(const or_params* P, const sumpoly* s) {
  size_t n = s->f[0][0].len;
  mfe* red[2];
  for (int a = 0; a < 2; ++a) {
    mle x = mle_clone(&s->f[a][0]), y = mle_clone(&s->f[a][1]);
    red[a] = (mfe*)malloc(n * sizeof(mfe));
    for (size_t i = 0; i < n; ++i) red[a][i] = m_mul(P, x.ev[i], y.ev[i]);
    mle_free(&x);
    mle_free(&y);
  }
  mfe* res = (mfe*)malloc(n * sizeof(mfe));
  for (size_t i = 0; i < n; ++i) res[i] = m_add(P, red[0][i], red[1][i]);
  mfe sum = m_zero();
  for (size_t i = 0; i < n; ++i) sum = m_add(P, sum, res[i]);
  free(res);
  free(red[0]);
  free(red[1]);
  return sum;
}

/* gkr_prove (:86-115) + get_round_partial_polynomial_proof_gkr (:152-166) */
int or_gkr_prove(int field, const or_fe* const tables[4], uint32_t nvars, or_transcript* t, or_fe* out_coeffs,
                 uint8_t* out_ncoeffs, or_fe* out_challenges) {
  const or_params* P = params(field);
  if (!P) return -1;
  size_t N = (size_t)1 << nvars;
  sumpoly cur;
  for (int k = 0; k < 4; ++k) cur.f[k / 2][k % 2] = mle_from_canon(P, tables[k], N);
  const int degree = 2; /* SumPoly::get_degree = #factors of polys[0] */
  for (uint32_t round = 0; round < nvars; ++round) {
    mfe xs[3], ys[3];
    for (int i = 0; i <= degree; ++i) {
      xs[i] = m_from_u64(P, (uint64_t)i);
      sumpoly part = sp_partial_evaluate(P, &cur, xs[i]);
      ys[i] = sp_reduce_sum(P, &part);
      sp_free(&part);
    }
    upoly rp = up_interpolate(P, xs, ys, degree + 1);
    tr_append_fes(P, t, rp.c, (size_t)rp.n);
    out_ncoeffs[round] = (uint8_t)rp.n;
    for (int i = 0; i < 3; ++i) out_coeffs[3 * round + i] = m_to_canon(P, i < rp.n ? rp.c[i] : m_zero());
    mfe r = tr_challenge(P, t);
    out_challenges[round] = m_to_canon(P, r);
    sumpoly nx = sp_partial_evaluate(P, &cur, r);
    sp_free(&cur);
    cur = nx;
  }
  sp_free(&cur);
  return 0;
}

/* The fast CPU restatement ("also report the fast OpenMP
 * restatement on all cores"): the same transcript as or_gkr_prove, without the
 * reference's per-round copies. Per round one parallel pass computes the three
 * evaluations e_t = sum_j A_t S_t + M_t P_t (X_t = X_lo + t (X_hi - X_lo)),
 * the round polynomial is interpolated and trimmed exactly as above, and a
 * second pass folds the four tables in place: 10 Montgomery muls per pair. */
int or_gkr_prove_fast(int field, const or_fe* const tables[4], uint32_t nvars, or_transcript* t, or_fe* out_coeffs,
                      uint8_t* out_ncoeffs, or_fe* out_challenges) {
  const or_params* P = params(field);
  if (!P) return -1;
  const size_t N = (size_t)1 << nvars;
  mfe* X[4];
  for (int k = 0; k < 4; ++k) {
    X[k] = (mfe*)malloc(N * sizeof(mfe));
    if (!X[k]) {
      for (int q = 0; q < k; ++q) free(X[q]);
      return -1;
    }
    mfe* dst = X[k];
    const or_fe* src = tables[k];
#pragma omp parallel for schedule(static)
    for (size_t i = 0; i < N; ++i) dst[i] = m_from_canon(P, &src[i]);
  }
  mfe xs[3];
  for (int i = 0; i < 3; ++i) xs[i] = m_from_u64(P, (uint64_t)i);
  size_t len = N;
  for (uint32_t round = 0; round < nvars; ++round) {
    const size_t h = len / 2;
    mfe e[3] = {m_zero(), m_zero(), m_zero()};
#pragma omp parallel
    {
      mfe acc[3] = {m_zero(), m_zero(), m_zero()};
#pragma omp for schedule(static) nowait
      for (size_t j = 0; j < h; ++j) {
        mfe v[4][3];
        for (int k = 0; k < 4; ++k) {
          v[k][0] = X[k][j];
          v[k][1] = X[k][j + h];
          v[k][2] = m_sub(P, m_add(P, v[k][1], v[k][1]), v[k][0]);
        }
        for (int q = 0; q < 3; ++q)
          acc[q] = m_add(P, acc[q], m_add(P, m_mul(P, v[0][q], v[1][q]), m_mul(P, v[2][q], v[3][q])));
      }
#pragma omp critical
      for (int q = 0; q < 3; ++q) e[q] = m_add(P, e[q], acc[q]);
    }
    upoly rp = up_interpolate(P, xs, e, 3);
    tr_append_fes(P, t, rp.c, (size_t)rp.n);
    out_ncoeffs[round] = (uint8_t)rp.n;
    for (int i = 0; i < 3; ++i) out_coeffs[3 * round + i] = m_to_canon(P, i < rp.n ? rp.c[i] : m_zero());
    const mfe r = tr_challenge(P, t);
    out_challenges[round] = m_to_canon(P, r);
#pragma omp parallel for schedule(static)
    for (size_t j = 0; j < h; ++j)
      for (int k = 0; k < 4; ++k) X[k][j] = m_add(P, X[k][j], m_mul(P, r, m_sub(P, X[k][j + h], X[k][j])));
    len = h;
  }
  for (int k = 0; k < 4; ++k) free(X[k]);
  return 0;
}

int or_threads(void) {
#ifdef _OPENMP
  return omp_get_max_threads();
#else
  return 1;
#endif
}

/* gkr_verify (:117-150) */
int or_gkr_verify(int field, const or_fe* coeffs, const uint8_t* ncoeffs, uint32_t nrounds, const or_fe* claimed_sum,
                  or_transcript* t, or_fe* out_final_claim, or_fe* out_challenges) {
  const or_params* P = params(field);
  if (!P) return -1;
  mfe claim = m_from_canon(P, claimed_sum);
  mfe zero = m_zero(), one = m_from_u64(P, 1);
  for (uint32_t k = 0; k < nrounds; ++k) {
    upoly rp;
    rp.n = ncoeffs[k];
    for (int i = 0; i < rp.n; ++i) rp.c[i] = m_from_canon(P, &coeffs[3 * k + i]);
    mfe f0 = up_evaluate(P, &rp, zero), f1 = up_evaluate(P, &rp, one);
    if (!m_eq(m_add(P, f0, f1), claim)) {
      *out_final_claim = m_to_canon(P, zero);
      out_challenges[0] = m_to_canon(P, zero);
      return 0;
    }
    tr_append_fes(P, t, rp.c, (size_t)rp.n);
    mfe r = tr_challenge(P, t);
    out_challenges[k] = m_to_canon(P, r);
    claim = up_evaluate(P, &rp, r);
  }
  *out_final_claim = m_to_canon(P, claim);
  return 1;
}

/* ------------------------------------------------------------------------ */
/* Synthetic inputs: counter-based SplitMix64, mod p        */
/* ------------------------------------------------------------------------ */
static uint64_t sm64(uint64_t x) {
  uint64_t z = x + 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
void or_synth_fill(int field, uint64_t seed, uint32_t table, uint64_t index0, uint64_t count, or_fe* out) {
  const or_params* P = params(field);
  if (!P) return;
  uint64_t key = sm64(sm64(seed) + table);
  /* counter-based: every element depends only on its index, so the parallel
   * fill is identical to the serial one (the headline-size fixtures fill
   * 4 x 2^26 elements) */
#pragma omp parallel for schedule(static) if (count >= (1u << 16))
  for (uint64_t n = 0; n < count; ++n) {
    uint64_t i = index0 + n;
    uint64_t v[4];
    for (int k = 0; k < 4; ++k) v[k] = sm64(key + 4 * i + (uint64_t)k);
    while (geq_p(v, P->p)) sub_p(v, P->p);
    memcpy(out[n].l, v, 32);
  }
}
