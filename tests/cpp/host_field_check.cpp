// Host field arithmetic of the per-round hand-off (csrc/hfield.hpp), checked on
// the CPU (tests/test_host_field_cpu.py builds and runs this):
//  * hlimbs_to_fe's fast path for <= 9 limb sums of products (the matrix-core
//    steps' output) against its generic path (the same words padded to L = 10,
//    which takes the generic route), on random, small, all-ones and 32-bit words;
//  * hfe_half against multiplication by 1/2 (finish_round's c2, the Lagrange
//    weights of two_rounds);
//  * wide_to_fe's one-REDC path against the generic conversion (sums of 1-4
//    products of BLS12-381 Fr elements: 3p^2 exceeds p R there, so both paths run).
// Prints the time of 27 conversions (one three-round step's worth).
#include <chrono>
#include <cstdio>
#include <cstring>
#include <random>
#include "hfield.hpp"
using namespace zk;
template <class F>
int check(const char* name) {
  std::mt19937_64 g(7);
  int bad = 0;
  for (int it = 0; it < 2000000; ++it) {
    uint64_t w[10] = {0};
    const int L = 1 + (int)(g() % 9);
    const int mode = it % 4;
    for (int i = 0; i < L; ++i) w[i] = mode == 0 ? g() : mode == 1 ? (g() >> 20) : mode == 2 ? ~0ull : (g() & 0xffffffffull);
    const Fe a = hlimbs_to_fe<F>(w, L, true);
    const Fe b = hlimbs_to_fe<F>(w, 10, true);
    bad += memcmp(&a, &b, sizeof a) != 0;
  }
  uint64_t w[9];
  std::mt19937_64 g2(1);
  for (auto& x : w) x = g2() >> 24;
  Fe out[27];
  const int N = 200000;
  auto t0 = std::chrono::steady_clock::now();
  uint32_t sink = 0;
  for (int it = 0; it < N; ++it) {
    w[it % 9] ^= it;
    for (int k = 0; k < 27; ++k) out[k] = hlimbs_to_fe<F>(w, 9, true);
    sink += out[it % 27].v[0];
  }
  const double us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count() / N;
  printf("%s: %d mismatches; 27 conversions %.3f us (%u)\n", name, bad, us, sink & 1);
  return bad;
}
int main() {
  int bad = check<Bn254Fr>("bn254_fr") + check<Bn254Fq>("bn254_fq") + check<Bls12_381Fr>("bls12_381_fr");
  // hfe_half against multiplication by 1/2
  std::mt19937_64 g(3);
  for (int it = 0; it < 1000000; ++it) {
    Fe x;
    for (int i = 0; i < 8; ++i) x.v[i] = (uint32_t)g();
    x.v[7] &= 0x0fffffffu;
    x = hfe_to_mont<Bn254Fr>(x);
    const Fe a = hfe_half<Bn254Fr>(x), b = hfe_mul<Bn254Fr>(x, fe_inv2<Bn254Fr>());
    bad += memcmp(&a, &b, sizeof a) != 0;
  }
  // wide_to_fe's one-REDC path against the generic conversion of the same 576-bit value
  for (int it = 0; it < 1000000; ++it) {
    uint64_t acc[9] = {0};
    const int np = 1 + it % 4;
    for (int k = 0; k < np; ++k) {
      Fe a, b;
      for (int i = 0; i < 8; ++i) {
        a.v[i] = (uint32_t)g();
        b.v[i] = (uint32_t)g();
      }
      a = hfe_to_mont<Bls12_381Fr>(a);
      b = hfe_to_mont<Bls12_381Fr>(b);
      h64::mac_wide(acc, h64::of(a), h64::of(b));
    }
    uint64_t w[18];
    for (int k = 0; k < 9; ++k) {
      w[2 * k] = (uint32_t)acc[k];
      w[2 * k + 1] = acc[k] >> 32;
    }
    const Fe x = wide_to_fe<Bls12_381Fr>(acc), y = hlimbs_to_fe<Bls12_381Fr>(w, 18, true);
    bad += memcmp(&x, &y, sizeof x) != 0;
  }
  printf("total mismatches %d\n", bad);
  return bad != 0;
}
