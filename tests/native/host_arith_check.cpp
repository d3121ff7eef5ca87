// Host-arithmetic checker for tests/test_host_arith_cpu.py (test infrastructure,
// not the product): reads lines "L product w0 .. w_{L-1}" (hex u64 limb sums at
// 32-bit positions) and prints hlimbs_to_fe's result (hex, 4 LE u64 limbs, the
// Montgomery image); lines "M a0..a3 b0..b3 c0..c3 d0..d3" print wide_to_fe of
// mac_wide(a, b) + mac_wide(c, d). Field: argv[1] = 0 (BN254 Fr), 1 (BN254 Fq), 2 (BLS12-381 Fr).
#include <cinttypes>
#include <cstdio>
#include <cstring>
#include <string>

#include "hfield.hpp"

using namespace zk;

template <class F>
int run() {
  char op[8];
  while (scanf("%7s", op) == 1) {
    Fe r;
    if (op[0] == 'M') {
      uint64_t v[16];
      for (auto& x : v) scanf("%" SCNx64, &x);
      uint64_t acc[9] = {0};
      h64::V a, b, c, d;
      memcpy(a.l, v, 32);
      memcpy(b.l, v + 4, 32);
      memcpy(c.l, v + 8, 32);
      memcpy(d.l, v + 12, 32);
      h64::mac_wide(acc, a, b);
      h64::mac_wide(acc, c, d);
      r = wide_to_fe<F>(acc);
    } else {
      int L = atoi(op), product = 0;
      scanf("%d", &product);
      uint64_t w[24];
      for (int i = 0; i < L; ++i) scanf("%" SCNx64, &w[i]);
      r = hlimbs_to_fe<F>(w, L, product != 0);
    }
    const h64::V o = h64::of(r);
    printf("%016" PRIx64 " %016" PRIx64 " %016" PRIx64 " %016" PRIx64 "\n", o.l[0], o.l[1], o.l[2], o.l[3]);
  }
  return 0;
}

int main(int argc, char** argv) {
  const int f = argc > 1 ? atoi(argv[1]) : 0;
  return f == 0 ? run<Bn254Fr>() : f == 1 ? run<Bn254Fq>() : run<Bls12_381Fr>();
}
