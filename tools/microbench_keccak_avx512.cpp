// AVX-512 Keccak-f[1600] (one state in five zmm rows) against the scalar/BMI permutation of
// csrc/keccak.hpp: bit-exactness over random states, and ns per permutation.
// g++ -O3 -std=c++17 tools/microbench_keccak_avx512.cpp -o /tmp/mb_kavx
#include <immintrin.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>
#include <chrono>
#include "../zk-research-implementations_amd/csrc/keccak.hpp"

__attribute__((target("avx512f,avx512vl"))) static void permute_avx512(uint64_t* A) {
  static const uint64_t RC[24] = {
      0x0000000000000001ull, 0x0000000000008082ull, 0x800000000000808aull, 0x8000000080008000ull,
      0x000000000000808bull, 0x0000000080000001ull, 0x8000000080008081ull, 0x8000000000008009ull,
      0x000000000000008aull, 0x0000000000000088ull, 0x0000000080008009ull, 0x000000008000000aull,
      0x000000008000808bull, 0x800000000000008bull, 0x8000000000008089ull, 0x8000000000008003ull,
      0x8000000000008002ull, 0x8000000000000080ull, 0x000000000000800aull, 0x800000008000000aull,
      0x8000000080008081ull, 0x8000000000008080ull, 0x0000000080000001ull, 0x8000000080008008ull};
  const __mmask8 m5 = 0x1F;
  __m512i R0 = _mm512_maskz_loadu_epi64(m5, A + 0), R1 = _mm512_maskz_loadu_epi64(m5, A + 5),
          R2 = _mm512_maskz_loadu_epi64(m5, A + 10), R3 = _mm512_maskz_loadu_epi64(m5, A + 15),
          R4 = _mm512_maskz_loadu_epi64(m5, A + 20);
  const __m512i pm1 = _mm512_setr_epi64(4, 0, 1, 2, 3, 5, 6, 7), pp1 = _mm512_setr_epi64(1, 2, 3, 4, 0, 5, 6, 7),
                pp2 = _mm512_setr_epi64(2, 3, 4, 0, 1, 5, 6, 7);
  const __m512i rot0 = _mm512_setr_epi64(0, 1, 62, 28, 27, 0, 0, 0), rot1 = _mm512_setr_epi64(36, 44, 6, 55, 20, 0, 0, 0),
                rot2 = _mm512_setr_epi64(3, 10, 43, 25, 39, 0, 0, 0), rot3 = _mm512_setr_epi64(41, 45, 15, 21, 8, 0, 0, 0),
                rot4 = _mm512_setr_epi64(18, 2, 61, 56, 14, 0, 0, 0);
  // pi: new row k lane y = R_y[(3k + y) % 5]. Stage A pairs rows (0,1) and (2,3):
  // P01lo = (R0[i(0,0)], R1[i(0,1)], R0[i(1,0)], R1[i(1,1)], ... k = 0..3), P01hi = (k = 4, ...)
  // i(k, y) = (3k + y) % 5; in permutex2var, indices 0-7 pick a, 8-15 pick b
#define I(k, y) (((3 * (k) + (y)) % 5))
  const __m512i a01lo = _mm512_setr_epi64(I(0, 0), 8 + I(0, 1), I(1, 0), 8 + I(1, 1), I(2, 0), 8 + I(2, 1), I(3, 0), 8 + I(3, 1));
  const __m512i a01hi = _mm512_setr_epi64(I(4, 0), 8 + I(4, 1), 0, 0, 0, 0, 0, 0);
  const __m512i a23lo = _mm512_setr_epi64(I(0, 2), 8 + I(0, 3), I(1, 2), 8 + I(1, 3), I(2, 2), 8 + I(2, 3), I(3, 2), 8 + I(3, 3));
  const __m512i a23hi = _mm512_setr_epi64(I(4, 2), 8 + I(4, 3), 0, 0, 0, 0, 0, 0);
  // stage B: out_k = (P01[2k], P01[2k+1], P23[2k], P23[2k+1]) then lane 4 = R4[i(k, 4)]
  const __m512i b0 = _mm512_setr_epi64(0, 1, 8, 9, 0, 0, 0, 0), b1 = _mm512_setr_epi64(2, 3, 10, 11, 0, 0, 0, 0),
                b2 = _mm512_setr_epi64(4, 5, 12, 13, 0, 0, 0, 0), b3 = _mm512_setr_epi64(6, 7, 14, 15, 0, 0, 0, 0);
  const __m512i c0 = _mm512_setr_epi64(0, 1, 2, 3, 8 + I(0, 4), 5, 6, 7), c1 = _mm512_setr_epi64(0, 1, 2, 3, 8 + I(1, 4), 5, 6, 7),
                c2 = _mm512_setr_epi64(0, 1, 2, 3, 8 + I(2, 4), 5, 6, 7), c3 = _mm512_setr_epi64(0, 1, 2, 3, 8 + I(3, 4), 5, 6, 7),
                c4 = _mm512_setr_epi64(0, 1, 2, 3, 8 + I(4, 4), 5, 6, 7);
#undef I
  for (int round = 0; round < 24; ++round) {
    const __m512i C = _mm512_ternarylogic_epi64(_mm512_ternarylogic_epi64(R0, R1, R2, 0x96), R3, R4, 0x96);
    const __m512i D = _mm512_xor_si512(_mm512_permutexvar_epi64(pm1, C), _mm512_rol_epi64(_mm512_permutexvar_epi64(pp1, C), 1));
    R0 = _mm512_rolv_epi64(_mm512_xor_si512(R0, D), rot0);
    R1 = _mm512_rolv_epi64(_mm512_xor_si512(R1, D), rot1);
    R2 = _mm512_rolv_epi64(_mm512_xor_si512(R2, D), rot2);
    R3 = _mm512_rolv_epi64(_mm512_xor_si512(R3, D), rot3);
    R4 = _mm512_rolv_epi64(_mm512_xor_si512(R4, D), rot4);
    const __m512i P01lo = _mm512_permutex2var_epi64(R0, a01lo, R1), P01hi = _mm512_permutex2var_epi64(R0, a01hi, R1);
    const __m512i P23lo = _mm512_permutex2var_epi64(R2, a23lo, R3), P23hi = _mm512_permutex2var_epi64(R2, a23hi, R3);
    const __m512i B0 = _mm512_permutex2var_epi64(_mm512_permutex2var_epi64(P01lo, b0, P23lo), c0, R4);
    const __m512i B1 = _mm512_permutex2var_epi64(_mm512_permutex2var_epi64(P01lo, b1, P23lo), c1, R4);
    const __m512i B2 = _mm512_permutex2var_epi64(_mm512_permutex2var_epi64(P01lo, b2, P23lo), c2, R4);
    const __m512i B3 = _mm512_permutex2var_epi64(_mm512_permutex2var_epi64(P01lo, b3, P23lo), c3, R4);
    const __m512i B4 = _mm512_permutex2var_epi64(_mm512_permutex2var_epi64(P01hi, b0, P23hi), c4, R4);
    // chi: B ^ (~B[x+1] & B[x+2])   (ternary logic a ^ (~b & c) = 0xD2)
    R0 = _mm512_ternarylogic_epi64(B0, _mm512_permutexvar_epi64(pp1, B0), _mm512_permutexvar_epi64(pp2, B0), 0xD2);
    R1 = _mm512_ternarylogic_epi64(B1, _mm512_permutexvar_epi64(pp1, B1), _mm512_permutexvar_epi64(pp2, B1), 0xD2);
    R2 = _mm512_ternarylogic_epi64(B2, _mm512_permutexvar_epi64(pp1, B2), _mm512_permutexvar_epi64(pp2, B2), 0xD2);
    R3 = _mm512_ternarylogic_epi64(B3, _mm512_permutexvar_epi64(pp1, B3), _mm512_permutexvar_epi64(pp2, B3), 0xD2);
    R4 = _mm512_ternarylogic_epi64(B4, _mm512_permutexvar_epi64(pp1, B4), _mm512_permutexvar_epi64(pp2, B4), 0xD2);
    R0 = _mm512_mask_xor_epi64(R0, 1, R0, _mm512_set1_epi64((long long)RC[round]));
  }
  _mm512_mask_storeu_epi64(A + 0, m5, R0);
  _mm512_mask_storeu_epi64(A + 5, m5, R1);
  _mm512_mask_storeu_epi64(A + 10, m5, R2);
  _mm512_mask_storeu_epi64(A + 15, m5, R3);
  _mm512_mask_storeu_epi64(A + 20, m5, R4);
}

int main() {
  uint64_t s = 0x1234567;
  auto rnd = [&]() { s ^= s << 13; s ^= s >> 7; s ^= s << 17; return s; };
  for (int t = 0; t < 1000; ++t) {
    uint64_t A[25], B[25];
    for (int i = 0; i < 25; ++i) A[i] = B[i] = rnd();
    zk::Keccak256::permute(A);
    permute_avx512(B);
    if (memcmp(A, B, sizeof A)) { printf("MISMATCH at %d\n", t); return 1; }
  }
  uint64_t A[25] = {0};
  const int N = 2000000;
  auto t0 = std::chrono::steady_clock::now();
  for (int i = 0; i < N; ++i) zk::Keccak256::permute(A);
  auto t1 = std::chrono::steady_clock::now();
  for (int i = 0; i < N; ++i) permute_avx512(A);
  auto t2 = std::chrono::steady_clock::now();
  printf("ok; scalar %.1f ns, avx512 %.1f ns per permutation (%llx)\n",
         std::chrono::duration<double, std::nano>(t1 - t0).count() / N, std::chrono::duration<double, std::nano>(t2 - t1).count() / N, (unsigned long long)A[0]);
}
