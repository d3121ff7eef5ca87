// Keccak-f[1600] for one wave on the scalar unit.
//
// Every lane of the calling wave passes the same state; the words are made
// wave-uniform with readfirstlane so the compiler keeps the permutation on
// SGPRs / SALU (s_xor_b64, s_andn2_b64, 64-bit shifts): one permutation per
// Fiat-Shamir round, no per-lane duplication of the work.
// Semantics identical to zk::Keccak256::permute (keccak.hpp).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace zk {

__device__ __forceinline__ uint64_t uni64(uint64_t x) {
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)x);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(x >> 32));
  return (uint64_t)lo | ((uint64_t)hi << 32);
}
__device__ __forceinline__ uint64_t drol(uint64_t x, int s) { return (x << s) | (x >> (64 - s)); }

__device__ __forceinline__ void keccak_f1600_uniform(uint64_t* A) {
  uint64_t a[25];
#pragma unroll
  for (int i = 0; i < 25; ++i) a[i] = uni64(A[i]);
  constexpr uint64_t RC[24] = {
      0x0000000000000001ull, 0x0000000000008082ull, 0x800000000000808aull, 0x8000000080008000ull,
      0x000000000000808bull, 0x0000000080000001ull, 0x8000000080008081ull, 0x8000000000008009ull,
      0x000000000000008aull, 0x0000000000000088ull, 0x0000000080008009ull, 0x000000008000000aull,
      0x000000008000808bull, 0x800000000000008bull, 0x8000000000008089ull, 0x8000000000008003ull,
      0x8000000000008002ull, 0x8000000000000080ull, 0x000000000000800aull, 0x800000008000000aull,
      0x8000000080008081ull, 0x8000000000008080ull, 0x0000000080000001ull, 0x8000000080008008ull};
#pragma unroll 1
  for (int round = 0; round < 24; ++round) {
    const uint64_t C0 = a[0] ^ a[5] ^ a[10] ^ a[15] ^ a[20];
    const uint64_t C1 = a[1] ^ a[6] ^ a[11] ^ a[16] ^ a[21];
    const uint64_t C2 = a[2] ^ a[7] ^ a[12] ^ a[17] ^ a[22];
    const uint64_t C3 = a[3] ^ a[8] ^ a[13] ^ a[18] ^ a[23];
    const uint64_t C4 = a[4] ^ a[9] ^ a[14] ^ a[19] ^ a[24];
    const uint64_t D0 = C4 ^ drol(C1, 1), D1 = C0 ^ drol(C2, 1), D2 = C1 ^ drol(C3, 1), D3 = C2 ^ drol(C4, 1),
                   D4 = C3 ^ drol(C0, 1);
    const uint64_t B0 = a[0] ^ D0;
    const uint64_t B10 = drol(a[1] ^ D1, 1);
    const uint64_t B20 = drol(a[2] ^ D2, 62);
    const uint64_t B5 = drol(a[3] ^ D3, 28);
    const uint64_t B15 = drol(a[4] ^ D4, 27);
    const uint64_t B16 = drol(a[5] ^ D0, 36);
    const uint64_t B1 = drol(a[6] ^ D1, 44);
    const uint64_t B11 = drol(a[7] ^ D2, 6);
    const uint64_t B21 = drol(a[8] ^ D3, 55);
    const uint64_t B6 = drol(a[9] ^ D4, 20);
    const uint64_t B7 = drol(a[10] ^ D0, 3);
    const uint64_t B17 = drol(a[11] ^ D1, 10);
    const uint64_t B2 = drol(a[12] ^ D2, 43);
    const uint64_t B12 = drol(a[13] ^ D3, 25);
    const uint64_t B22 = drol(a[14] ^ D4, 39);
    const uint64_t B23 = drol(a[15] ^ D0, 41);
    const uint64_t B8 = drol(a[16] ^ D1, 45);
    const uint64_t B18 = drol(a[17] ^ D2, 15);
    const uint64_t B3 = drol(a[18] ^ D3, 21);
    const uint64_t B13 = drol(a[19] ^ D4, 8);
    const uint64_t B14 = drol(a[20] ^ D0, 18);
    const uint64_t B24 = drol(a[21] ^ D1, 2);
    const uint64_t B9 = drol(a[22] ^ D2, 61);
    const uint64_t B19 = drol(a[23] ^ D3, 56);
    const uint64_t B4 = drol(a[24] ^ D4, 14);
    a[0] = B0 ^ (~B1 & B2) ^ RC[round];
    a[1] = B1 ^ (~B2 & B3);
    a[2] = B2 ^ (~B3 & B4);
    a[3] = B3 ^ (~B4 & B0);
    a[4] = B4 ^ (~B0 & B1);
    a[5] = B5 ^ (~B6 & B7);
    a[6] = B6 ^ (~B7 & B8);
    a[7] = B7 ^ (~B8 & B9);
    a[8] = B8 ^ (~B9 & B5);
    a[9] = B9 ^ (~B5 & B6);
    a[10] = B10 ^ (~B11 & B12);
    a[11] = B11 ^ (~B12 & B13);
    a[12] = B12 ^ (~B13 & B14);
    a[13] = B13 ^ (~B14 & B10);
    a[14] = B14 ^ (~B10 & B11);
    a[15] = B15 ^ (~B16 & B17);
    a[16] = B16 ^ (~B17 & B18);
    a[17] = B17 ^ (~B18 & B19);
    a[18] = B18 ^ (~B19 & B15);
    a[19] = B19 ^ (~B15 & B16);
    a[20] = B20 ^ (~B21 & B22);
    a[21] = B21 ^ (~B22 & B23);
    a[22] = B22 ^ (~B23 & B24);
    a[23] = B23 ^ (~B24 & B20);
    a[24] = B24 ^ (~B20 & B21);
  }
#pragma unroll
  for (int i = 0; i < 25; ++i) A[i] = a[i];
}

}  // namespace zk
