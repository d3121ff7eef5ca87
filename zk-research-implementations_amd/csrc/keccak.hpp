// Keccak-256 sponge and the Fiat-Shamir transcript (host side).
//
// Restates fiat_shamir/src/fiat_shamir_transcript.rs:5-37 over sha3 0.10.8's
// `Keccak256` (Keccak[c=512]: rate 136 B, original Keccak padding 0x01..0x80;
// Cargo.lock:869-872 sha3 0.10.8, :559-562 keccak 0.1.5):
//   append(b)              -> absorb b
//   get_random_challenge() -> d = finalize_reset(); absorb(d); F::from_le_bytes_mod_order(d)
#pragma once
#include <stddef.h>
#include <stdint.h>
#include <string.h>

namespace zk {

struct Keccak256 {
  static constexpr size_t RATE = 136;
  uint64_t st[25];
  uint8_t buf[RATE];
  size_t fill;

  Keccak256() { reset(); }
  void reset() {
    memset(st, 0, sizeof st);
    fill = 0;
  }

  static inline uint64_t rol(uint64_t x, int s) { return (x << s) | (x >> (64 - s)); }

  // The permutation body is compiled twice: with BMI1/BMI2 (andn for chi,
  // rorx for the rotations) for hosts that have them, and for baseline
  // x86-64; permute() picks one once per process. The transcript's absorb of
  // a plain prove's table is a serial sponge on the host, so its
  // speed is the floor of plain prove / verify.
  static void permute(uint64_t* A) {
#if defined(__x86_64__) && !defined(__HIP_DEVICE_COMPILE__)
    static const bool bmi = __builtin_cpu_supports("bmi") && __builtin_cpu_supports("bmi2");
    if (bmi) {
      permute_bmi(A);
      return;
    }
#endif
    permute_body(A);
  }
#if defined(__x86_64__) && !defined(__HIP_DEVICE_COMPILE__)
  __attribute__((target("bmi,bmi2"))) static void permute_bmi(uint64_t* A) { permute_body(A); }
#endif
  __attribute__((always_inline)) static inline void permute_body(uint64_t* A) {
    static const uint64_t RC[24] = {
        0x0000000000000001ull, 0x0000000000008082ull, 0x800000000000808aull, 0x8000000080008000ull,
        0x000000000000808bull, 0x0000000080000001ull, 0x8000000080008081ull, 0x8000000000008009ull,
        0x000000000000008aull, 0x0000000000000088ull, 0x0000000080008009ull, 0x000000008000000aull,
        0x000000008000808bull, 0x800000000000008bull, 0x8000000000008089ull, 0x8000000000008003ull,
        0x8000000000008002ull, 0x8000000000000080ull, 0x000000000000800aull, 0x800000008000000aull,
        0x8000000080008081ull, 0x8000000000008080ull, 0x0000000080000001ull, 0x8000000080008008ull};
    for (int round = 0; round < 24; ++round) {
      // theta
      uint64_t C0 = A[0] ^ A[5] ^ A[10] ^ A[15] ^ A[20];
      uint64_t C1 = A[1] ^ A[6] ^ A[11] ^ A[16] ^ A[21];
      uint64_t C2 = A[2] ^ A[7] ^ A[12] ^ A[17] ^ A[22];
      uint64_t C3 = A[3] ^ A[8] ^ A[13] ^ A[18] ^ A[23];
      uint64_t C4 = A[4] ^ A[9] ^ A[14] ^ A[19] ^ A[24];
      uint64_t D0 = C4 ^ rol(C1, 1), D1 = C0 ^ rol(C2, 1), D2 = C1 ^ rol(C3, 1), D3 = C2 ^ rol(C4, 1),
               D4 = C3 ^ rol(C0, 1);
      // rho + pi: B[y][2x+3y] = rol(A[x][y], r[x][y])
      uint64_t B0 = A[0] ^ D0;
      uint64_t B10 = rol(A[1] ^ D1, 1);
      uint64_t B20 = rol(A[2] ^ D2, 62);
      uint64_t B5 = rol(A[3] ^ D3, 28);
      uint64_t B15 = rol(A[4] ^ D4, 27);
      uint64_t B16 = rol(A[5] ^ D0, 36);
      uint64_t B1 = rol(A[6] ^ D1, 44);
      uint64_t B11 = rol(A[7] ^ D2, 6);
      uint64_t B21 = rol(A[8] ^ D3, 55);
      uint64_t B6 = rol(A[9] ^ D4, 20);
      uint64_t B7 = rol(A[10] ^ D0, 3);
      uint64_t B17 = rol(A[11] ^ D1, 10);
      uint64_t B2 = rol(A[12] ^ D2, 43);
      uint64_t B12 = rol(A[13] ^ D3, 25);
      uint64_t B22 = rol(A[14] ^ D4, 39);
      uint64_t B23 = rol(A[15] ^ D0, 41);
      uint64_t B8 = rol(A[16] ^ D1, 45);
      uint64_t B18 = rol(A[17] ^ D2, 15);
      uint64_t B3 = rol(A[18] ^ D3, 21);
      uint64_t B13 = rol(A[19] ^ D4, 8);
      uint64_t B14 = rol(A[20] ^ D0, 18);
      uint64_t B24 = rol(A[21] ^ D1, 2);
      uint64_t B9 = rol(A[22] ^ D2, 61);
      uint64_t B19 = rol(A[23] ^ D3, 56);
      uint64_t B4 = rol(A[24] ^ D4, 14);
      // chi
      A[0] = B0 ^ (~B1 & B2);
      A[1] = B1 ^ (~B2 & B3);
      A[2] = B2 ^ (~B3 & B4);
      A[3] = B3 ^ (~B4 & B0);
      A[4] = B4 ^ (~B0 & B1);
      A[5] = B5 ^ (~B6 & B7);
      A[6] = B6 ^ (~B7 & B8);
      A[7] = B7 ^ (~B8 & B9);
      A[8] = B8 ^ (~B9 & B5);
      A[9] = B9 ^ (~B5 & B6);
      A[10] = B10 ^ (~B11 & B12);
      A[11] = B11 ^ (~B12 & B13);
      A[12] = B12 ^ (~B13 & B14);
      A[13] = B13 ^ (~B14 & B10);
      A[14] = B14 ^ (~B10 & B11);
      A[15] = B15 ^ (~B16 & B17);
      A[16] = B16 ^ (~B17 & B18);
      A[17] = B17 ^ (~B18 & B19);
      A[18] = B18 ^ (~B19 & B15);
      A[19] = B19 ^ (~B15 & B16);
      A[20] = B20 ^ (~B21 & B22);
      A[21] = B21 ^ (~B22 & B23);
      A[22] = B22 ^ (~B23 & B24);
      A[23] = B23 ^ (~B24 & B20);
      A[24] = B24 ^ (~B20 & B21);
      // iota
      A[0] ^= RC[round];
    }
  }

  void absorb_block(const uint8_t* blk) {
    for (size_t i = 0; i < RATE / 8; ++i) {
      uint64_t w;
      memcpy(&w, blk + 8 * i, 8);  // little-endian host
      st[i] ^= w;
    }
    permute(st);
  }

  void update(const uint8_t* data, size_t len) {
    if (fill) {
      size_t take = RATE - fill < len ? RATE - fill : len;
      memcpy(buf + fill, data, take);
      fill += take;
      data += take;
      len -= take;
      if (fill < RATE) return;
      absorb_block(buf);
      fill = 0;
    }
    while (len >= RATE) {
      absorb_block(data);
      data += RATE;
      len -= RATE;
    }
    memcpy(buf, data, len);
    fill = len;
  }

  // Digest::finalize_reset
  void finalize_reset(uint8_t out[32]) {
    memset(buf + fill, 0, RATE - fill);
    buf[fill] ^= 0x01;
    buf[RATE - 1] ^= 0x80;
    absorb_block(buf);
    memcpy(out, st, 32);
    reset();
  }
};

}  // namespace zk
