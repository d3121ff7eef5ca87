// Latency of one dependent 256-bit Montgomery product on ONE wave (round 5,
// the device Fiat-Shamir step of k_gkr_dtail<F, true> is a
// one-wave dependent chain of ~13 such products plus two Keccak-f):
//   single : zk::fe_mul on one lane (8 x 32-bit limbs, CIOS, 136 v_mad_u64_u32)
//   lanes  : the same product spread over 9 lanes (lane j holds limb j of a,
//            b, p and a redundant 64-bit accumulator limb): per CIOS row one
//            readlane of b_i, one v_mad_u64_u32 per lane, a DPP row_shr:1 to
//            move the high halves one limb up, a readlane of the low limb for
//            m, a second v_mad_u64_u32, a DPP row_shl:1 to divide by 2^32;
//            then carry resolution and the conditional subtraction of p
//            across lanes (ballot-driven, usually 2-3 steps)
// Both chains run K dependent products from the same inputs; the lane product
// is checked bit for bit against fe_mul before timing. Reports ns and shader
// cycles (s_memtime) per product.
// Build: hipcc -O3 --offload-arch=gfx950 -o tools/mb_lanemul tools/microbench_lanemul.hip
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <random>

#include "../zk-research-implementations_amd/csrc/field.hpp"

#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e_ = (x);                                                        \
    if (e_ != hipSuccess) {                                                     \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                  \
    }                                                                           \
  } while (0)

using F = zk::Bn254Fr;
using zk::Fe;

// lane j <- lane j-1 (lane 0 of each 16-lane row <- 0)
__device__ __forceinline__ uint32_t shr1(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xf, 0xf, true);
}
// lane j <- lane j+1 (lane 15 of each row <- 0)
__device__ __forceinline__ uint32_t shl1(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x101, 0xf, 0xf, true);
}

// a, b: limb j in lane j (j < 8), 0 in lanes >= 8; pj likewise. Returns a*b*2^-256 mod p, limb j in lane j.
__device__ __forceinline__ uint32_t lane_mul(uint32_t a, uint32_t b, uint32_t pj) {
  const uint32_t lane = __lane_id();
  uint64_t acc = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const uint32_t bi = __builtin_amdgcn_readlane(b, i);
    acc = (uint64_t)a * bi + acc;  // acc < 2^33 before: no overflow
    acc = (uint64_t)(uint32_t)acc + shr1((uint32_t)(acc >> 32));
    const uint32_t m = __builtin_amdgcn_readlane((uint32_t)acc, 0) * F::PINV;
    acc = (uint64_t)m * pj + acc;  // limb 0 now divisible by 2^32
    acc = (uint64_t)shl1((uint32_t)acc) + (uint32_t)(acc >> 32);  // / 2^32: new_j = lo_{j+1} + hi_j
  }
  // resolve the redundant carries (value < 2p < 2^256: nothing leaves lane 7)
  uint32_t t = (uint32_t)acc, c = (uint32_t)(acc >> 32);
  while (__builtin_amdgcn_ballot_w64(c != 0) & 0x1ffull) {
    const uint64_t s = (uint64_t)t + shr1(c);
    t = (uint32_t)s;
    c = (uint32_t)(s >> 32);
  }
  // t >= p ? (the highest limb where t and p differ decides)
  const uint64_t ne = __builtin_amdgcn_ballot_w64(lane < 8 && t != pj) & 0xffull;
  bool ge = ne == 0;
  if (ne) {
    const int k = 63 - __builtin_clzll(ne);
    ge = __builtin_amdgcn_readlane(t, k) > __builtin_amdgcn_readlane(pj, k);
  }
  if (ge) {  // t - p with borrows resolved the same way
    int64_t d = (int64_t)t - (int64_t)pj;
    uint32_t r = (uint32_t)d;
    int32_t br = (int32_t)(d >> 32);  // 0 or -1
    while (__builtin_amdgcn_ballot_w64(br != 0) & 0xffull) {
      const int64_t s = (int64_t)r + (int32_t)shr1((uint32_t)br);
      r = (uint32_t)s;
      br = (int32_t)(s >> 32);
    }
    t = r;
  }
  return lane < 8 ? t : 0u;
}

__global__ void k_check(const Fe* a, const Fe* b, Fe* single, Fe* lanes, int n) {
  const uint32_t lane = __lane_id();
  for (int i = 0; i < n; ++i) {
    if (lane == 0) single[i] = zk::fe_mul<F>(a[i], b[i]);
    const uint32_t aj = lane < 8 ? a[i].v[lane] : 0u, bj = lane < 8 ? b[i].v[lane] : 0u;
    const uint32_t pj = lane < 8 ? F::P[lane] : 0u;
    const uint32_t r = lane_mul(aj, bj, pj);
    if (lane < 8) lanes[i].v[lane] = r;
  }
}

// K dependent products x <- x * y on one wave; times[0..1]: realtime (10 ns ticks), [2..3]: shader clock
__global__ void k_chain_single(const Fe* in, Fe* out, int K, uint64_t* times) {
  if (__lane_id() != 0) return;
  Fe x = in[0], y = in[1];
  const uint64_t r0 = __builtin_amdgcn_s_memrealtime(), c0 = __builtin_amdgcn_s_memtime();
  for (int k = 0; k < K; ++k) x = zk::fe_mul<F>(x, y);
  asm volatile("" ::"v"(x.v[0]), "v"(x.v[7]));
  const uint64_t c1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
  out[0] = x;
  times[0] = r0;
  times[1] = r1;
  times[2] = c0;
  times[3] = c1;
}
__global__ void k_chain_lanes(const Fe* in, Fe* out, int K, uint64_t* times) {
  const uint32_t lane = __lane_id();
  uint32_t x = lane < 8 ? in[0].v[lane] : 0u, y = lane < 8 ? in[1].v[lane] : 0u;
  const uint32_t pj = lane < 8 ? F::P[lane] : 0u;
  const uint64_t r0 = __builtin_amdgcn_s_memrealtime(), c0 = __builtin_amdgcn_s_memtime();
  for (int k = 0; k < K; ++k) x = lane_mul(x, y, pj);
  asm volatile("" ::"v"(x));
  const uint64_t c1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
  if (lane < 8) out[0].v[lane] = x;
  if (lane == 0) {
    times[0] = r0;
    times[1] = r1;
    times[2] = c0;
    times[3] = c1;
  }
}

static Fe rand_fe(std::mt19937_64& g) {
  Fe x;
  for (int i = 0; i < 8; ++i) x.v[i] = (uint32_t)g();
  x.v[7] &= 0x1fffffffu;  // < 2^253 < p
  return x;
}

int main() {
  const int n = 4096;
  std::mt19937_64 g(42);
  Fe *a, *b, *s, *l, *io, *o1, *o2;
  uint64_t* t;
  CK(hipMallocManaged(&a, n * sizeof(Fe)));
  CK(hipMallocManaged(&b, n * sizeof(Fe)));
  CK(hipMallocManaged(&s, n * sizeof(Fe)));
  CK(hipMallocManaged(&l, n * sizeof(Fe)));
  CK(hipMallocManaged(&io, 2 * sizeof(Fe)));
  CK(hipMallocManaged(&o1, sizeof(Fe)));
  CK(hipMallocManaged(&o2, sizeof(Fe)));
  CK(hipMallocManaged(&t, 8 * sizeof(uint64_t)));
  for (int i = 0; i < n; ++i) {
    a[i] = rand_fe(g);
    b[i] = rand_fe(g);
  }
  // edge operands: 0, 1, p - 1 (largest canonical)
  for (int k = 0; k < 8; ++k) {
    a[0].v[k] = 0;
    a[1].v[k] = F::P[k];
    b[2].v[k] = F::P[k];
  }
  a[1].v[0] -= 1;
  b[2].v[0] -= 1;
  a[3] = b[3];
  hipLaunchKernelGGL(k_check, dim3(1), dim3(64), 0, 0, a, b, s, l, n);
  CK(hipDeviceSynchronize());
  int bad = 0;
  for (int i = 0; i < n; ++i)
    for (int k = 0; k < 8; ++k) bad += s[i].v[k] != l[i].v[k];
  printf("lane-parallel product vs fe_mul: %d of %d products differ\n", bad ? bad : 0, n);
  if (bad) return 1;
  io[0] = a[5];
  io[1] = b[5];
  for (int K : {1000, 4000}) {
    hipLaunchKernelGGL(k_chain_single, dim3(1), dim3(64), 0, 0, io, o1, K, t);
    CK(hipDeviceSynchronize());
    const double ns1 = (t[1] - t[0]) * 10.0 / K, cyc1 = (double)(t[3] - t[2]) / K;
    hipLaunchKernelGGL(k_chain_lanes, dim3(1), dim3(64), 0, 0, io, o2, K, t + 4);
    CK(hipDeviceSynchronize());
    const double ns2 = (t[5] - t[4]) * 10.0 / K, cyc2 = (double)(t[7] - t[6]) / K;
    int same = 1;
    for (int k = 0; k < 8; ++k) same &= o1->v[k] == o2->v[k];
    printf("K %5d dependent products on one wave: single lane %.1f ns (%.0f clk) | 9 lanes %.1f ns (%.0f clk) | same result %d\n",
           K, ns1, cyc1, ns2, cyc2, same);
  }
  return 0;
}
