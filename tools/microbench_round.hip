// Is the fused GKR round VALU-bound or HBM-bound? The k_gkr_round loop body
// (2 threads per pair, 8 loads, 4 folds, 2 unreduced products) run three ways
// at the round-1 size of a 24-variable proof (2^22 output pairs):
//   real    : streams 4 tables of 2^24 elements, writes 4 x 2^23 (768 B / pair)
//   compute : same arithmetic, every index masked into a 1 MiB L2-resident window
//   memory  : same loads/stores, arithmetic replaced by xor
// hipcc -O3 --offload-arch=gfx950 tools/microbench_round.hip -o tools/mb_round
#include <hip/hip_runtime.h>
#include <stdio.h>

#include "../zk-research-implementations_amd/csrc/kernels.hpp"

using namespace zk;
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

template <class F, int MODE, int WAVES = 1>  // 0 real, 1 compute-only, 2 memory-only; WAVES: min waves/SIMD
__global__ __launch_bounds__(kBlock, WAVES) void k_round(const Fe* __restrict__ A, const Fe* __restrict__ S,
                                                  const Fe* __restrict__ M, const Fe* __restrict__ P,
                                                  Fe* __restrict__ A2, Fe* __restrict__ S2, Fe* __restrict__ M2,
                                                  Fe* __restrict__ P2, uint64_t h, Fe r, Fe* out) {
  Wide w0 = wide_zero<F>(), w2 = wide_zero<F>();
  const uint64_t g = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
  const uint32_t q = (uint32_t)(g >> 6) & 1u;
  uint64_t j = ((g >> 7) << 6) | (g & 63);
  const uint64_t step = (uint64_t)gridDim.x * (kBlock / 2);
  const Fe* __restrict__ X = q ? M : A;
  const Fe* __restrict__ Z = q ? P : S;
  Fe* __restrict__ X2 = q ? M2 : A2;
  Fe* __restrict__ Z2 = q ? P2 : S2;
  const uint64_t mask = MODE == 1 ? (1u << 13) - 1 : ~0ull;  // 8192 elements = 256 KiB per stream
  Fe acc = fe_zero<F>();
  for (; j < h; j += step) {
    const uint64_t jj = j & mask, hh = MODE == 1 ? (1u << 13) : h;
    const Fe x0 = ld_fe(X, jj), x1 = ld_fe(X, jj + hh), x2 = ld_fe(X, jj + 2 * hh), x3 = ld_fe(X, jj + 3 * hh);
    const Fe z0 = ld_fe(Z, jj), z1 = ld_fe(Z, jj + hh), z2 = ld_fe(Z, jj + 2 * hh), z3 = ld_fe(Z, jj + 3 * hh);
    __builtin_amdgcn_sched_barrier(0);
    if (MODE == 2) {
      Fe a, b;
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        a.v[i] = x0.v[i] ^ x2.v[i] ^ z0.v[i];
        b.v[i] = x1.v[i] ^ x3.v[i] ^ z3.v[i] ^ z1.v[i] ^ z2.v[i];
      }
      st_fe(X2, jj, a);
      st_fe(X2, jj + hh, b);
      st_fe(Z2, jj, b);
      st_fe(Z2, jj + hh, a);
    } else {
      const Fe a0 = fold1<F>(x0, x2, r), a1 = fold1<F>(x1, x3, r);
      const Fe s0 = fold1<F>(z0, z2, r), s1 = fold1<F>(z1, z3, r);
      st_fe(X2, jj, a0);
      st_fe(X2, jj + hh, a1);
      st_fe(Z2, jj, s0);
      st_fe(Z2, jj + hh, s1);
      wide_mac<F>(w0, a0, s0);
      wide_mac<F>(w2, at2<F>(a0, a1), at2<F>(s0, s1));
    }
  }
  acc = fe_add<F>(wide_redc<F>(w0), wide_redc<F>(w2));
  if (acc.v[0] == 0x12345u) out[0] = acc;  // keep the work alive
}

// round 0 body (k_gkr_round0: 2 threads per pair, 4 loads, 3 unreduced products)
#ifndef R0_WAVES
#define R0_WAVES 1
#endif
template <class F, int MODE>  // 0 real, 1 compute-only, 2 memory-only
__global__ __launch_bounds__(kBlock, R0_WAVES) void k_round0(const Fe* __restrict__ A, const Fe* __restrict__ S,
                                                   const Fe* __restrict__ M, const Fe* __restrict__ P, uint64_t h,
                                                   Fe* out) {
  Wide w0 = wide_zero<F>(), w1 = wide_zero<F>(), w2 = wide_zero<F>();
  uint64_t j, step;
  uint32_t q;
  pair_slot(j, q, step);
  const Fe* __restrict__ X = q ? M : A;
  const Fe* __restrict__ Z = q ? P : S;
  const uint64_t mask = MODE == 1 ? (1u << 13) - 1 : ~0ull;
  uint32_t x = 0;
  for (; j < h; j += step) {
    const uint64_t jj = j & mask, hh = MODE == 1 ? (1u << 13) : h;
    const Fe x0 = ld_fe(X, jj), x1 = ld_fe(X, jj + hh), z0 = ld_fe(Z, jj), z1 = ld_fe(Z, jj + hh);
    __builtin_amdgcn_sched_barrier(0);
    if (MODE == 2) {
#pragma unroll
      for (int i = 0; i < 8; ++i) x ^= x0.v[i] ^ x1.v[i] ^ z0.v[i] ^ z1.v[i];
    } else {
      wide_mac<F>(w0, x0, z0);
      wide_mac<F>(w1, x1, z1);
      wide_mac<F>(w2, at2<F>(x0, x1), at2<F>(z0, z1));
    }
  }
  for (int i = 0; i < 17; ++i) x ^= w0.w[i] ^ w1.w[i] ^ w2.w[i];
  if (x == 0x12345u) out[0].v[0] = x;  // keep the work alive
}

int main() {
  using F = Bn254Fr;
  const uint64_t N = 1ull << 24, h = N / 4;  // round 1 of a 24-var proof
  Fe *A, *S, *M, *P, *W, *out;
  CK(hipMalloc(&A, N * 32)); CK(hipMalloc(&S, N * 32)); CK(hipMalloc(&M, N * 32)); CK(hipMalloc(&P, N * 32));
  CK(hipMalloc(&W, 4 * (N / 2) * 32)); CK(hipMalloc(&out, 64));
  for (Fe* t : {A, S, M, P}) CK(hipMemset(t, 0x11, N * 32));
  Fe r;
  for (int i = 0; i < 8; ++i) r.v[i] = 0x01020304u * (i + 1) & 0x0fffffff;
  RoundIn rin{};
  rin.r = r;
  int per_cu = 0;
  CK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k_round<F, 0>, kBlock, 0));
  hipDeviceProp_t prop;
  CK(hipGetDeviceProperties(&prop, 0));
  const int grid = prop.multiProcessorCount * per_cu;
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  auto run = [&](const char* name, auto kern) {
    kern<<<grid, kBlock>>>(A, S, M, P, W, W + N / 2, W + N, W + 3 * N / 2, h, r, out);
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(e0));
    for (int i = 0; i < 5; ++i) kern<<<grid, kBlock>>>(A, S, M, P, W, W + N / 2, W + N, W + 3 * N / 2, h, r, out);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    const double us = ms * 1e3 / 5, bytes = 768.0 * h;
    printf("%-8s %8.1f us   %7.1f GB/s equivalent (grid %d = %d/CU)\n", name, us, bytes / (us * 1e-6) / 1e9, grid, per_cu);
    return 0;
  };
  {
    int pc0 = 0;
    CK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&pc0, k_round0<F, 0>, kBlock, 0));
    const int g0 = prop.multiProcessorCount * pc0;
    const uint64_t h0 = N / 2;  // round 0 of a 24-var proof: 2^23 pairs over 4 tables of 2^24
    auto run0 = [&](const char* name, auto kern) {
      kern<<<g0, kBlock>>>(A, S, M, P, h0, out);
      CK(hipDeviceSynchronize());
      CK(hipEventRecord(e0));
      for (int i = 0; i < 5; ++i) kern<<<g0, kBlock>>>(A, S, M, P, h0, out);
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      const double us = ms * 1e3 / 5, bytes = 256.0 * h0;
      printf("round0 %-8s %8.1f us   %7.1f GB/s equivalent (grid %d = %d/CU)\n", name, us, bytes / (us * 1e-6) / 1e9, g0, pc0);
      return 0;
    };
    run0("real", k_round0<F, 0>);
    run0("compute", k_round0<F, 1>);
    run0("memory", k_round0<F, 2>);
  }
  run("real", k_round<F, 0>);
  run("compute", k_round<F, 1>);
  run("memory", k_round<F, 2>);
  // occupancy sweep: the grid follows each variant's own occupancy
  auto runw = [&](const char* name, auto kern) {
    int pcu = 0;
    CK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&pcu, kern, kBlock, 0));
    const int gw = prop.multiProcessorCount * pcu;
    kern<<<gw, kBlock>>>(A, S, M, P, W, W + N / 2, W + N, W + 3 * N / 2, h, r, out);
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(e0));
    for (int i = 0; i < 5; ++i) kern<<<gw, kBlock>>>(A, S, M, P, W, W + N / 2, W + N, W + 3 * N / 2, h, r, out);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    const double us = ms * 1e3 / 5;
    printf("%-12s %8.1f us   %7.1f GB/s (grid %d = %d/CU)\n", name, us, 768.0 * h / (us * 1e-6) / 1e9, gw, pcu);
    return 0;
  };
  runw("real w2", k_round<F, 0, 2>);
  runw("real w3", k_round<F, 0, 3>);
  runw("real w4", k_round<F, 0, 4>);
  runw("memory w2", k_round<F, 2, 2>);
  runw("memory w3", k_round<F, 2, 3>);
  runw("memory w4", k_round<F, 2, 4>);
  runw("memory w6", k_round<F, 2, 6>);
  runw("memory w8", k_round<F, 2, 8>);

  // the production kernels across round sizes, with the full epilogue
  // (two-level fan-in + publish to pinned host memory); back-to-back launches
  uint64_t* parts;
  uint32_t* ctr;
  uint64_t* hout;
  CK(hipMalloc(&parts, (256 * 8 + 8) * kSlotU64 * 8));
  CK(hipMalloc(&ctr, 4096));
  CK(hipMemset(ctr, 0, 4096));
  CK(hipHostMalloc(&hout, 4096, hipHostMallocMapped | hipHostMallocCoherent));
  RoundSink sk{parts, ctr, reinterpret_cast<uint64_t*>(ctr + 640), nullptr, hout, reinterpret_cast<uint32_t*>(hout + 64), 1};
  int pc[2] = {0, 0};
  CK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&pc[0], k_gkr_round<F>, kBlock, 0));
  CK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&pc[1], k_gkr_round_lanes<F>, kBlock, 0));
  printf("size sweep (blocks/CU: round %d, lanes %d)\n", pc[0], pc[1]);
  const char* names[2] = {"round", "lanes"};
  for (int lg = 22; lg >= 0; lg -= 1) {
    const uint64_t hh = 1ull << lg;
    for (int v = 0; v < 2; ++v) {
      if (v == 1 && lg > 17) continue;
      const int lanes = v == 1;
      const uint64_t work = (lanes ? 8 : 2) * hh;
      uint64_t g = (work + kBlock - 1) / kBlock;
      const uint64_t cap = (uint64_t)prop.multiProcessorCount * pc[lanes];
      if (g > cap) g = cap;
      auto launch = [&] {
        if (v == 1)
          k_gkr_round_lanes<F><<<(uint32_t)g, kBlock>>>(A, S, M, P, W, W + N / 2, W + N, W + 3 * N / 2, hh, rin, sk);
        else
          k_gkr_round<F><<<(uint32_t)g, kBlock>>>(A, S, M, P, W, W + N / 2, W + N, W + 3 * N / 2, hh, rin, sk);
      };
      launch();
      CK(hipDeviceSynchronize());
      const int reps = lg > 18 ? 5 : 50;
      CK(hipEventRecord(e0));
      for (int i = 0; i < reps; ++i) launch();
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      const double us = ms * 1e3 / reps;
      printf("  pairs 2^%-2d %-6s grid %6llu  %9.2f us  %8.1f GB/s\n", lg, names[v],
             (unsigned long long)g, us, 768.0 * hh / (us * 1e-6) / 1e9);
    }
  }
  return 0;
}
