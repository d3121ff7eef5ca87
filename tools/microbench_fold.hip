// partial_evaluate fold (BASELINE config 2: 20-var BN254 Fr, bit 0, r fixed),
// variants timed over 10 rotated 48 MiB buffer sets (input 32 MiB + output
// 16 MiB each: past the 256 MiB MALL), 200 launches each:
//   fold     : zk::k_fold (one output per thread, fe_mul by r: CIOS)
//   foldc    : r's 10 constants built once per block in LDS, fold1c (80 + 16
//              multiply-adds, no carry chain) — the fold kernels' product
//   foldc2   : foldc with two outputs per thread, all four loads first
//   copy     : the same loads and stores, no arithmetic (the pattern's limit)
// Every variant's output is compared with `fold`'s.
// Build: hipcc -O3 -std=c++17 --offload-arch=gfx950 -o tools/mb_fold tools/microbench_fold.hip
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "../zk-research-implementations_amd/csrc/kernels.hpp"

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
constexpr int kB = 256;

__global__ __launch_bounds__(kB) void k_foldc(const Fe* __restrict__ X, Fe* __restrict__ Y, uint64_t half, Fe r) {
  __shared__ Fe ct[10];
  zk::fold_consts<F, 1>(r, r, r, ct);
  const uint64_t stride = (uint64_t)gridDim.x * kB;
  for (uint64_t v = (uint64_t)blockIdx.x * kB + threadIdx.x; v < half; v += stride)
    zk::st_fe(Y, v, zk::fold1c<F, 0>(zk::ld_fe(X, v), zk::ld_fe(X, v + half), ct));
}

__global__ __launch_bounds__(kB) void k_foldc2(const Fe* __restrict__ X, Fe* __restrict__ Y, uint64_t half, Fe r) {
  __shared__ Fe ct[10];
  zk::fold_consts<F, 1>(r, r, r, ct);
  const uint64_t stride = (uint64_t)gridDim.x * kB * 2;
  for (uint64_t v = (uint64_t)blockIdx.x * kB * 2 + threadIdx.x; v < half; v += stride) {
    const uint64_t w = v + kB;  // half is a multiple of 2 kB here
    const Fe a0 = zk::ld_fe(X, v), b0 = zk::ld_fe(X, v + half), a1 = zk::ld_fe(X, w), b1 = zk::ld_fe(X, w + half);
    zk::st_fe(Y, v, zk::fold1c<F, 0>(a0, b0, ct));
    zk::st_fe(Y, w, zk::fold1c<F, 0>(a1, b1, ct));
  }
}

__global__ __launch_bounds__(kB) void k_copy(const Fe* __restrict__ X, Fe* __restrict__ Y, uint64_t half, Fe r) {
  const uint64_t stride = (uint64_t)gridDim.x * kB;
  for (uint64_t v = (uint64_t)blockIdx.x * kB + threadIdx.x; v < half; v += stride) {
    Fe a = zk::ld_fe(X, v), b = zk::ld_fe(X, v + half);
#pragma unroll
    for (int k = 0; k < 8; ++k) a.v[k] ^= b.v[k];
    zk::st_fe(Y, v, a);
  }
}

int main(int argc, char** argv) {
  const int nv = argc > 1 ? atoi(argv[1]) : 20, reps = 200, nbuf = 10;
  const uint64_t n = 1ull << nv, half = n / 2;
  std::vector<Fe*> X(nbuf), Y(nbuf);
  for (int b = 0; b < nbuf; ++b) {
    CK(hipMalloc(&X[b], n * sizeof(Fe)));
    CK(hipMalloc(&Y[b], half * sizeof(Fe)));
    hipLaunchKernelGGL(zk::k_synth<F>, dim3(1024), dim3(kB), 0, 0, X[b], n, (uint64_t)(77 + b), (uint64_t)0, (uint64_t)1);
  }
  CK(hipDeviceSynchronize());
  Fe r;
  for (int k = 0; k < 8; ++k) r.v[k] = 0x1234567u * (k + 1);
  r.v[7] &= 0x0fffffffu;
  hipDeviceProp_t pr;
  CK(hipGetDeviceProperties(&pr, 0));
  std::vector<Fe> want(half), got(half);
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const double bytes = 96.0 * half;
  static uint32_t s_bit = 0;
  s_bit = (uint32_t)(nv - 1);  // partial_evaluate(0, r): the contiguous halves
  typedef void (*Launch)(uint64_t, const Fe*, Fe*, uint64_t, Fe);
  struct V {
    const char* name;
    const void* kern;
    Launch go;
    int per_thread;
  } vs[] = {
      {"fold", (const void*)zk::k_fold<F>,
       [](uint64_t g, const Fe* x, Fe* y, uint64_t h, Fe r) { hipLaunchKernelGGL(zk::k_fold<F>, dim3(g), dim3(kB), 0, 0, x, y, h, s_bit, r); }, 1},
      {"foldc", (const void*)k_foldc,
       [](uint64_t g, const Fe* x, Fe* y, uint64_t h, Fe r) { hipLaunchKernelGGL(k_foldc, dim3(g), dim3(kB), 0, 0, x, y, h, r); }, 1},
      {"foldc2", (const void*)k_foldc2,
       [](uint64_t g, const Fe* x, Fe* y, uint64_t h, Fe r) { hipLaunchKernelGGL(k_foldc2, dim3(g), dim3(kB), 0, 0, x, y, h, r); }, 2},
      {"copy", (const void*)k_copy,
       [](uint64_t g, const Fe* x, Fe* y, uint64_t h, Fe r) { hipLaunchKernelGGL(k_copy, dim3(g), dim3(kB), 0, 0, x, y, h, r); }, 1}};
  for (auto& v : vs) {  // parity with k_fold first
    if (v.kern == (const void*)k_copy) continue;
    const bool ref = v.kern == (const void*)zk::k_fold<F>;
    v.go((half / v.per_thread + kB - 1) / kB, X[0], Y[0], half, r);
    CK(hipDeviceSynchronize());
    CK(hipMemcpy(ref ? want.data() : got.data(), Y[0], half * sizeof(Fe), hipMemcpyDeviceToHost));
    if (!ref && memcmp(want.data(), got.data(), half * sizeof(Fe)) != 0) {
      printf("%s: output differs from k_fold\n", v.name);
      return 1;
    }
  }
  printf("all variants equal k_fold's output (%llu elements)\n", (unsigned long long)half);
  for (int rep = 0; rep < 2; ++rep)
    for (auto& v : vs)
      for (int gmode = 0; gmode < 2; ++gmode) {  // full grid / resident grid
        int per_cu = 1;
        CK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, v.kern, kB, 0));
        uint64_t g = (half / v.per_thread + kB - 1) / kB;
        if (gmode == 1) g = std::min<uint64_t>(g, (uint64_t)pr.multiProcessorCount * per_cu);
        for (int i = 0; i < 20; ++i) v.go(g, X[i % nbuf], Y[i % nbuf], half, r);
        CK(hipEventRecord(e0));
        for (int i = 0; i < reps; ++i) v.go(g, X[i % nbuf], Y[i % nbuf], half, r);
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, e0, e1));
        const double us = 1000.0 * ms / reps;
        printf("%-7s grid %6llu (%s, %d/CU)  %7.2f us  %6.0f GB/s  frac %.3f\n", v.name, (unsigned long long)g,
               gmode ? "resident" : "full", per_cu, us, bytes / us / 1e3, bytes / us / 1e3 / 8000.0);
      }
  printf("(back-to-back launches: the time includes each launch's ramp and drain)\n");
  return 0;
}
