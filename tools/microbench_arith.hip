// Microbenchmark: VALU throughput of the integer/FP64 primitives a 256-bit
// Montgomery multiply can be built from on gfx950, plus the field multiply
// itself and a streaming-copy HBM calibration. Standalone: hipcc -O3
// --offload-arch=gfx950 tools/microbench_arith.hip -o /tmp/mb && /tmp/mb
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
#include "../zk-research-implementations_amd/csrc/field.hpp"

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

constexpr int ITER = 2048;

__global__ void k_mad64(uint64_t* out, uint32_t s) {
  uint64_t a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
  uint32_t x = s + threadIdx.x, y = s ^ blockIdx.x;
  for (int i = 0; i < ITER; ++i) {
    a0 = (uint64_t)x * y + a0; a1 = (uint64_t)y * x + a1; a2 = (uint64_t)(x + 1) * y + a2; a3 = (uint64_t)(x + 2) * y + a3;
    a4 = (uint64_t)(x + 3) * y + a4; a5 = (uint64_t)(x + 4) * y + a5; a6 = (uint64_t)(x + 5) * y + a6; a7 = (uint64_t)(x + 6) * y + a7;
    x ^= (uint32_t)a0;
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}

__global__ void k_mullo(uint32_t* out, uint32_t s) {
  uint32_t a[8];
  for (int k = 0; k < 8; ++k) a[k] = threadIdx.x + k;
  uint32_t y = s ^ blockIdx.x;
  for (int i = 0; i < ITER; ++i) {
#pragma unroll
    for (int k = 0; k < 8; ++k) a[k] = a[k] * y + 0;
    y += 2;
  }
  uint32_t r = 0;
  for (int k = 0; k < 8; ++k) r ^= a[k];
  out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}

__global__ void k_mulhi(uint32_t* out, uint32_t s) {
  uint32_t a[8];
  for (int k = 0; k < 8; ++k) a[k] = threadIdx.x + k + 7;
  uint32_t y = s ^ blockIdx.x;
  for (int i = 0; i < ITER; ++i) {
#pragma unroll
    for (int k = 0; k < 8; ++k) a[k] = __umulhi(a[k], y) ^ k;
    y += 3;
  }
  uint32_t r = 0;
  for (int k = 0; k < 8; ++k) r ^= a[k];
  out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}

__global__ void k_addc(uint32_t* out, uint32_t s) {
  uint32_t a[8], b[8];
  for (int k = 0; k < 8; ++k) { a[k] = threadIdx.x + k; b[k] = s + k; }
  for (int i = 0; i < ITER; ++i) {
    uint32_t c = 0;
#pragma unroll
    for (int k = 0; k < 8; ++k) a[k] = zk::addc32(a[k], b[k], c, &c);
    b[0] ^= c;
  }
  uint32_t r = 0;
  for (int k = 0; k < 8; ++k) r ^= a[k];
  out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}

__global__ void k_fma64(double* out, double s) {
  double a[8];
  for (int k = 0; k < 8; ++k) a[k] = threadIdx.x + k;
  double y = s;
  for (int i = 0; i < ITER; ++i) {
#pragma unroll
    for (int k = 0; k < 8; ++k) a[k] = __fma_rn(a[k], y, 1.0);
  }
  double r = 0;
  for (int k = 0; k < 8; ++k) r += a[k];
  out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}

template <int CHAINS>
__global__ void k_modmul(zk::Fe* out, uint32_t s) {
  using F = zk::Bn254Fr;
  zk::Fe x[CHAINS], y;
  for (int c = 0; c < CHAINS; ++c)
    for (int i = 0; i < 8; ++i) x[c].v[i] = (threadIdx.x * 977u + i * 131u + c) & 0x0fffffffu;
  for (int i = 0; i < 8; ++i) y.v[i] = (s + i * 7919u) & 0x0fffffffu;
  for (int it = 0; it < ITER / 16; ++it) {
#pragma unroll
    for (int c = 0; c < CHAINS; ++c) x[c] = zk::fe_mul<F>(x[c], y);
  }
  zk::Fe r = x[0];
  for (int c = 1; c < CHAINS; ++c) r = zk::fe_add<F>(r, x[c]);
  out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}

__global__ void k_copy(const uint4* __restrict__ in, uint4* __restrict__ out, size_t n) {
  size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  size_t stride = (size_t)gridDim.x * blockDim.x;
  for (; i < n; i += stride) out[i] = in[i];
}

int main() {
  const int blocks = 256 * 8, threads = 256;
  const size_t nthreads = (size_t)blocks * threads;
  void* buf;
  CK(hipMalloc(&buf, nthreads * 64));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  float ms;
  auto rate = [&](const char* name, double ops_per_thread, auto launch) {
    launch();  // warm
    (void)hipDeviceSynchronize();
    (void)hipEventRecord(e0);
    for (int r = 0; r < 5; ++r) launch();
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    (void)hipEventElapsedTime(&ms, e0, e1);
    double sec = ms / 1e3 / 5;
    double ops = ops_per_thread * nthreads;
    // wave-instructions per cycle per CU at 2.4 GHz
    double wi_per_cu_cycle = ops / 64.0 / 256.0 / (sec * 2.4e9);
    printf("%-14s %9.3f ms  %10.1f Gop/s  %.3f wave-instr/CU/cycle (%.2f cyc per wave-instr per SIMD)\n", name, sec * 1e3,
           ops / sec / 1e9, wi_per_cu_cycle, 4.0 / wi_per_cu_cycle);
  };
  rate("mad_u64_u32", 8.0 * ITER, [&] { k_mad64<<<blocks, threads>>>((uint64_t*)buf, 3); });
  rate("mul_lo_u32", 8.0 * ITER, [&] { k_mullo<<<blocks, threads>>>((uint32_t*)buf, 3); });
  rate("mul_hi_u32", 8.0 * ITER, [&] { k_mulhi<<<blocks, threads>>>((uint32_t*)buf, 3); });
  rate("addc_u32", 8.0 * ITER, [&] { k_addc<<<blocks, threads>>>((uint32_t*)buf, 3); });
  rate("fma_f64", 8.0 * ITER, [&] { k_fma64<<<blocks, threads>>>((double*)buf, 1.0000001); });
  rate("modmul x1", 1.0 * ITER / 16, [&] { k_modmul<1><<<blocks, threads>>>((zk::Fe*)buf, 3); });
  rate("modmul x2", 2.0 * ITER / 16, [&] { k_modmul<2><<<blocks, threads>>>((zk::Fe*)buf, 3); });
  rate("modmul x4", 4.0 * ITER / 16, [&] { k_modmul<4><<<blocks, threads>>>((zk::Fe*)buf, 3); });

  // HBM calibration: 1 GiB copy
  size_t n = (1ull << 30) / 16;
  uint4 *a, *b;
  CK(hipMalloc(&a, n * 16));
  CK(hipMalloc(&b, n * 16));
  (void)hipMemset(a, 1, n * 16);
  k_copy<<<256 * 8, 256>>>(a, b, n);
  (void)hipDeviceSynchronize();
  (void)hipEventRecord(e0);
  for (int r = 0; r < 5; ++r) k_copy<<<256 * 8, 256>>>(a, b, n);
  (void)hipEventRecord(e1);
  (void)hipEventSynchronize(e1);
  (void)hipEventElapsedTime(&ms, e0, e1);
  printf("copy 1GiB: %.3f ms  %.1f GB/s (r+w)\n", ms / 5, 2.0 * n * 16 / (ms / 5 / 1e3) / 1e9);
  return 0;
}
