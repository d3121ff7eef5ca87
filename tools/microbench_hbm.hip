// HBM access-shape microbenchmark: what per-lane shape streams 32-byte field
// elements fastest on gfx950? hipcc -O3 --offload-arch=gfx950 tools/microbench_hbm.hip -o tools/mb_hbm
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

// 1) lane-contiguous 16 B per lane, grid-stride
__global__ void copy16(const uint4* __restrict__ in, uint4* __restrict__ out, size_t n) {
  size_t stride = (size_t)gridDim.x * blockDim.x;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += stride) out[i] = in[i];
}
// 2) 4 independent 16-B loads in flight per lane
__global__ void copy16x4(const uint4* __restrict__ in, uint4* __restrict__ out, size_t n) {
  size_t stride = (size_t)gridDim.x * blockDim.x;
  size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  for (; i + 3 * stride < n; i += 4 * stride) {
    uint4 a = in[i], b = in[i + stride], c = in[i + 2 * stride], d = in[i + 3 * stride];
    out[i] = a; out[i + stride] = b; out[i + 2 * stride] = c; out[i + 3 * stride] = d;
  }
  for (; i < n; i += stride) out[i] = in[i];
}
// 3) AoS 32-byte element per lane (two dwordx4 at a 32-B lane stride)
__global__ void copy32aos(const uint4* __restrict__ in, uint4* __restrict__ out, size_t nelem) {
  size_t stride = (size_t)gridDim.x * blockDim.x;
  for (size_t e = blockIdx.x * (size_t)blockDim.x + threadIdx.x; e < nelem; e += stride) {
    uint4 a = in[2 * e], b = in[2 * e + 1];
    out[2 * e] = a; out[2 * e + 1] = b;
  }
}
// 4) AoS 32-B elements, 4 elements in flight per lane
__global__ void copy32aos_x4(const uint4* __restrict__ in, uint4* __restrict__ out, size_t nelem) {
  size_t stride = (size_t)gridDim.x * blockDim.x;
  size_t e = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  for (; e + 3 * stride < nelem; e += 4 * stride) {
    uint4 v[8];
#pragma unroll
    for (int k = 0; k < 4; ++k) { v[2 * k] = in[2 * (e + k * stride)]; v[2 * k + 1] = in[2 * (e + k * stride) + 1]; }
#pragma unroll
    for (int k = 0; k < 4; ++k) { out[2 * (e + k * stride)] = v[2 * k]; out[2 * (e + k * stride) + 1] = v[2 * k + 1]; }
  }
  for (; e < nelem; e += stride) { out[2 * e] = in[2 * e]; out[2 * e + 1] = in[2 * e + 1]; }
}
// 5) read-only AoS 32-B (xor-reduce), 4 in flight
__global__ void read32aos_x4(const uint4* __restrict__ in, uint4* __restrict__ out, size_t nelem) {
  size_t stride = (size_t)gridDim.x * blockDim.x;
  size_t e = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  uint4 acc = make_uint4(0, 0, 0, 0);
  for (; e + 3 * stride < nelem; e += 4 * stride) {
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      uint4 a = in[2 * (e + k * stride)], b = in[2 * (e + k * stride) + 1];
      acc.x ^= a.x ^ b.x; acc.y ^= a.y ^ b.y; acc.z ^= a.z ^ b.z; acc.w ^= a.w ^ b.w;
    }
  }
  if (acc.x == 0x12345678u) out[0] = acc;
}
// 6) read-only lane-contiguous 16 B, 4 in flight
__global__ void read16_x4(const uint4* __restrict__ in, uint4* __restrict__ out, size_t n) {
  size_t stride = (size_t)gridDim.x * blockDim.x;
  size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  uint4 acc = make_uint4(0, 0, 0, 0);
  for (; i + 3 * stride < n; i += 4 * stride) {
#pragma unroll
    for (int k = 0; k < 4; ++k) { uint4 a = in[i + k * stride]; acc.x ^= a.x; acc.y ^= a.y; acc.z ^= a.z; acc.w ^= a.w; }
  }
  if (acc.x == 0x12345678u) out[0] = acc;
}
// 7) the fused-round access pattern without arithmetic: 2 tables x 4 quarter
// streams read, 2 x 2 half streams written, 32-B AoS elements
__global__ void fused_pattern(const uint4* __restrict__ X, const uint4* __restrict__ Z, uint4* __restrict__ X2,
                              uint4* __restrict__ Z2, size_t h) {
  size_t stride = (size_t)gridDim.x * blockDim.x;
  for (size_t j = blockIdx.x * (size_t)blockDim.x + threadIdx.x; j < h; j += stride) {
    uint4 x[8], z[8];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      x[2 * k] = X[2 * (j + k * h)]; x[2 * k + 1] = X[2 * (j + k * h) + 1];
      z[2 * k] = Z[2 * (j + k * h)]; z[2 * k + 1] = Z[2 * (j + k * h) + 1];
    }
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      uint4 a = x[2 * k], b = x[2 * k + 1], c = x[2 * k + 4], d = x[2 * k + 5];
      X2[2 * (j + k * h)] = make_uint4(a.x ^ c.x, a.y ^ c.y, a.z ^ c.z, a.w ^ c.w);
      X2[2 * (j + k * h) + 1] = make_uint4(b.x ^ d.x, b.y ^ d.y, b.z ^ d.z, b.w ^ d.w);
      a = z[2 * k]; b = z[2 * k + 1]; c = z[2 * k + 4]; d = z[2 * k + 5];
      Z2[2 * (j + k * h)] = make_uint4(a.x ^ c.x, a.y ^ c.y, a.z ^ c.z, a.w ^ c.w);
      Z2[2 * (j + k * h) + 1] = make_uint4(b.x ^ d.x, b.y ^ d.y, b.z ^ d.z, b.w ^ d.w);
    }
  }
}

int main() {
  const size_t bytes = 2ull << 30;  // 2 GiB per buffer (>> 256 MiB Infinity Cache)
  uint4 *a, *b, *c, *d;
  CK(hipMalloc(&a, bytes));
  CK(hipMalloc(&b, bytes));
  CK(hipMalloc(&c, bytes));
  CK(hipMalloc(&d, bytes));
  CK(hipMemset(a, 1, bytes));
  CK(hipMemset(b, 2, bytes));
  const size_t n16 = bytes / 16, n32 = bytes / 32;
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  int grids[] = {1024, 2048, 4096, 8192};
  auto run = [&](const char* name, double moved, auto launch) {
    for (int g : grids) {
      launch(g);
      CK(hipDeviceSynchronize());
      CK(hipEventRecord(e0));
      for (int r = 0; r < 5; ++r) launch(g);
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      printf("%-16s grid %5d: %8.1f GB/s\n", name, g, moved / (ms / 5 / 1e3) / 1e9);
    }
    return 0;
  };
  run("copy16", 2.0 * bytes, [&](int g) { copy16<<<g, 256>>>(a, b, n16); });
  run("copy16x4", 2.0 * bytes, [&](int g) { copy16x4<<<g, 256>>>(a, b, n16); });
  run("copy32aos", 2.0 * bytes, [&](int g) { copy32aos<<<g, 256>>>(a, b, n32); });
  run("copy32aos_x4", 2.0 * bytes, [&](int g) { copy32aos_x4<<<g, 256>>>(a, b, n32); });
  run("read32aos_x4", 1.0 * bytes, [&](int g) { read32aos_x4<<<g, 256>>>(a, b, n32); });
  run("read16_x4", 1.0 * bytes, [&](int g) { read16_x4<<<g, 256>>>(a, b, n16); });
  // fused pattern: 2 tables of 2 GiB read (4h elements each), 2 outputs of 1 GiB
  const size_t h = n32 / 4;
  run("fused_pattern", 2.0 * bytes + 1.0 * bytes, [&](int g) { fused_pattern<<<g, 256>>>(a, b, c, d, h); });
  return 0;
}
