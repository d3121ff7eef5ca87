// Does the address pattern of a fused GKR round limit its memory side?
// Same bytes as round 1 of a 24-variable proof (read 4 x 2^24 elements,
// write 4 x 2^23; 768 B per output pair), no arithmetic (xor), three layouts:
//   quarters : the production pattern — per table 4 loads at j + q h (h = 2^22
//              elements = 128 MiB apart), 2 stores at j, j + h
//   skewed   : the same streams, each quarter shifted by q * SKEW elements
//              (breaks the power-of-two alignment; not a valid fold, a probe)
//   pairwise : the bit-reversed layout's pattern — per table 4 contiguous loads
//              at 4i..4i+3, 2 contiguous stores at 2i, 2i+1
// and a plain copy of the same byte count as the control.
// hipcc -O3 --offload-arch=gfx950 tools/microbench_mix.hip -o tools/mb_mix
#include <hip/hip_runtime.h>
#include <stdio.h>

#include "../zk-research-implementations_amd/csrc/kernels.hpp"

using namespace zk;
#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)

constexpr uint64_t kSkew = 4096 + 64;  // elements

__device__ __forceinline__ Fe xr(const Fe& a, const Fe& b) {
  Fe c;
#pragma unroll
  for (int i = 0; i < 8; ++i) c.v[i] = a.v[i] ^ b.v[i];
  return c;
}

template <int MODE>  // 0 quarters, 1 skewed, 2 pairwise
__global__ __launch_bounds__(kBlock) void k_mix(const Fe* __restrict__ A, const Fe* __restrict__ S,
                                               const Fe* __restrict__ M, const Fe* __restrict__ P,
                                               Fe* __restrict__ A2, Fe* __restrict__ S2, Fe* __restrict__ M2,
                                               Fe* __restrict__ P2, uint64_t h) {
  const uint64_t g = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
  const uint32_t q = (uint32_t)(g >> 6) & 1u;
  uint64_t j = ((g >> 7) << 6) | (g & 63);
  const uint64_t step = (uint64_t)gridDim.x * (kBlock / 2);
  const Fe* __restrict__ X = q ? M : A;
  const Fe* __restrict__ Z = q ? P : S;
  Fe* __restrict__ X2 = q ? M2 : A2;
  Fe* __restrict__ Z2 = q ? P2 : S2;
  for (; j < h; j += step) {
    uint64_t i0, i1, i2, i3, o0, o1;
    if (MODE == 2) {
      i0 = 4 * j; i1 = i0 + 1; i2 = i0 + 2; i3 = i0 + 3; o0 = 2 * j; o1 = o0 + 1;
    } else {
      const uint64_t sk = MODE == 1 ? kSkew : 0;
      i0 = j; i1 = j + h + sk; i2 = j + 2 * h + 2 * sk; i3 = j + 3 * h + 3 * sk; o0 = j; o1 = j + h + sk;
    }
    const Fe x0 = ld_fe(X, i0), x1 = ld_fe(X, i1), x2 = ld_fe(X, i2), x3 = ld_fe(X, i3);
    const Fe z0 = ld_fe(Z, i0), z1 = ld_fe(Z, i1), z2 = ld_fe(Z, i2), z3 = ld_fe(Z, i3);
    st_fe(X2, o0, xr(x0, x2));
    st_fe(X2, o1, xr(x1, x3));
    st_fe(Z2, o0, xr(z0, z2));
    st_fe(Z2, o1, xr(z1, z3));
  }
}

// control: read 2 elements, write 1, contiguous (same byte count per element pair)
__global__ __launch_bounds__(kBlock) void k_copy(const Fe* __restrict__ in, Fe* __restrict__ out, uint64_t n_out) {
  const uint64_t stride = (uint64_t)gridDim.x * kBlock;
  for (uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x; i < n_out; i += stride)
    st_fe(out, i, xr(ld_fe(in, 2 * i), ld_fe(in, 2 * i + 1)));
}

int main() {
  const uint64_t N = 1ull << 24, h = N / 4, pad = 4 * kSkew;
  Fe *T[4], *O[4];
  for (int k = 0; k < 4; ++k) {
    CK(hipMalloc(&T[k], (N + pad) * 32));
    CK(hipMalloc(&O[k], (N / 2 + pad) * 32));
    CK(hipMemset(T[k], 0x11 * (k + 1), (N + pad) * 32));
  }
  hipDeviceProp_t prop;
  CK(hipGetDeviceProperties(&prop, 0));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const double bytes = 768.0 * h;  // 4 tables x (4 reads + 2 writes) x 32 B per pair slot
  auto time = [&](const char* name, auto&& fn) {
    fn();
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(e0));
    for (int i = 0; i < 10; ++i) fn();
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    const double us = ms * 1e3 / 10;
    printf("%-22s %8.1f us  %7.1f GB/s\n", name, us, bytes / (us * 1e-6) / 1e9);
    return 0;
  };
  for (int bpc : {2, 4, 8}) {
    const uint32_t grid = prop.multiProcessorCount * bpc;
    printf("grid %u (%d blocks/CU)\n", grid, bpc);
    time("  quarters", [&] { k_mix<0><<<grid, kBlock>>>(T[0], T[1], T[2], T[3], O[0], O[1], O[2], O[3], h); });
    time("  skewed", [&] { k_mix<1><<<grid, kBlock>>>(T[0], T[1], T[2], T[3], O[0], O[1], O[2], O[3], h); });
    time("  pairwise", [&] { k_mix<2><<<grid, kBlock>>>(T[0], T[1], T[2], T[3], O[0], O[1], O[2], O[3], h); });
    time("  copy 4 tables", [&] {
      for (int k = 0; k < 4; ++k) k_copy<<<grid, kBlock>>>(T[k], O[k], N / 2);
    });
  }
  return 0;
}
