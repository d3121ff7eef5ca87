// Memory-only variants of the first fold pass (k_gkr_t33 / a fold-by-four pass)
// at the 24-variable sizes: what the read:write mix costs and whether the output
// layout or the store timing changes it. Arithmetic is replaced by xor; every
// variant reads its inputs once (4 tables x 2^24 x 32 B = 2.15 GB).
//   R8   : 8 inputs per output (fold by three), no stores (a data guard keeps the loads)
//   W8   : 8 inputs -> 1 output at e (level-3 table order), one store per fold
//   W8C  : 8 inputs -> 1 output, chunk-major output ([chunk][fold][64 lanes]: 16 KiB runs)
//   W8B  : 8 inputs -> 1 output, the 8 outputs of a chunk stored together after its loads
//   R16  : 16 inputs per output (fold by four), no stores
//   W16  : 16 inputs -> 1 output (134 MB written)
// Build: hipcc -O3 --offload-arch=gfx950 -o tools/mb_wmix tools/microbench_wmix.hip
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e_ = (x);                                                        \
    if (e_ != hipSuccess) {                                                     \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                  \
    }                                                                           \
  } while (0)

enum { R8, W8, W8C, W8B, R16, W16 };

struct Tabs {
  const uint4* in[4];
  uint4* out[4];
};

__device__ __forceinline__ void xr(uint4& a, const uint4& c) {
  a.x ^= c.x;
  a.y ^= c.y;
  a.z ^= c.z;
  a.w ^= c.w;
}

// lanes = 64 consecutive outputs of one corner; NIN inputs NIN*O' apart... exactly
// the t33 pattern64 addressing: e = ch*64 + l + f*O, inputs e + k*(NF*O), k < NIN.
template <int MODE, int NIN, int NF>
__global__ __launch_bounds__(256) void k_mix(Tabs t, size_t O) {
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  const uint4* __restrict__ X = t.in[w];
  uint4* __restrict__ X2 = t.out[w];
  const size_t nch = O / 64, hs = (size_t)NF * O;
  for (size_t ch = blockIdx.x; ch < nch; ch += gridDim.x) {
    uint4 ka[NF], kb[NF];
#pragma unroll
    for (int f = 0; f < NF; ++f) {
      const size_t e = ch * 64 + l + (size_t)f * O;
      uint4 a = X[2 * e], b = X[2 * e + 1];
#pragma unroll
      for (int k = 1; k < NIN; ++k) {
        xr(a, X[2 * (e + k * hs)]);
        xr(b, X[2 * (e + k * hs) + 1]);
      }
      if (MODE == R8 || MODE == R16) {
        if ((a.x ^ b.y) == 0x12345678u) X2[2 * e] = a;  // practically never
      } else if (MODE == W8 || MODE == W16) {
        X2[2 * e] = a;
        X2[2 * e + 1] = b;
      } else if (MODE == W8C) {
        const size_t o = (ch * NF + f) * 64 + l;
        X2[2 * o] = a;
        X2[2 * o + 1] = b;
      } else {
        ka[f] = a;
        kb[f] = b;
      }
    }
    if (MODE == W8B) {
#pragma unroll
      for (int f = 0; f < NF; ++f) {
        const size_t e = ch * 64 + l + (size_t)f * O;
        X2[2 * e] = ka[f];
        X2[2 * e + 1] = kb[f];
      }
    }
  }
}

template <int MODE, int NIN, int NF>
float run(const Tabs& t, size_t O, int grid, int reps) {
  // host-side bounds check: the largest input index and output index the kernel forms
  const size_t in_max = (O - 1) + (size_t)(NF - 1) * O + (size_t)(NIN - 1) * NF * O, out_max = NF * O - 1;
  if (O % 64 || in_max >= (1ull << 24) || out_max >= (1ull << 24) / 8) {
    fprintf(stderr, "bad sizes: O %zu in_max %zu out_max %zu\n", O, in_max, out_max);
    exit(1);
  }
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  std::vector<float> v;
  for (int r = 0; r < reps; ++r) {
    CK(hipEventRecord(e0));
    hipLaunchKernelGGL((k_mix<MODE, NIN, NF>), dim3(grid), dim3(256), 0, 0, t, O);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    v.push_back(ms * 1000.f);
  }
  std::sort(v.begin(), v.end());
  CK(hipEventDestroy(e0));
  CK(hipEventDestroy(e1));
  return v[v.size() / 2];
}


// the real kernel's schedule: the next fold's NIN inputs are loaded (into registers)
// before the current fold is combined and stored (one fold ahead); ST = store or not
template <int NIN, int NF, bool ST>
__global__ __launch_bounds__(256, 1) void k_mix_pf(Tabs t, size_t O) {
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  const uint4* __restrict__ X = t.in[w];
  uint4* __restrict__ X2 = t.out[w];
  const size_t nch = O / 64, hs = (size_t)NF * O;
  uint4 na[NIN], nb[NIN];
  auto load = [&](size_t ch, int f) {
    const size_t e = ch * 64 + l + (size_t)f * O;
#pragma unroll
    for (int k = 0; k < NIN; ++k) {
      na[k] = X[2 * (e + k * hs)];
      nb[k] = X[2 * (e + k * hs) + 1];
    }
  };
  if (blockIdx.x < nch) load(blockIdx.x, 0);
  for (size_t ch = blockIdx.x; ch < nch; ch += gridDim.x) {
#pragma unroll 1
    for (int f = 0; f < NF; ++f) {
      uint4 ca[NIN], cb[NIN];
#pragma unroll
      for (int k = 0; k < NIN; ++k) {
        ca[k] = na[k];
        cb[k] = nb[k];
      }
      if (f + 1 < NF) load(ch, f + 1);
      else if (ch + gridDim.x < nch) load(ch + gridDim.x, 0);
      uint4 a = ca[0], b = cb[0];
#pragma unroll
      for (int k = 1; k < NIN; ++k) {
        xr(a, ca[k]);
        xr(b, cb[k]);
      }
      const size_t e = ch * 64 + l + (size_t)f * O;
      if (ST) {
        X2[2 * e] = a;
        X2[2 * e + 1] = b;
      } else if ((a.x ^ b.y) == 0x12345678u) {
        X2[2 * e] = a;
      }
    }
  }
}

template <int NIN, int NF, bool ST>
float run_pf(const Tabs& t, size_t O, int grid, int reps) {
  const size_t in_max = (O - 1) + (size_t)(NF - 1) * O + (size_t)(NIN - 1) * NF * O, out_max = NF * O - 1;
  if (O % 64 || in_max >= (1ull << 24) || out_max >= (1ull << 24) / 8) {
    fprintf(stderr, "bad sizes: O %zu in_max %zu out_max %zu\n", O, in_max, out_max);
    exit(1);
  }
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  std::vector<float> v;
  for (int r = 0; r < reps; ++r) {
    CK(hipEventRecord(e0));
    hipLaunchKernelGGL((k_mix_pf<NIN, NF, ST>), dim3(grid), dim3(256), 0, 0, t, O);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    v.push_back(ms * 1000.f);
  }
  std::sort(v.begin(), v.end());
  CK(hipEventDestroy(e0));
  CK(hipEventDestroy(e1));
  return v[v.size() / 2];
}

int main() {
  const size_t N = 1ull << 24;  // elements per input table
  Tabs t;
  for (int i = 0; i < 4; ++i) {
    uint4* p;
    CK(hipMalloc(&p, N * 32));
    CK(hipMemset(p, 0x11 * (i + 1), N * 32));
    t.in[i] = p;
    CK(hipMalloc(&t.out[i], N / 8 * 32));
  }
  const double rd = 4.0 * N * 32;
  const int reps = 7;
  for (int grid : {256, 512, 1024}) {
    const size_t O8 = N / 64, O16 = N / 256;  // fold by three writes 8 O8 = N/8, fold by four 16 O16 = N/16
    float r8 = run<R8, 8, 8>(t, O8, grid, reps);
    float w8 = run<W8, 8, 8>(t, O8, grid, reps);
    float w8c = run<W8C, 8, 8>(t, O8, grid, reps);
    float w8b = run<W8B, 8, 8>(t, O8, grid, reps);
    float r16 = run<R16, 16, 16>(t, O16, grid, reps);
    float w16 = run<W16, 16, 16>(t, O16, grid, reps);
    const double wr8 = 4.0 * N / 8 * 32, wr16 = 4.0 * N / 16 * 32;
    printf("grid %4d: R8 %6.1f us (%.2f TB/s) | W8 %6.1f (%.2f) | W8C %6.1f (%.2f) | W8B %6.1f (%.2f) | "
           "R16 %6.1f (%.2f) | W16 %6.1f (%.2f)\n",
           grid, r8, rd / r8 / 1e6, w8, (rd + wr8) / w8 / 1e6, w8c, (rd + wr8) / w8c / 1e6, w8b,
           (rd + wr8) / w8b / 1e6, r16, rd / r16 / 1e6, w16, (rd + wr16) / w16 / 1e6);
    fflush(stdout);
  }
  for (int grid : {256, 512}) {
    const size_t O8 = N / 64, O16 = N / 256;
    float r8 = run_pf<8, 8, false>(t, O8, grid, reps), w8 = run_pf<8, 8, true>(t, O8, grid, reps);
    float r16 = run_pf<16, 16, false>(t, O16, grid, reps), w16 = run_pf<16, 16, true>(t, O16, grid, reps);
    const double wr8 = 4.0 * N / 8 * 32, wr16 = 4.0 * N / 16 * 32;
    printf("prefetch one fold ahead, grid %4d: R8 %6.1f us (%.2f TB/s) | W8 %6.1f (%.2f) | R16 %6.1f (%.2f) | W16 %6.1f (%.2f)\n",
           grid, r8, rd / r8 / 1e6, w8, (rd + wr8) / w8 / 1e6, r16, rd / r16 / 1e6, w16, (rd + wr16) / w16 / 1e6);
    fflush(stdout);
  }
  return 0;
}
