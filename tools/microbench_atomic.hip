// Work-queue counters for dynamic chunk hand-out (round 5): what a device-scope
// atomicAdd on a shared counter costs while every CU streams HBM, as a block
// of k_gkr_d0t / k_gkr_t33 would draw its next chunk. Grid of G blocks x 256
// threads; every wave streams its own slice of a 2 GiB buffer (so HBM is busy,
// as in the kernels); thread 0 of each block draws K chunk indices, one per
// iteration of `per` streamed KiB, from
//   shared : one counter for the whole grid
//   xcd    : one counter per XCD (blockIdx % 8)
//   none   : no draws (the streaming-only baseline)
// and records the draw's latency (s_memrealtime, 10 ns ticks). Reports the
// kernel time and the draw latency distribution.
// Build: hipcc -O3 --offload-arch=gfx950 -o tools/mb_atomic tools/microbench_atomic.hip
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

enum { NONE = 0, SHARED = 1, XCD = 2 };

// iters iterations per block; each streams `per` uint4 per lane-group of the
// block (a grid-stride slice) and, in thread 0, draws one index
template <int MODE>
__global__ __launch_bounds__(256) void k_draw(const uint4* __restrict__ in, size_t n4, uint32_t* ctr, int iters,
                                              int per, uint32_t* lat, uint4* sink) {
  uint4 acc = make_uint4(0, 0, 0, 0);
  const size_t stride = (size_t)gridDim.x * 256;
  size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
  uint32_t got = 0;
  for (int it = 0; it < iters; ++it) {
    uint32_t t0 = 0, v = 0;
    if (MODE != NONE && threadIdx.x == 0) {
      t0 = (uint32_t)__builtin_amdgcn_s_memrealtime();
      uint32_t* c = MODE == SHARED ? ctr : ctr + 32 * (blockIdx.x & 7u);
      v = __hip_atomic_fetch_add(c, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
#pragma unroll 4
    for (int k = 0; k < per; ++k) {
      const uint4 x = in[i % n4];
      acc.x ^= x.x;
      acc.y += x.y;
      i += stride;
    }
    if (MODE != NONE && threadIdx.x == 0) {
      got += v;
      const uint32_t t1 = (uint32_t)__builtin_amdgcn_s_memrealtime();
      lat[(size_t)blockIdx.x * iters + it] = t1 - t0;  // draw issued -> result in hand (after the slice's loads)
    }
  }
  if ((acc.x ^ acc.y ^ got) == 0x9e3779b9u) sink[threadIdx.x] = acc;
}

// the draw alone, latency measured right at the result (no loads in between)
template <int MODE>
__global__ __launch_bounds__(256) void k_draw_bare(const uint4* __restrict__ in, size_t n4, uint32_t* ctr, int iters,
                                                   int per, uint32_t* lat, uint4* sink) {
  uint4 acc = make_uint4(0, 0, 0, 0);
  const size_t stride = (size_t)gridDim.x * 256;
  size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
  uint32_t got = 0;
  for (int it = 0; it < iters; ++it) {
    if (threadIdx.x == 0) {
      const uint32_t t0 = (uint32_t)__builtin_amdgcn_s_memrealtime();
      uint32_t* c = MODE == SHARED ? ctr : ctr + 32 * (blockIdx.x & 7u);
      const uint32_t v = __hip_atomic_fetch_add(c, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      got += v;
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      const uint32_t t1 = (uint32_t)__builtin_amdgcn_s_memrealtime();
      lat[(size_t)blockIdx.x * iters + it] = t1 - t0 + (got & 0);
    }
#pragma unroll 4
    for (int k = 0; k < per; ++k) {
      const uint4 x = in[i % n4];
      acc.x ^= x.x;
      acc.y += x.y;
      i += stride;
    }
  }
  if ((acc.x ^ acc.y ^ got) == 0x9e3779b9u) sink[threadIdx.x] = acc;
}

template <class K>
void run(const char* name, K kern, const uint4* in, size_t n4, uint32_t* ctr, int grid, int iters, int per,
         uint32_t* lat, uint4* sink) {
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  std::vector<float> ts;
  std::vector<uint32_t> h((size_t)grid * iters);
  for (int r = 0; r < 5; ++r) {
    CK(hipMemset(ctr, 0, 4096));
    CK(hipMemset(lat, 0, (size_t)grid * iters * 4));
    CK(hipEventRecord(e0));
    hipLaunchKernelGGL(kern, dim3(grid), dim3(256), 0, 0, in, n4, ctr, iters, per, lat, sink);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    ts.push_back(ms * 1000.f);
  }
  CK(hipMemcpy(h.data(), lat, h.size() * 4, hipMemcpyDeviceToHost));
  std::sort(ts.begin(), ts.end());
  std::sort(h.begin(), h.end());
  const double bytes = (double)grid * 256 * iters * per * 16;
  printf("%-28s grid %4d iters %4d per %3d: %8.1f us (%.2f TB/s) | draw latency us: p10 %.2f med %.2f p90 %.2f p99 %.2f max %.2f\n",
         name, grid, iters, per, ts[2], bytes / ts[2] / 1e6, h[h.size() / 10] * 0.01, h[h.size() / 2] * 0.01,
         h[h.size() * 9 / 10] * 0.01, h[h.size() * 99 / 100] * 0.01, h.back() * 0.01);
  fflush(stdout);
  CK(hipEventDestroy(e0));
  CK(hipEventDestroy(e1));
}

int main() {
  const size_t bytes = 2ull << 30, n4 = bytes / 16;
  uint4 *in, *sink;
  uint32_t *ctr, *lat;
  CK(hipMalloc(&in, bytes));
  CK(hipMemset(in, 0x5a, bytes));
  CK(hipMalloc(&sink, 4096));
  CK(hipMalloc(&ctr, 4096));
  const int maxlat = 4096 * 512;
  CK(hipMalloc(&lat, (size_t)maxlat * 4));
  // per = 8 uint4 per thread per iteration = 32 KiB per block per draw (k_gkr_d0t
  // moves 2 x 8 KiB per wave-pair chunk; t33 ~ 200 KiB per chunk)
  for (int grid : {512, 256}) {
    for (int per : {8, 32}) {
      const int iters = (int)std::min<size_t>(n4 / ((size_t)grid * 256 * per), (size_t)maxlat / grid);
      run("none (stream only)", k_draw<NONE>, in, n4, ctr, grid, iters, per, lat, sink);
      run("shared counter", k_draw<SHARED>, in, n4, ctr, grid, iters, per, lat, sink);
      run("per-XCD counters", k_draw<XCD>, in, n4, ctr, grid, iters, per, lat, sink);
      run("shared counter, bare wait", k_draw_bare<SHARED>, in, n4, ctr, grid, iters, per, lat, sink);
      run("per-XCD counters, bare wait", k_draw_bare<XCD>, in, n4, ctr, grid, iters, per, lat, sink);
    }
  }
  return 0;
}
