// Kernel-to-kernel gap on one stream: block 0 stamps entry (s_memrealtime,
// 100 MHz), the last block to finish stamps exit; gap = entry(i+1) - exit(i).
// Cases: one block; 1024 blocks; 1024 blocks each writing a buffer (dirty L2
// at kernel end); the one-block chain captured in a hipGraph.
// hipcc --offload-arch=gfx950 -O3 -o tools/mb_gap tools/microbench_gap.hip
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <cstdio>
#include <cstdint>
#include <vector>
#include <algorithm>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); return 1; } } while (0)

__global__ void k_mark(uint64_t* ts, uint32_t* counter, int i, uint4* buf, uint64_t n16) {
  if (blockIdx.x == 0 && threadIdx.x == 0) ts[2 * i] = __builtin_amdgcn_s_memrealtime();
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; j < n16; j += stride)
    buf[j] = make_uint4((uint32_t)j, i, 0, 0);
  __syncthreads();
  if (threadIdx.x == 0) {
    __threadfence();
    const uint32_t prev = atomicAdd(counter + i, 1u);
    if (prev == gridDim.x - 1) ts[2 * i + 1] = __builtin_amdgcn_s_memrealtime();
  }
}

// variants: LDS = 87 KB of static LDS (occupancy 1, as k_gkr_t33); HOST = the
// last block also stores to pinned coherent host memory (as publish_limbs)
template <bool LDS, bool HOST>
__global__ __launch_bounds__(256) void k_mark2(uint64_t* ts, uint32_t* counter, int i, uint64_t* host) {
  if (blockIdx.x == 0 && threadIdx.x == 0) ts[2 * i] = __builtin_amdgcn_s_memrealtime();
  if constexpr (LDS) {
    __shared__ uint32_t big[87 * 1024 / 4];
    for (int j = threadIdx.x; j < 87 * 256; j += 256) big[j] = j * i;
    __syncthreads();
    if (big[(threadIdx.x * 7 + i) % (87 * 256)] == 0xdeadbeefu) ts[0] = 0;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    __threadfence();
    const uint32_t prev = atomicAdd(counter + i, 1u);
    if (prev == gridDim.x - 1) {
      if constexpr (HOST) __hip_atomic_store(host + i, (uint64_t)i + 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
      ts[2 * i + 1] = __builtin_amdgcn_s_memrealtime();
    }
  }
}

static void report(const char* name, const std::vector<uint64_t>& h, int n) {
  std::vector<double> gaps, durs;
  for (int i = 1; i < n; ++i) gaps.push_back((double)(h[2 * i] - h[2 * i - 1]) * 0.01);
  for (int i = 1; i < n; ++i) durs.push_back((double)(h[2 * i + 1] - h[2 * i]) * 0.01);
  std::sort(gaps.begin(), gaps.end());
  std::sort(durs.begin(), durs.end());
  printf("%-44s gap exit->entry: min %.2f med %.2f max %.2f us | kernel entry->exit med %.2f us\n", name, gaps.front(),
         gaps[gaps.size() / 2], gaps.back(), durs[durs.size() / 2]);
}

int main() {
  const int n = 32;
  uint64_t* ts;
  uint32_t* cnt;
  uint4* buf;
  const uint64_t big = 64ull << 20;  // bytes written per kernel in the dirty case
  CK(hipMalloc(&ts, 2 * n * sizeof(uint64_t)));
  CK(hipMalloc(&cnt, n * sizeof(uint32_t)));
  CK(hipMalloc(&buf, big));
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  std::vector<uint64_t> h(2 * n);
  struct Case { const char* name; int grid; uint64_t n16; };
  const Case cases[] = {{"1 block, no stores", 1, 0},
                        {"1024 blocks, no stores", 1024, 0},
                        {"1024 blocks, 64 MB of stores each", 1024, big / 16},
                        {"1024 blocks, 4 MB of stores each", 1024, (4ull << 20) / 16}};
  for (int rep = 0; rep < 2; ++rep) {
    for (const Case& c : cases) {
      CK(hipMemsetAsync(cnt, 0, n * sizeof(uint32_t), s));
      for (int i = 0; i < n; ++i) hipLaunchKernelGGL(k_mark, dim3(c.grid), dim3(256), 0, s, ts, cnt, i, buf, c.n16);
      CK(hipStreamSynchronize(s));
      CK(hipMemcpy(h.data(), ts, h.size() * sizeof(uint64_t), hipMemcpyDeviceToHost));
      if (rep == 1) report(c.name, h, n);
    }
  }
  uint64_t* host;
  CK(hipHostMalloc(reinterpret_cast<void**>(&host), 4096, hipHostMallocMapped | hipHostMallocCoherent));
  struct V { const char* name; void (*k)(uint64_t*, uint32_t*, int, uint64_t*); int grid; };
  const V vs[] = {{"256 blocks, plain", k_mark2<false, false>, 256},
                  {"256 blocks, 87 KB LDS", k_mark2<true, false>, 256},
                  {"256 blocks, host store at the end", k_mark2<false, true>, 256},
                  {"256 blocks, 87 KB LDS + host store", k_mark2<true, true>, 256},
                  {"4096 blocks, 87 KB LDS + host store", k_mark2<true, true>, 4096}};
  for (const V& v : vs) {
    for (int rep = 0; rep < 2; ++rep) {
      CK(hipMemsetAsync(cnt, 0, n * sizeof(uint32_t), s));
      for (int i = 0; i < n; ++i) hipLaunchKernelGGL(v.k, dim3(v.grid), dim3(256), 0, s, ts, cnt, i, host);
      CK(hipStreamSynchronize(s));
    }
    CK(hipMemcpy(h.data(), ts, h.size() * sizeof(uint64_t), hipMemcpyDeviceToHost));
    report(v.name, h, n);
  }
  // hipExtLaunchKernelGGL with null events (the library's launch call)
  for (int rep = 0; rep < 2; ++rep) {
    CK(hipMemsetAsync(cnt, 0, n * sizeof(uint32_t), s));
    for (int i = 0; i < n; ++i)
      hipExtLaunchKernelGGL(k_mark2<true, true>, dim3(256), dim3(256), 0, s, nullptr, nullptr, 0, ts, cnt, i, host);
    CK(hipStreamSynchronize(s));
  }
  CK(hipMemcpy(h.data(), ts, h.size() * sizeof(uint64_t), hipMemcpyDeviceToHost));
  report("hipExtLaunchKernelGGL, 87 KB LDS + host", h, n);
  // the same chain captured in a graph
  for (int g : {1, 1024}) {
    hipGraph_t graph;
    hipGraphExec_t exec;
    CK(hipStreamBeginCapture(s, hipStreamCaptureModeGlobal));
    for (int i = 0; i < n; ++i) hipLaunchKernelGGL(k_mark, dim3(g), dim3(256), 0, s, ts, cnt, i, buf, (uint64_t)0);
    CK(hipStreamEndCapture(s, &graph));
    CK(hipGraphInstantiate(&exec, graph, nullptr, nullptr, 0));
    for (int rep = 0; rep < 2; ++rep) {
      CK(hipMemsetAsync(cnt, 0, n * sizeof(uint32_t), s));
      CK(hipGraphLaunch(exec, s));
      CK(hipStreamSynchronize(s));
    }
    CK(hipMemcpy(h.data(), ts, h.size() * sizeof(uint64_t), hipMemcpyDeviceToHost));
    report(g == 1 ? "hipGraph, 1 block" : "hipGraph, 1024 blocks", h, n);
    CK(hipGraphExecDestroy(exec));
    CK(hipGraphDestroy(graph));
  }
  return 0;
}
