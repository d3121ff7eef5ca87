// Probe for a one-shot all-reduce over IPC-mapped receive buffers (two
// processes, usually on one card here; one per GPU on a multi-GPU node):
//   1. each rank allocates an uncached device buffer (hipDeviceMallocUncached),
//      exports it (hipIpcGetMemHandle) through a file, opens the peer's;
//   2. a one-block kernel writes 16 words into the peer's slot with
//      system-scope stores, drains, raises the slot's tag, then polls its own
//      buffer for the peer's tag and checks the peer's words;
//   3. ping-pong: K rounds of "write tag k to the peer, wait for the peer's
//      tag k" inside one kernel — the round-trip latency.
// Usage: p2p_probe RANK DIR [DEVICE]   (run ranks 0 and 1 concurrently)
// Build: hipcc -O3 -std=c++17 --offload-arch=gfx950 -o tools/p2p_probe tools/p2p_probe.hip
#include <hip/hip_runtime.h>
#include <unistd.h>

#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <thread>

#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e_ = (x);                                                        \
    if (e_ != hipSuccess) {                                                     \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                  \
    }                                                                           \
  } while (0)

constexpr uint64_t kTicks = 500000000ull;  // 5 s of s_memrealtime

__global__ void k_exchange(uint64_t* mine, uint64_t* peer, int rank, uint64_t* out) {
  const int t = threadIdx.x;
  const int other = 1 - rank;
  if (t < 16) __hip_atomic_store(peer + rank * 64 + t, (uint64_t)(rank + 1) * 1000 + t, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (t == 0) {
    __hip_atomic_store(peer + rank * 64 + 63, (uint64_t)7, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    uint64_t ok = 1;
    while (__hip_atomic_load(mine + other * 64 + 63, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) != 7) {
      __builtin_amdgcn_s_sleep(1);
      if (__builtin_amdgcn_s_memrealtime() - t0 > kTicks) { ok = 0; break; }
    }
    uint64_t bad = 0;
    for (int i = 0; i < 16; ++i)
      bad += __hip_atomic_load(mine + other * 64 + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != (uint64_t)(other + 1) * 1000 + i;
    out[0] = ok;
    out[1] = bad;
    out[2] = __builtin_amdgcn_s_memrealtime() - t0;
  }
}

__global__ void k_pingpong(uint64_t* mine, uint64_t* peer, int rank, int K, uint64_t* out) {
  if (threadIdx.x != 0) return;
  const int other = 1 - rank;
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  uint64_t ok = 1;
  for (int k = 1; k <= K && ok; ++k) {
    if (rank == 0) __hip_atomic_store(peer + 128 + rank, (uint64_t)k, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    const uint64_t w0 = __builtin_amdgcn_s_memrealtime();
    while (__hip_atomic_load(mine + 128 + other, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) < (uint64_t)k)
      if (__builtin_amdgcn_s_memrealtime() - w0 > kTicks) { ok = 0; break; }
    if (rank == 1) __hip_atomic_store(peer + 128 + rank, (uint64_t)k, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  }
  out[3] = ok;
  out[4] = __builtin_amdgcn_s_memrealtime() - t0;
}

int main(int argc, char** argv) {
  if (argc < 3) {
    fprintf(stderr, "usage: p2p_probe RANK DIR [DEVICE]\n");
    return 2;
  }
  const int rank = atoi(argv[1]);
  const std::string dir = argv[2];
  const int dev = argc > 3 ? atoi(argv[3]) : 0;
  CK(hipSetDevice(dev));
  uint64_t* mine = nullptr;
  CK(hipExtMallocWithFlags((void**)&mine, 4096, hipDeviceMallocUncached));
  CK(hipMemset(mine, 0, 4096));
  uint64_t* out = nullptr;
  CK(hipHostMalloc((void**)&out, 64, hipHostMallocDefault));
  for (int i = 0; i < 8; ++i) out[i] = 0;
  hipIpcMemHandle_t h;
  CK(hipIpcGetMemHandle(&h, mine));
  {
    const std::string tmp = dir + "/p2p_" + std::to_string(rank) + ".tmp", fin = dir + "/p2p_" + std::to_string(rank) + ".h";
    FILE* f = fopen(tmp.c_str(), "wb");
    fwrite(&h, sizeof(h), 1, f);
    fclose(f);
    rename(tmp.c_str(), fin.c_str());
  }
  hipIpcMemHandle_t ph;
  const std::string pf = dir + "/p2p_" + std::to_string(1 - rank) + ".h";
  const auto w0 = std::chrono::steady_clock::now();
  for (;;) {
    FILE* f = fopen(pf.c_str(), "rb");
    if (f && fread(&ph, sizeof(ph), 1, f) == 1) {
      fclose(f);
      break;
    }
    if (f) fclose(f);
    if (std::chrono::steady_clock::now() - w0 > std::chrono::seconds(30)) {
      fprintf(stderr, "rank %d: no peer handle\n", rank);
      return 1;
    }
    std::this_thread::sleep_for(std::chrono::milliseconds(5));
  }
  uint64_t* peer = nullptr;
  CK(hipIpcOpenMemHandle((void**)&peer, ph, hipIpcMemLazyEnablePeerAccess));
  hipLaunchKernelGGL(k_exchange, dim3(1), dim3(64), 0, 0, mine, peer, rank, out);
  CK(hipDeviceSynchronize());
  printf("rank %d exchange: arrived %llu, wrong words %llu, %.2f us\n", rank, (unsigned long long)out[0],
         (unsigned long long)out[1], out[2] / 100.0);
  const int K = 2000;
  hipLaunchKernelGGL(k_pingpong, dim3(1), dim3(64), 0, 0, mine, peer, rank, K, out);
  CK(hipDeviceSynchronize());
  printf("rank %d ping-pong: ok %llu, %d round trips, %.3f us each\n", rank, (unsigned long long)out[3], K,
         out[4] / 100.0 / K);
  CK(hipIpcCloseMemHandle(peer));
  CK(hipFree(mine));
  return (out[0] == 1 && out[1] == 0 && out[3] == 1) ? 0 : 1;
}
