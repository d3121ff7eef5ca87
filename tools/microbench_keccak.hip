// Latency of one wave-uniform Keccak-f[1600] (dkeccak.hpp) on gfx950 and a
// check against the host permutation. hipcc -O3 --offload-arch=gfx950 tools/microbench_keccak.hip -o tools/mb_keccak
#include <hip/hip_runtime.h>
#include <stdio.h>
#include "dkeccak.hpp"
#include "../zk-research-implementations_amd/csrc/keccak.hpp"

__global__ void k_keccak(uint64_t* st, int iters, unsigned long long* cycles) {
  if (threadIdx.x >= 64) return;
  uint64_t a[25];
  for (int i = 0; i < 25; ++i) a[i] = st[i];
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < iters; ++it) zk::keccak_f1600_uniform(a);
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) {
    for (int i = 0; i < 25; ++i) st[i] = a[i];
    cycles[0] = t1 - t0;
  }
}

int main() {
  uint64_t h[25], *d;
  unsigned long long *dc, cyc;
  for (int i = 0; i < 25; ++i) h[i] = 0x0123456789abcdefull * (i + 1);
  uint64_t ref[25];
  for (int i = 0; i < 25; ++i) ref[i] = h[i];
  for (int k = 0; k < 100; ++k) zk::Keccak256::permute(ref);
  if (hipMalloc(&d, 200) || hipMalloc(&dc, 8)) return 1;
  (void)hipMemcpy(d, h, 200, hipMemcpyHostToDevice);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  (void)hipEventRecord(e0);
  k_keccak<<<1, 64>>>(d, 100, dc);
  (void)hipEventRecord(e1);
  (void)hipEventSynchronize(e1);
  float ms;
  (void)hipEventElapsedTime(&ms, e0, e1);
  (void)hipMemcpy(h, d, 200, hipMemcpyDeviceToHost);
  (void)hipMemcpy(&cyc, dc, 8, hipMemcpyDeviceToHost);
  int ok = 1;
  for (int i = 0; i < 25; ++i) ok &= h[i] == ref[i];
  printf("device keccak %s; %.3f us per permutation (event), %.0f s_memtime ticks per permutation\n",
         ok ? "matches host" : "MISMATCH", ms * 1e3 / 100, cyc / 100.0);
  return !ok;
}
