// Where does a GKR round kernel spend its time? Builds the production
// kernels (kernels.hpp) with ZK_PHASE_TRACE: every block stamps
// s_memrealtime (100 MHz, device-global) at
//   0 start, 1 main loop done, 2 per-thread REDC done, 3 block sum done,
//   4 fan-in arrival counted, 5 (last block) totals formed, 6 published
// and this prints, per size, the spread of each phase over blocks
// (in us, relative to the earliest block start).
// hipcc -O3 --offload-arch=gfx950 tools/microbench_phases.hip -o tools/mb_phases
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <algorithm>
#include <vector>
__device__ unsigned long long* zk_phase_trace;
#define ZK_PHASE_TRACE 1
#include "../zk-research-implementations_amd/csrc/kernels.hpp"

using namespace zk;
#define CK(x) do { hipError_t ck_ = (x); if (ck_ != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(ck_), __LINE__); return 1; } } while (0)

int main() {
  using F = Bn254Fr;
  const uint64_t N = 1ull << 22;
  Fe *A, *S, *M, *P, *W;
  CK(hipMalloc(&A, N * 32)); CK(hipMalloc(&S, N * 32)); CK(hipMalloc(&M, N * 32)); CK(hipMalloc(&P, N * 32));
  CK(hipMalloc(&W, 4 * (N / 2) * 32));
  for (Fe* t : {A, S, M, P}) CK(hipMemset(t, 0x11, N * 32));
  Fe r;
  for (int i = 0; i < 8; ++i) r.v[i] = 0x01020304u * (i + 1) & 0x0fffffff;
  RoundIn rin{};
  rin.r = r;
  uint64_t* parts; uint32_t* ctr; uint64_t* hout; unsigned long long* tr;
  CK(hipMalloc(&parts, (256 * 8 + 8) * kSlotU64 * 8));
  CK(hipMalloc(&ctr, 4096)); CK(hipMemset(ctr, 0, 4096));
  CK(hipHostMalloc(&hout, 4096, hipHostMallocMapped | hipHostMallocCoherent));
  const int maxb = 2048;
  CK(hipMalloc(&tr, maxb * 8 * 8));
  CK(hipMemcpyToSymbol(HIP_SYMBOL(zk_phase_trace), &tr, sizeof(tr)));
  RoundSink sk{parts, ctr, reinterpret_cast<uint64_t*>(ctr + 640), nullptr, hout, reinterpret_cast<uint32_t*>(hout + 64), 1};
  int pc[2] = {0, 0};
  CK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&pc[0], k_gkr_round<F>, kBlock, 0));
  CK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&pc[1], k_gkr_round_lanes<F>, kBlock, 0));
  hipDeviceProp_t prop;
  CK(hipGetDeviceProperties(&prop, 0));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  const char* ph[7] = {"start", "loop", "redc", "bsum", "arrive", "totals", "publish"};
  for (int lanes = 0; lanes < 2; ++lanes)
    for (int lg : {20, 18, 16, 14, 12, 9, 6, 3}) {
      if (lanes && lg > 15) continue;
      const uint64_t hh = 1ull << lg;
      uint64_t g = ((lanes ? 8 : 2) * hh + kBlock - 1) / kBlock;
      g = std::min<uint64_t>(g, (uint64_t)prop.multiProcessorCount * pc[lanes]);
      auto launch = [&] {
        if (lanes)
          k_gkr_round_lanes<F><<<(uint32_t)g, kBlock>>>(A, S, M, P, W, W + N / 2, W + N, W + 3 * N / 2, hh, rin, sk);
        else
          k_gkr_round<F><<<(uint32_t)g, kBlock>>>(A, S, M, P, W, W + N / 2, W + N, W + 3 * N / 2, hh, rin, sk);
      };
      for (int i = 0; i < 3; ++i) launch();
      CK(hipDeviceSynchronize());
      CK(hipMemset(tr, 0, maxb * 64));
      CK(hipDeviceSynchronize());
      CK(hipEventRecord(e0));
      launch();
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      std::vector<unsigned long long> t(g * 8);
      CK(hipMemcpy(t.data(), tr, g * 64, hipMemcpyDeviceToHost));
      unsigned long long t0 = ~0ull;
      for (uint64_t b = 0; b < g; ++b) t0 = std::min(t0, t[b * 8]);
      printf("%s pairs 2^%-2d grid %4llu  event %7.2f us\n", lanes ? "lanes" : "round", lg, (unsigned long long)g, ms * 1e3);
      for (int i = 0; i < 7; ++i) {
        std::vector<double> v;
        for (uint64_t b = 0; b < g; ++b)
          if (t[b * 8 + i]) v.push_back((t[b * 8 + i] - t0) * 0.01);
        if (v.empty()) continue;
        std::sort(v.begin(), v.end());
        printf("    %-8s n=%4zu  min %7.2f  med %7.2f  max %7.2f us\n", ph[i], v.size(), v.front(), v[v.size() / 2], v.back());
      }
    }
  return 0;
}
