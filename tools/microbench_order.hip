// Round 6: memory-only variants of the first k_gkr_t33's access pattern (the
// W8 shape of microbench_wmix.hip: per chunk of 64 octants a wave folds eight
// corners, each fold reading eight 2 KiB runs — inputs e + k 8 O, k < 8 — and
// writing one 2 KiB run at e = ch 64 + l + f O; xor instead of arithmetic) with
// what the kernel could still change without a new layout:
//   STRIDE  chunks ch = b, b + G, ... (the kernel's order: all blocks on adjacent chunks)
//   BLOCK   block b takes chunks [b cpb, (b + 1) cpb) (each block walks its own region)
//   ROT     STRIDE, but block b starts its eight folds at corner b % 8 (concurrent
//           writes spread over eight regions instead of one)
// each with one or two folds of loads in flight (AHEAD; the kernel runs two).
// Sizes: 4 input tables of 2^24 x 32 B (2.15 GB read), 4 outputs of 2^21 x 32 B.
// Build: hipcc -O3 --offload-arch=gfx950 -o tools/mb_order tools/microbench_order.hip
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

enum { STRIDE = 0, BLOCK = 1, ROT = 2 };
struct Tabs {
  const uint4* in[4];
  uint4* out[4];
};
typedef uint32_t v4u __attribute__((ext_vector_type(4)));
__device__ __forceinline__ uint4 ld_nt(const uint4* p) {
  const v4u v = __builtin_nontemporal_load(reinterpret_cast<const v4u*>(p));
  return make_uint4(v.x, v.y, v.z, v.w);
}
__device__ __forceinline__ void xr(uint4& a, const uint4& c) {
  a.x ^= c.x;
  a.y ^= c.y;
  a.z ^= c.z;
  a.w ^= c.w;
}

// O: octants of the output level; the 8 inputs of output e are e + k 8 O
template <int ORDER, int AHEAD, bool ST, bool LNT = false>
__global__ __launch_bounds__(256, 1) void k_order(Tabs t, size_t O) {
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  const uint4* __restrict__ X = t.in[w];
  uint4* __restrict__ X2 = t.out[w];
  const size_t nch = O / 64, h8 = 8 * O;
  const size_t G = gridDim.x, cpb = nch / G;  // (host: nch % G == 0)
  const int f0 = ORDER == ROT ? (int)(blockIdx.x & 7) : 0;
  auto chunk = [&](size_t i) -> size_t { return ORDER == BLOCK ? blockIdx.x * cpb + i : blockIdx.x + i * G; };
  // unit u = i 8 + f: fold f of the block's i-th chunk; loads of unit u into slot u % (AHEAD + 1)
  constexpr int NS = AHEAD + 1;
  uint4 a[NS][8], b[NS][8];
  const size_t units = cpb * 8;
  auto load = [&](size_t u, int s) {
    const size_t uu = u < units ? u : 0;  // (past the end: unit 0 again, unconditional like the kernel)
    const size_t e = chunk(uu / 8) * 64 + l + (size_t)((f0 + uu % 8) & 7) * O;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      if (LNT) {  // non-temporal loads (MB_MALL)
        a[s][k] = ld_nt(&X[2 * (e + k * h8)]);
        b[s][k] = ld_nt(&X[2 * (e + k * h8) + 1]);
      } else {
        a[s][k] = X[2 * (e + k * h8)];
        b[s][k] = X[2 * (e + k * h8) + 1];
      }
    }
  };
#pragma unroll
  for (int s = 0; s < AHEAD; ++s) load(s, s);
  for (size_t u0 = 0; u0 < units; u0 += NS) {
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      const size_t u = u0 + s;
      load(u + AHEAD, (s + AHEAD) % NS);
      if (u < units) {
        uint4 x = a[s][0], y = b[s][0];
#pragma unroll
        for (int k = 1; k < 8; ++k) {
          xr(x, a[s][k]);
          xr(y, b[s][k]);
        }
        const size_t e = chunk(u / 8) * 64 + l + (size_t)((f0 + u % 8) & 7) * O;
        if (ST) {
          X2[2 * e] = x;
          X2[2 * e + 1] = y;
        } else if ((x.x ^ y.y) == 0x12345678u) {
          X2[2 * e] = x;
        }
      }
    }
  }
}

// longer runs: each lane folds RUN consecutive outputs per fold (the wave's
// runs are 2 RUN KiB per input and output), chunks of 64 RUN octants, the
// kernel's chunk order, AHEAD folds of loads in flight
template <int RUN, int AHEAD>
__global__ __launch_bounds__(256, 1) void k_runs(Tabs t, size_t O) {
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  const uint4* __restrict__ X = t.in[w];
  uint4* __restrict__ X2 = t.out[w];
  const size_t OCT = 64 * RUN, nch = O / OCT, h8 = 8 * O, G = gridDim.x;
  const size_t cpb = (nch + G - 1) / G;
  constexpr int NS = AHEAD + 1;
  uint4 a[NS][8][RUN], b[NS][8][RUN];
  const size_t units = cpb * 8;
  auto base = [&](size_t u) -> size_t {  // first output of lane l in unit u (clamped like the kernel)
    size_t ch = blockIdx.x + (u / 8) * G;
    if (ch >= nch) ch = 0;
    return ch * OCT + (size_t)l * RUN + (size_t)(u % 8) * O;
  };
  auto load = [&](size_t u, int s) {
    const size_t e = base(u);
#pragma unroll
    for (int k = 0; k < 8; ++k)
#pragma unroll
      for (int q = 0; q < RUN; ++q) {
        a[s][k][q] = X[2 * (e + q + k * h8)];
        b[s][k][q] = X[2 * (e + q + k * h8) + 1];
      }
  };
#pragma unroll
  for (int s = 0; s < AHEAD; ++s) load(s, s);
  for (size_t u0 = 0; u0 < units; u0 += NS) {
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      const size_t u = u0 + s;
      if (AHEAD) load(u + AHEAD, (s + AHEAD) % NS); else load(u, s);
      if (u < units && blockIdx.x + (u / 8) * G < nch) {
        const size_t e = base(u);
#pragma unroll
        for (int q = 0; q < RUN; ++q) {
          uint4 x = a[s][0][q], y = b[s][0][q];
#pragma unroll
          for (int k = 1; k < 8; ++k) {
            xr(x, a[s][k][q]);
            xr(y, b[s][k][q]);
          }
          X2[2 * (e + q)] = x;
          X2[2 * (e + q) + 1] = y;
        }
      }
    }
  }
}
template <int RUN, int AHEAD>
float run_runs(const Tabs& t, size_t O, int grid, int reps) {
  if (O % (64 * RUN)) exit(1);
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  std::vector<float> v;
  for (int r = 0; r < reps; ++r) {
    CK(hipEventRecord(e0));
    hipLaunchKernelGGL((k_runs<RUN, AHEAD>), dim3(grid), dim3(256), 0, 0, t, O);
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

// an octant-major input layout (the eight corners of an output adjacent: its
// 256 B at 8 e): a wave reads one contiguous 16 KiB run per 64 outputs (16
// lane-contiguous uint4 loads) and writes their 2 KiB run — the same bytes as
// k_order in one read stream and one write stream; AHEAD units of loads in flight
template <int AHEAD>
__global__ __launch_bounds__(256, 1) void k_seq(Tabs t, size_t nout) {
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  const uint4* __restrict__ X = t.in[w];
  uint4* __restrict__ X2 = t.out[w];
  const size_t nch = nout / 64, G = gridDim.x, units = (nch + G - 1) / G;
  constexpr int NS = AHEAD + 1;
  uint4 a[NS][16];
  auto chunk = [&](size_t u) -> size_t {
    const size_t ch = blockIdx.x + u * G;
    return ch < nch ? ch : 0;
  };
  auto load = [&](size_t u, int s) {
    const uint4* p = X + chunk(u) * 1024 + l;
#pragma unroll
    for (int j = 0; j < 16; ++j) a[s][j] = p[j * 64];
  };
#pragma unroll
  for (int s = 0; s < AHEAD; ++s) load(s, s);
  for (size_t u0 = 0; u0 < units; u0 += NS) {
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      const size_t u = u0 + s;
      if (AHEAD) load(u + AHEAD, (s + AHEAD) % NS); else load(u, s);
      if (u < units && blockIdx.x + u * G < nch) {
        uint4 x = a[s][0], y = a[s][1];
#pragma unroll
        for (int j = 2; j < 16; j += 2) {
          xr(x, a[s][j]);
          xr(y, a[s][j + 1]);
        }
        const size_t e = (blockIdx.x + u * G) * 64 + l;
        X2[2 * e] = x;
        X2[2 * e + 1] = y;
      }
    }
  }
}
template <int AHEAD>
float run_seq(const Tabs& t, size_t nout, int grid, int reps) {
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  std::vector<float> v;
  for (int r = 0; r < reps; ++r) {
    CK(hipEventRecord(e0));
    hipLaunchKernelGGL((k_seq<AHEAD>), dim3(grid), dim3(256), 0, 0, t, nout);
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

// MB_MALL: does the second fold pass find the first one's outputs in the
// Infinity Cache? W8 over the inputs (plain or non-temporal loads) writes the
// 268 MB level; then the same pattern one level down (O / 8) reads it back,
// timed alone. 'cold': the read-back after a read-only stream of the inputs.
template <bool LNT>
void mall_pair(const Tabs& t, const Tabs& t2, size_t O, int grid, float& first, float& second, bool cold) {
  hipEvent_t e0, e1, e2;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  CK(hipEventCreate(&e2));
  CK(hipEventRecord(e0));
  if (cold)
    hipLaunchKernelGGL((k_order<STRIDE, 2, false, false>), dim3(grid), dim3(256), 0, 0, t, O);
  else
    hipLaunchKernelGGL((k_order<STRIDE, 2, true, LNT>), dim3(grid), dim3(256), 0, 0, t, O);
  CK(hipEventRecord(e1));
  hipLaunchKernelGGL((k_order<STRIDE, 2, true, false>), dim3(256), dim3(256), 0, 0, t2, O / 8);
  CK(hipEventRecord(e2));
  CK(hipEventSynchronize(e2));
  CK(hipEventElapsedTime(&first, e0, e1));
  CK(hipEventElapsedTime(&second, e1, e2));
  first *= 1000.f;
  second *= 1000.f;
  CK(hipEventDestroy(e0));
  CK(hipEventDestroy(e1));
  CK(hipEventDestroy(e2));
}

template <int ORDER, int AHEAD, bool ST, bool LNT = false>
float run(const Tabs& t, size_t O, int grid, int reps) {
  const size_t nch = O / 64;
  if (O % 64 || nch % grid || 8 * O * 8 > (1ull << 24)) {
    fprintf(stderr, "bad sizes\n");
    exit(1);
  }
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  std::vector<float> v;
  for (int r = 0; r < reps; ++r) {
    CK(hipEventRecord(e0));
    hipLaunchKernelGGL((k_order<ORDER, AHEAD, ST, LNT>), dim3(grid), dim3(256), 0, 0, t, O);
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
  const size_t N = 1ull << 24;
  Tabs t;
  for (int i = 0; i < 4; ++i) {
    uint4* p;
    CK(hipMalloc(&p, N * 32));
    CK(hipMemset(p, 0x11 * (i + 1), N * 32));
    t.in[i] = p;
    CK(hipMalloc(&t.out[i], N / 8 * 32));
  }
  const size_t O = N / 64;  // 2^18 octants
  const double rd = 4.0 * N * 32, wr = 4.0 * N / 8 * 32;
  const int reps = 9;
  if (getenv("MB_RNT")) {  // round 6: the read-only pattern (k_gkr_d0t's shape) with non-temporal loads
    for (int pass = 0; pass < 3; ++pass)
      for (int grid : {256, 512, 1024}) {
        const float p1 = run<STRIDE, 1, false, false>(t, O, grid, reps), n1 = run<STRIDE, 1, false, true>(t, O, grid, reps);
        const float p2 = run<STRIDE, 2, false, false>(t, O, grid, reps), n2 = run<STRIDE, 2, false, true>(t, O, grid, reps);
        auto tb = [&](float us) { return rd / us / 1e6; };
        printf("grid %4d R8: plain 1 ahead %6.1f us (%.2f TB/s) nt %6.1f (%.2f) | plain 2 ahead %6.1f (%.2f) nt %6.1f (%.2f)\n",
               grid, p1, tb(p1), n1, tb(n1), p2, tb(p2), n2, tb(n2));
        fflush(stdout);
      }
    return 0;
  }
  if (getenv("MB_MALL")) {
    Tabs t2;
    for (int i = 0; i < 4; ++i) {
      t2.in[i] = t.out[i];
      CK(hipMalloc(&t2.out[i], N / 64 * 32));
    }
    const double rb = 4.0 * N / 8 * 32 + 4.0 * N / 64 * 32;
    for (int pass = 0; pass < 8; ++pass) {
      float f0, s0, f1, s1, f2, s2;
      mall_pair<false>(t, t2, O, 256, f0, s0, false);
      mall_pair<true>(t, t2, O, 256, f1, s1, false);
      mall_pair<false>(t, t2, O, 256, f2, s2, true);
      printf("W8 plain loads %6.1f us -> read-back %5.1f us (%.2f TB/s) | W8 nt loads %6.1f -> read-back %5.1f (%.2f) | "
             "after a read-only stream (cold) %5.1f (%.2f)\n",
             f0, s0, rb / s0 / 1e6, f1, s1, rb / s1 / 1e6, s2, rb / s2 / 1e6);
      fflush(stdout);
    }
    return 0;
  }
  if (getenv("MB_SEQ")) {  // round 6: octant-major inputs against the kernel's layout
    for (int pass = 0; pass < 3; ++pass)
      for (int grid : {256, 512, 1024}) {
        const float k2 = run<STRIDE, 2, true>(t, O, grid, reps);
        const float q1 = run_seq<1>(t, N / 8, grid, reps), q2 = run_seq<2>(t, N / 8, grid, reps);
        const float q0 = run_seq<0>(t, N / 8, grid, reps);
        auto tb = [&](float us) { return (rd + wr) / us / 1e6; };
        printf("grid %4d: kernel layout (8 x 2 KiB runs, 2 ahead) %6.1f us (%.2f TB/s) | octant-major 1 ahead %6.1f (%.2f) "
               "2 ahead %6.1f (%.2f) none %6.1f (%.2f)\n",
               grid, k2, tb(k2), q1, tb(q1), q2, tb(q2), q0, tb(q0));
        fflush(stdout);
      }
    return 0;
  }
  if (getenv("MB_RUNS")) {  // round 6: run length (2 / 4 / 8 KiB per input and output run)
    for (int pass = 0; pass < 2; ++pass)
      for (int grid : {256, 512}) {
        const float r1a1 = run_runs<1, 1>(t, O, grid, reps), r1a2 = run_runs<1, 2>(t, O, grid, reps);
        const float r2a1 = run_runs<2, 1>(t, O, grid, reps), r2a0 = run_runs<2, 0>(t, O, grid, reps);
        const float r4a0 = run_runs<4, 0>(t, O, grid, reps);
        auto tb = [&](float us) { return (rd + wr) / us / 1e6; };
        printf("grid %d W8 runs: 2 KiB %6.1f us (%.2f TB/s) / 2 ahead %6.1f (%.2f) | 4 KiB %6.1f (%.2f) / no prefetch "
               "%6.1f (%.2f) | 8 KiB (no prefetch) %6.1f (%.2f)\n",
               grid, r1a1, tb(r1a1), r1a2, tb(r1a2), r2a1, tb(r2a1), r2a0, tb(r2a0), r4a0, tb(r4a0));
        fflush(stdout);
      }
    return 0;
  }
  for (int pass = 0; pass < 2; ++pass) {
    for (int grid : {256, 512}) {
      const float s1 = run<STRIDE, 1, true>(t, O, grid, reps), s2 = run<STRIDE, 2, true>(t, O, grid, reps);
      const float b1 = run<BLOCK, 1, true>(t, O, grid, reps), b2 = run<BLOCK, 2, true>(t, O, grid, reps);
      const float r1 = run<ROT, 1, true>(t, O, grid, reps), r2 = run<ROT, 2, true>(t, O, grid, reps);
      const float s2r = run<STRIDE, 2, false>(t, O, grid, reps), b2r = run<BLOCK, 2, false>(t, O, grid, reps);
      auto tb = [&](float us, double by) { return by / us / 1e6; };
      printf("grid %d W8: stride %6.1f us (%.2f TB/s) / 2 ahead %6.1f (%.2f) | blocked %6.1f (%.2f) / %6.1f (%.2f) | "
             "rotated corners %6.1f (%.2f) / %6.1f (%.2f) || R8 2 ahead: stride %6.1f (%.2f) blocked %6.1f (%.2f)\n",
             grid, s1, tb(s1, rd + wr), s2, tb(s2, rd + wr), b1, tb(b1, rd + wr), b2, tb(b2, rd + wr), r1, tb(r1, rd + wr),
             r2, tb(r2, rd + wr), s2r, tb(s2r, rd), b2r, tb(b2r, rd));
      fflush(stdout);
    }
  }
  return 0;
}
