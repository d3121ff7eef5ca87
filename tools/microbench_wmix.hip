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
// and (round 4) R8 / W8 with the inputs landed in LDS by LDS-DMA (k_mix_glds).
// Round 5: `mb_wmix calib` (see calib() below).
// Build: hipcc -O3 --offload-arch=gfx950 -o tools/mb_wmix tools/microbench_wmix.hip
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <string>
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

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ void nt_store(uint4* p, const uint4& v) {
  const u32x4 x = {v.x, v.y, v.z, v.w};
  __builtin_nontemporal_store(x, reinterpret_cast<u32x4*>(p));
}

typedef uint32_t v4u_nt __attribute__((ext_vector_type(4)));
__device__ __forceinline__ uint4 ld_nt(const uint4* p) {
  const v4u_nt v = __builtin_nontemporal_load(reinterpret_cast<const v4u_nt*>(p));
  return make_uint4(v.x, v.y, v.z, v.w);
}
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
// LDC / STC: loads / stores lane-contiguous (instruction i of a wave moves the
// i-th contiguous KiB of the wave's 2 KiB run: whole lines per instruction)
// instead of the kernel's element-per-lane shape (lane l: bytes 32 l .. 32 l + 31
// in two 16-B instructions, each touching every line of the run half)
// RUN (round 5): each wave writes its chunk's NF folds as ONE contiguous run
// (output index (ch NF + f) 64 + l: 16 KiB per chunk and table) instead of NF
// runs of 2 KiB spread over the level-3 table; NTS: non-temporal stores
template <int NIN, int NF, bool ST, bool LDC = false, bool STC = false, bool RUN = false, bool NTS = false, bool NTL = false>
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
      if (LDC && NTL) {  // (round 6: non-temporal, whole lines per instruction)
        const size_t r = ch * 64 + (size_t)f * O + k * hs;
        na[k] = ld_nt(&X[2 * r + l]);
        nb[k] = ld_nt(&X[2 * r + 64 + l]);
      } else if (NTL) {
        na[k] = ld_nt(&X[2 * (e + k * hs)]);
        nb[k] = ld_nt(&X[2 * (e + k * hs) + 1]);
      } else if (LDC) {
        const size_t r = ch * 64 + (size_t)f * O + k * hs;  // the run's first element
        na[k] = X[2 * r + l];
        nb[k] = X[2 * r + 64 + l];
      } else {
        na[k] = X[2 * (e + k * hs)];
        nb[k] = X[2 * (e + k * hs) + 1];
      }
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
      const size_t e = RUN ? (ch * NF + f) * 64 + l : ch * 64 + l + (size_t)f * O;
      if (ST && NTS) {
        nt_store(&X2[2 * e], a);
        nt_store(&X2[2 * e + 1], b);
      } else if (ST && STC) {
        const size_t r = ch * 64 + (size_t)f * O;
        X2[2 * r + l] = a;
        X2[2 * r + 64 + l] = b;
      } else if (ST) {
        X2[2 * e] = a;
        X2[2 * e + 1] = b;
      } else if ((a.x ^ b.y) == 0x12345678u) {
        X2[2 * e] = a;
      }
    }
  }
}

template <int NIN, int NF, bool ST, bool LDC = false, bool STC = false, bool RUN = false, bool NTS = false, bool NTL = false>
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
    hipLaunchKernelGGL((k_mix_pf<NIN, NF, ST, LDC, STC, RUN, NTS, NTL>), dim3(grid), dim3(256), 0, 0, t, O);
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

// The same pattern with the inputs landed in LDS by LDS-DMA (global_load_lds_dwordx4:
// no VGPR destination) instead of a register prefetch: each wave streams its own
// table through a private ring of DEPTH units (a unit = KU of a fold's 8 inputs,
// KU x 2 KiB), waits for a unit with a counted vmcnt (no barrier: every wave reads
// only what it loaded itself), reads its element of each input (two ds_read_b128),
// and stores the fold's output as the kernel does. WPS = waves per SIMD the launch
// bound allows (LDS: 4 WPS waves x DEPTH x KU x 2 KiB per CU).
template <int N>
__device__ __forceinline__ void wait_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}
template <int NF, bool ST, int KU, int DEPTH, int WPS, int AUX = 0>
__global__ __launch_bounds__(256, WPS) void k_mix_glds(Tabs t, size_t O) {
  constexpr int NIN = 8, UPF = NIN / KU;  // units per fold
  __shared__ uint4 ring[4][DEPTH][KU][128];
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  const uint4* __restrict__ X = t.in[w];
  uint4* __restrict__ X2 = t.out[w];
  const size_t nch = O / 64, hs = (size_t)NF * O;
  const size_t my = nch > blockIdx.x ? (nch - 1 - blockIdx.x) / gridDim.x + 1 : 0;  // chunks of this block
  const size_t nu = my * NF * UPF;                                                  // units of this wave
  auto issue = [&](size_t u) {  // unit u -> slot u % DEPTH (past the end: chunk 0 again, never read)
    const size_t q = u < nu ? u : 0;
    const size_t ch = blockIdx.x + (q / (NF * UPF)) * gridDim.x;
    const int f = (int)((q / UPF) % NF), h = (int)(q % UPF);
    const size_t e0 = ch * 64 + (size_t)f * O;
#pragma unroll
    for (int k = 0; k < KU; ++k) {
      const char* g = (const char*)(X + 2 * (e0 + (size_t)(h * KU + k) * hs)) + 16 * l;
      __attribute__((address_space(3))) void* d = (__attribute__((address_space(3))) void*)&ring[w][u % DEPTH][k][0];
      __builtin_amdgcn_global_load_lds((const void*)g, d, 16, 0, AUX);
      __builtin_amdgcn_global_load_lds((const void*)(g + 1024), (__attribute__((address_space(3))) void*)&ring[w][u % DEPTH][k][64], 16, 0, AUX);
    }
  };
  if (nu == 0) return;
#pragma unroll
  for (int d = 0; d < DEPTH - 1; ++d) issue(d);
  uint4 a = make_uint4(0, 0, 0, 0), b = a;
  for (size_t u = 0; u < nu; ++u) {
    issue(u + DEPTH - 1);
    wait_vm<2 * KU * (DEPTH - 1)>();  // unit u landed (stores issued since count too: a conservative wait)
#pragma unroll
    for (int k = 0; k < KU; ++k) {
      xr(a, ring[w][u % DEPTH][k][2 * l]);
      xr(b, ring[w][u % DEPTH][k][2 * l + 1]);
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // the slot's reads are done before it is refilled
    if ((u + 1) % UPF == 0) {
      const size_t q = u / UPF, ch = blockIdx.x + (q / NF) * gridDim.x;
      const size_t e = ch * 64 + l + (q % NF) * O;
      if (ST) {
        X2[2 * e] = a;
        X2[2 * e + 1] = b;
      } else if ((a.x ^ b.y) == 0x12345678u) {
        X2[2 * e] = a;
      }
      a = make_uint4(0, 0, 0, 0);
      b = a;
    }
  }
  wait_vm<0>();
}

template <int NF, bool ST, int KU, int DEPTH, int WPS, int AUX = 0>
float run_glds(const Tabs& t, size_t O, int grid, int reps) {
  const size_t in_max = (O - 1) + (size_t)(NF - 1) * O + (size_t)7 * NF * O, out_max = NF * O - 1;
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
    hipLaunchKernelGGL((k_mix_glds<NF, ST, KU, DEPTH, WPS, AUX>), dim3(grid), dim3(256), 0, 0, t, O);
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

// plain copy of 2^24 x 32 B per table (read + write the same bytes), lane-contiguous uint4
__global__ __launch_bounds__(256) void k_copy(Tabs t, size_t n4) {
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  const uint4* __restrict__ X = t.in[w];
  uint4* __restrict__ Y = t.out[w];
  for (size_t i = (size_t)blockIdx.x * 64 + l; i < n4; i += (size_t)gridDim.x * 64) Y[i] = X[i];
}

// calibration copy (round 5): U uint4 per lane in flight (all U loads issued
// before the U stores), lane-contiguous; NT: non-temporal stores
template <int U, bool NT>
__global__ __launch_bounds__(256) void k_copyu(Tabs t, size_t n4) {
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  const uint4* __restrict__ X = t.in[w];
  uint4* __restrict__ Y = t.out[w];
  const size_t step = (size_t)gridDim.x * 64 * U;
  for (size_t i = (size_t)blockIdx.x * 64 * U + l; i < n4; i += step) {
    uint4 v[U];
#pragma unroll
    for (int k = 0; k < U; ++k) v[k] = X[i + 64 * k];
#pragma unroll
    for (int k = 0; k < U; ++k) {
      if (NT)
        nt_store(&Y[i + 64 * k], v[k]);
      else
        Y[i + 64 * k] = v[k];
    }
  }
}
template <int U, bool NT>
float run_copyu(const Tabs& t, size_t n4, int grid, int reps) {
  if (n4 % (64 * U)) exit(1);
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  std::vector<float> v;
  for (int r = 0; r < reps; ++r) {
    CK(hipEventRecord(e0));
    hipLaunchKernelGGL((k_copyu<U, NT>), dim3(grid), dim3(256), 0, 0, t, n4);
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

// round 5: `mb_wmix calib` — copies of 4 x 512 MiB (2 GiB read + 2 GiB written)
// at 1-4 blocks per CU, 1 or 4 uint4 per lane in flight, plain / non-temporal
// stores; then the first t33 pattern (W8, one fold ahead as the kernel) with
// today's output layout (eight 2 KiB runs per wave and chunk) against one
// contiguous 16 KiB run per wave and chunk, plain and non-temporal.
int calib() {
  const size_t N = 1ull << 24;
  Tabs t;
  for (int i = 0; i < 4; ++i) {
    uint4* p;
    CK(hipMalloc(&p, N * 32));
    CK(hipMemset(p, 0x11 * (i + 1), N * 32));
    t.in[i] = p;
    CK(hipMalloc(&t.out[i], N * 32));
    CK(hipMemset(t.out[i], 0, N * 32));
  }
  const int reps = 7;
  const size_t n4 = N * 2;  // uint4 per table: 512 MiB
  const double bytes = 2.0 * 4 * n4 * 16;
  for (int grid : {256, 512, 1024, 2048, 4096}) {
    const float a = run_copyu<1, false>(t, n4, grid, reps), b = run_copyu<4, false>(t, n4, grid, reps);
    const float c = run_copyu<1, true>(t, n4, grid, reps), d = run_copyu<4, true>(t, n4, grid, reps);
    printf("copy 2 GiB + 2 GiB, grid %4d: U1 %7.1f us %.2f TB/s | U4 %7.1f %.2f | U1 nt %7.1f %.2f | U4 nt %7.1f %.2f\n", grid,
           a, bytes / a / 1e6, b, bytes / b / 1e6, c, bytes / c / 1e6, d, bytes / d / 1e6);
    fflush(stdout);
  }
  const size_t O8 = N / 64;
  const double rd = 4.0 * N * 32, wr8 = 4.0 * N / 8 * 32;
  for (int grid : {256, 512}) {
    const float r8 = run_pf<8, 8, false>(t, O8, grid, reps);
    const float w8 = run_pf<8, 8, true>(t, O8, grid, reps);
    const float w8r = run_pf<8, 8, true, false, false, true>(t, O8, grid, reps);
    const float w8n = run_pf<8, 8, true, false, false, false, true>(t, O8, grid, reps);
    const float w8rn = run_pf<8, 8, true, false, false, true, true>(t, O8, grid, reps);
    printf("t33 pattern (one fold ahead), grid %d: R8 %6.1f us (%.2f TB/s) | W8 2 KiB runs %6.1f (%.2f) | W8 16 KiB run "
           "%6.1f (%.2f) | W8 nt %6.1f (%.2f) | W8 16 KiB run nt %6.1f (%.2f)\n",
           grid, r8, rd / r8 / 1e6, w8, (rd + wr8) / w8 / 1e6, w8r, (rd + wr8) / w8r / 1e6, w8n, (rd + wr8) / w8n / 1e6,
           w8rn, (rd + wr8) / w8rn / 1e6);
    fflush(stdout);
  }
  return 0;
}

int main(int argc, char** argv) {
  if (argc > 1 && std::string(argv[1]) == "calib") return calib();
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
  if (argc > 1 && std::string(argv[1]) == "pfnt") {  // round 6: register loads, nt, element vs lane-contiguous shape
    const size_t O8 = N / 64;
    const double wr8 = 4.0 * N / 8 * 32;
    for (int pass = 0; pass < 3; ++pass)
      for (int grid : {256, 512}) {
        const float re = run_pf<8, 8, false>(t, O8, grid, reps), ren = run_pf<8, 8, false, false, false, false, false, true>(t, O8, grid, reps);
        const float rl = run_pf<8, 8, false, true>(t, O8, grid, reps), rln = run_pf<8, 8, false, true, false, false, false, true>(t, O8, grid, reps);
        const float we = run_pf<8, 8, true>(t, O8, grid, reps), wen = run_pf<8, 8, true, false, false, false, false, true>(t, O8, grid, reps);
        const float wl = run_pf<8, 8, true, true>(t, O8, grid, reps), wln = run_pf<8, 8, true, true, false, false, false, true>(t, O8, grid, reps);
        const float wlls = run_pf<8, 8, true, true, true, false, false, true>(t, O8, grid, reps);  // + whole-line stores
        auto r_ = [&](float us) { return rd / us / 1e6; };
        auto w_ = [&](float us) { return (rd + wr8) / us / 1e6; };
        printf("regs grid %4d: R8 elem %6.1f (%.2f) nt %6.1f (%.2f) | R8 lane-contig %6.1f (%.2f) nt %6.1f (%.2f) | W8 elem %6.1f (%.2f) "
               "nt %6.1f (%.2f) | W8 lane-contig %6.1f (%.2f) nt %6.1f (%.2f) | + lane-contig stores %6.1f (%.2f)\n",
               grid, re, r_(re), ren, r_(ren), rl, r_(rl), rln, r_(rln), we, w_(we), wen, w_(wen), wl, w_(wl), wln, w_(wln),
               wlls, w_(wlls));
        fflush(stdout);
      }
    return 0;
  }
  if (argc > 1 && std::string(argv[1]) == "gldsnt") {  // round 6: LDS-DMA with the non-temporal policy (aux 2)
    const size_t O8 = N / 64;
    const double wr8 = 4.0 * N / 8 * 32;
    for (int pass = 0; pass < 3; ++pass)
      for (int grid : {256, 512, 1024}) {
        const float r1 = run_glds<8, false, 8, 2, 1>(t, O8, grid, reps), r1n = run_glds<8, false, 8, 2, 1, 2>(t, O8, grid, reps);
        const float r2 = run_glds<8, false, 4, 2, 2>(t, O8, grid, reps), r2n = run_glds<8, false, 4, 2, 2, 2>(t, O8, grid, reps);
        const float w1 = run_glds<8, true, 8, 2, 1>(t, O8, grid, reps), w1n = run_glds<8, true, 8, 2, 1, 2>(t, O8, grid, reps);
        printf("LDS-DMA grid %4d: R8 1 w/SIMD %6.1f us (%.2f TB/s) nt %6.1f (%.2f) | R8 2 w/SIMD %6.1f (%.2f) nt %6.1f (%.2f) | "
               "W8 1 w/SIMD %6.1f (%.2f) nt loads %6.1f (%.2f)\n",
               grid, r1, rd / r1 / 1e6, r1n, rd / r1n / 1e6, r2, rd / r2 / 1e6, r2n, rd / r2n / 1e6, w1, (rd + wr8) / w1 / 1e6,
               w1n, (rd + wr8) / w1n / 1e6);
        fflush(stdout);
      }
    return 0;
  }
  {  // calibration: copy 4 x 256 MiB (the output buffers hold N/8 elements: copy that much)
    const size_t n4 = N / 8 * 2;
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (int grid : {1024, 4096}) {
      std::vector<float> v;
      for (int r = 0; r < reps; ++r) {
        CK(hipEventRecord(e0));
        hipLaunchKernelGGL(k_copy, dim3(grid), dim3(256), 0, 0, t, n4);
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        v.push_back(ms * 1000.f);
      }
      std::sort(v.begin(), v.end());
      printf("copy (4 x %zu MiB read + written), grid %d: %.1f us = %.2f TB/s (read + write)\n", n4 * 16 >> 20, grid,
             v[reps / 2], 2.0 * 4 * n4 * 16 / v[reps / 2] / 1e6);
    }
  }
  for (int grid : {256, 512}) {
    const size_t O8 = N / 64;
    const double wr8 = 4.0 * N / 8 * 32;
    float r8 = run_pf<8, 8, false>(t, O8, grid, reps), w8 = run_pf<8, 8, true>(t, O8, grid, reps);
    float r8l = run_pf<8, 8, false, true>(t, O8, grid, reps);
    float w8ls = run_pf<8, 8, true, true, false>(t, O8, grid, reps);
    float w8sl = run_pf<8, 8, true, false, true>(t, O8, grid, reps);
    float w8ll = run_pf<8, 8, true, true, true>(t, O8, grid, reps);
    printf("fold by three, one fold ahead, grid %4d: R8 %6.1f us (%.2f TB/s) | W8 %6.1f (%.2f) | R8 lane-contig loads %6.1f (%.2f) | "
           "W8 lc loads %6.1f (%.2f) | W8 lc stores %6.1f (%.2f) | W8 lc both %6.1f (%.2f)\n",
           grid, r8, rd / r8 / 1e6, w8, (rd + wr8) / w8 / 1e6, r8l, rd / r8l / 1e6, w8ls, (rd + wr8) / w8ls / 1e6, w8sl,
           (rd + wr8) / w8sl / 1e6, w8ll, (rd + wr8) / w8ll / 1e6);
    fflush(stdout);
  }
  // LDS-DMA landing (round 4): one wave per SIMD with whole folds in a 2-deep
  // ring, and two waves per SIMD with half folds (4 inputs) in 2- and 3-deep rings
  for (int grid : {256, 512, 1024}) {
    const size_t O8 = N / 64;
    const double wr8 = 4.0 * N / 8 * 32;
    float r1 = run_glds<8, false, 8, 2, 1>(t, O8, grid, reps), w1 = run_glds<8, true, 8, 2, 1>(t, O8, grid, reps);
    float r2 = run_glds<8, false, 4, 2, 2>(t, O8, grid, reps), w2 = run_glds<8, true, 4, 2, 2>(t, O8, grid, reps);
    float w3 = run_glds<8, true, 2, 4, 2>(t, O8, grid, reps);
    printf("LDS-DMA, grid %4d: 1 wave/SIMD (fold units, depth 2): R8 %6.1f us (%.2f TB/s) W8 %6.1f (%.2f) | 2 waves/SIMD "
           "(half folds, depth 2): R8 %6.1f (%.2f) W8 %6.1f (%.2f) | 2 waves/SIMD (quarter folds, depth 4): W8 %6.1f (%.2f)\n",
           grid, r1, rd / r1 / 1e6, w1, (rd + wr8) / w1 / 1e6, r2, rd / r2 / 1e6, w2, (rd + wr8) / w2 / 1e6, w3,
           (rd + wr8) / w3 / 1e6);
    fflush(stdout);
  }
  return 0;
}
