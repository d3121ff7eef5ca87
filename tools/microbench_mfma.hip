// Probes for the integer-MFMA round sums ("Round sums on the
// matrix cores"): run on the box, prints what it finds.
//   1. v_mfma_i32_32x32x32_i8 operand maps: which lane/byte holds A[i][k] and
//      B[k][j] (two hypotheses, checked with random int8 data against the CPU).
//   2. ds_read_b64_tr_b8: which LDS byte lands in which lane/byte (dump).
//   4. v_permlane32_swap: what __builtin_amdgcn_permlane32_swap(x, x) returns.
//   5. k_dm_pattern: the memory side of k_gkr_dm alone (per wave: one table, per
//      64-quad chunk and corner four loads at quarter offsets + one store; xor
//      instead of arithmetic) at the 24-variable first double step (Q = 2^20).
//   6. k_t33_pattern: the memory side of k_gkr_t33 alone (per wave one table; per
//      chunk of 32 octants four folds, each 8 inputs 8 O apart -> one output;
//      xor instead of arithmetic) at the 24-variable first triple step (O = 2^18),
//      by grid size and by blocks per CU.
//   3. k_dot: sum_j A_j * S_j over 256-bit values through signed 8-bit digits,
//      an LDS row image, transposed reads and the i8 MFMA, checked exactly
//      against a CPU big-integer sum, and timed at 2^24 elements per table.
// Build: hipcc -O3 --offload-arch=gfx950 -o tools/mb_mfma tools/microbench_mfma.hip
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define CK(x)                                                                        \
  do {                                                                               \
    hipError_t e_ = (x);                                                             \
    if (e_ != hipSuccess) {                                                          \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));      \
      exit(1);                                                                       \
    }                                                                                \
  } while (0)

typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v16i __attribute__((ext_vector_type(16)));
typedef int v2i __attribute__((ext_vector_type(2)));
typedef __attribute__((address_space(3))) v2i lds_v2i;

// ---- 1. operand-map probe: fragments are built on the host per hypothesis
__global__ void k_mfma_probe(const v4i* a, const v4i* b, v16i* c) {
  int l = threadIdx.x;
  v16i acc = {};
  acc = __builtin_amdgcn_mfma_i32_32x32x32_i8(a[l], b[l], acc, 0, 0, 0);
  c[l] = acc;
}

// ---- 2. transposed-read probe
__global__ void k_tr8_probe(v2i* out, int mode) {
  __shared__ __attribute__((aligned(16))) unsigned char lds[1024];
  int l = threadIdx.x;
  for (int i = l; i < 1024; i += 64) lds[i] = (unsigned char)(i & 0xff);
  __syncthreads();
  int addr = mode == 0 ? 8 * l : 8 * (l ^ 1);
  v2i r = __builtin_amdgcn_ds_read_tr8_b64_v2i32((lds_v2i*)(lds + addr));
  out[l] = r;
}

// ---- 4. permlane32_swap probe
__global__ void k_swap_probe(int* out) {
  const int l = threadIdx.x;
  auto r = __builtin_amdgcn_permlane32_swap(l, l, false, false);
  out[2 * l] = r[0];
  out[2 * l + 1] = r[1];
}

// ---- 5. memory-only k_gkr_dm pattern
__global__ __launch_bounds__(256) void k_dm_pattern(const uint4* const* in, uint4* const* out, size_t Q) {
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  const uint4* X = in[w];
  uint4* X2 = out[w];
  const size_t nch = Q / 64, h4 = 4 * Q;
  for (size_t ch = blockIdx.x; ch < nch; ch += gridDim.x) {
    const size_t j = ch * 64 + l;
    for (int k = 0; k < 4; ++k) {
      const size_t i = j + k * Q;
      uint4 a = X[2 * i], b = X[2 * i + 1];
      for (int q = 1; q < 4; ++q) {
        const uint4 c = X[2 * (i + q * h4)], d = X[2 * (i + q * h4) + 1];
        a.x ^= c.x; a.y ^= c.y; a.z ^= c.z; a.w ^= c.w;
        b.x ^= d.x; b.y ^= d.y; b.z ^= d.z; b.w ^= d.w;
      }
      X2[2 * i] = a;
      X2[2 * i + 1] = b;
    }
  }
}

// ---- 6. memory-only k_gkr_t33 pattern
template <int PF>
__global__ __launch_bounds__(256) void k_t33_pattern(const uint4* const* in, uint4* const* out, size_t O) {
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63, ql = l & 31, hh = l >> 5;
  const uint4* X = in[w];
  uint4* X2 = out[w];
  const size_t nch = O / 32, h8 = 8 * O;
  for (size_t ch = blockIdx.x; ch < nch; ch += gridDim.x) {
    for (int f = 0; f < 4; ++f) {
      const size_t e = ch * 32 + ql + (size_t)(2 * f + hh) * O;
      uint4 a = X[2 * e], b = X[2 * e + 1];
#pragma unroll
      for (int k = 1; k < 8; ++k) {
        const uint4 c = X[2 * (e + k * h8)], d = X[2 * (e + k * h8) + 1];
        a.x ^= c.x; a.y ^= c.y; a.z ^= c.z; a.w ^= c.w;
        b.x ^= d.x; b.y ^= d.y; b.z ^= d.z; b.w ^= d.w;
      }
      X2[2 * e] = a;
      X2[2 * e + 1] = b;
    }
  }
}

// variants of the store: 0 none (reads only; a data-dependent guard keeps the loads), 1 nontemporal
template <int MODE>
__global__ __launch_bounds__(256) void k_t33_pattern_st(const uint4* const* in, uint4* const* out, size_t O) {
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63, ql = l & 31, hh = l >> 5;
  const uint4* X = in[w];
  uint4* X2 = out[w];
  const size_t nch = O / 32, h8 = 8 * O;
  for (size_t ch = blockIdx.x; ch < nch; ch += gridDim.x) {
    for (int f = 0; f < 4; ++f) {
      const size_t e = ch * 32 + ql + (size_t)(2 * f + hh) * O;
      uint4 a = X[2 * e], b = X[2 * e + 1];
#pragma unroll
      for (int k = 1; k < 8; ++k) {
        const uint4 c = X[2 * (e + k * h8)], d = X[2 * (e + k * h8) + 1];
        a.x ^= c.x; a.y ^= c.y; a.z ^= c.z; a.w ^= c.w;
        b.x ^= d.x; b.y ^= d.y; b.z ^= d.z; b.w ^= d.w;
      }
      if (MODE == 0) {
        if ((a.x ^ b.y) == 0x12345678u) X2[2 * e] = a;  // practically never
      } else if (MODE == 2) {
        // lane pairs trade halves so one store instruction covers contiguous 512 B per 32 lanes:
        // even lane l stores the low halves of elements l, l+1, odd lane the high halves
        const bool odd = l & 1;
        uint4 pa, pb;  // partner's a (low half) and b (high half)
        pa.x = __shfl_xor(a.x, 1); pa.y = __shfl_xor(a.y, 1); pa.z = __shfl_xor(a.z, 1); pa.w = __shfl_xor(a.w, 1);
        pb.x = __shfl_xor(b.x, 1); pb.y = __shfl_xor(b.y, 1); pb.z = __shfl_xor(b.z, 1); pb.w = __shfl_xor(b.w, 1);
        const size_t e0 = e & ~(size_t)1;  // the pair's first element
        // store 1: element e0 (both halves, by the two lanes); store 2: element e0 + 1
        X2[2 * e0 + (odd ? 1 : 0)] = odd ? pb : a;       // even: own low half of e0; odd: partner(e0) high half
        X2[2 * (e0 + 1) + (odd ? 1 : 0)] = odd ? b : pa;  // even: partner(e0+1) low; odd: own high of e0+1
      } else {
        typedef unsigned int u4v __attribute__((ext_vector_type(4)));
        const u4v av = {a.x, a.y, a.z, a.w}, bv = {b.x, b.y, b.z, b.w};
        __builtin_nontemporal_store(av, reinterpret_cast<u4v*>(&X2[2 * e]));
        __builtin_nontemporal_store(bv, reinterpret_cast<u4v*>(&X2[2 * e + 1]));
      }
    }
  }
}

// variants of the loads: nontemporal input loads (do not keep the 2 GiB stream in the caches) with
// plain (SMODE 0) or nontemporal (SMODE 1) stores
template <int SMODE>
__global__ __launch_bounds__(256) void k_t33_pattern_ntld(const uint4* const* in, uint4* const* out, size_t O) {
  typedef unsigned int u4v __attribute__((ext_vector_type(4)));
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63, ql = l & 31, hh = l >> 5;
  const u4v* X = reinterpret_cast<const u4v*>(in[w]);
  u4v* X2 = reinterpret_cast<u4v*>(out[w]);
  const size_t nch = O / 32, h8 = 8 * O;
  for (size_t ch = blockIdx.x; ch < nch; ch += gridDim.x) {
    for (int f = 0; f < 4; ++f) {
      const size_t e = ch * 32 + ql + (size_t)(2 * f + hh) * O;
      u4v a = __builtin_nontemporal_load(&X[2 * e]), b = __builtin_nontemporal_load(&X[2 * e + 1]);
#pragma unroll
      for (int k = 1; k < 8; ++k) {
        a ^= __builtin_nontemporal_load(&X[2 * (e + k * h8)]);
        b ^= __builtin_nontemporal_load(&X[2 * (e + k * h8) + 1]);
      }
      if (SMODE == 0) {
        X2[2 * e] = a;
        X2[2 * e + 1] = b;
      } else {
        __builtin_nontemporal_store(a, &X2[2 * e]);
        __builtin_nontemporal_store(b, &X2[2 * e + 1]);
      }
    }
  }
}

// variant: lanes = 64 consecutive octants of one corner (2 KB contiguous per input), 8 folds per chunk
__global__ __launch_bounds__(256) void k_t33_pattern64(const uint4* const* in, uint4* const* out, size_t O) {
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  const uint4* X = in[w];
  uint4* X2 = out[w];
  const size_t nch = O / 64, h8 = 8 * O;
  for (size_t ch = blockIdx.x; ch < nch; ch += gridDim.x) {
    for (int f = 0; f < 8; ++f) {
      const size_t e = ch * 64 + l + (size_t)f * O;
      uint4 a = X[2 * e], b = X[2 * e + 1];
#pragma unroll
      for (int k = 1; k < 8; ++k) {
        const uint4 c = X[2 * (e + k * h8)], d = X[2 * (e + k * h8) + 1];
        a.x ^= c.x; a.y ^= c.y; a.z ^= c.z; a.w ^= c.w;
        b.x ^= d.x; b.y ^= d.y; b.z ^= d.z; b.w ^= d.w;
      }
      X2[2 * e] = a;
      X2[2 * e + 1] = b;
    }
  }
}

// ---- 3. exact dot product through the matrix cores
// signed digits: V < 0.498 * 2^256  =>  V = sum_k (byte_k(V + K) ^ 0x80) * 2^(8k), K = 0x8080...80
__device__ inline void to_digits(uint32_t w[8]) {
  uint64_t c = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    uint64_t s = (uint64_t)w[i] + 0x80808080u + c;
    w[i] = (uint32_t)s ^ 0x80808080u;
    c = s >> 32;
  }
}

// one wave per 32-element chunk: lanes 0-31 element j of A, lanes 32-63 of S.
// LDS image per wave: [2 tables][32 elements][32 bytes]. MFMA A operand: rows =
// byte positions of A, k = element; B operand: k = element, cols = byte of S.
template <int HYP>
__global__ __launch_bounds__(256) void k_dot(const uint32_t* A, const uint32_t* S, size_t n, long long* part) {
  __shared__ __attribute__((aligned(16))) unsigned char img[4][2][32][32];
  __shared__ long long T[63];
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  if (threadIdx.x < 63) T[threadIdx.x] = 0;
  v16i acc = {};
  const size_t chunks = n / 32;
  const int g = l >> 4, i16 = l & 15;
  for (size_t c = (size_t)blockIdx.x * 4 + w; c < chunks; c += (size_t)gridDim.x * 4) {
    const uint32_t* src = (l < 32 ? A : S) + (c * 32 + (l & 31)) * 8;
    uint4 lo = *reinterpret_cast<const uint4*>(src), hi = *reinterpret_cast<const uint4*>(src + 4);
    uint32_t v[8] = {lo.x, lo.y, lo.z, lo.w, hi.x, hi.y, hi.z, hi.w};
    to_digits(v);
    uint4* dst = reinterpret_cast<uint4*>(&img[w][l >> 5][l & 31][0]);
    dst[0] = make_uint4(v[0], v[1], v[2], v[3]);
    dst[1] = make_uint4(v[4], v[5], v[6], v[7]);
    __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0)
    __builtin_amdgcn_wave_barrier();
    // transposed reads (hypothesis: lane 2q+p of a 16-lane group supplies row q,
    // bytes 8p..8p+7 of an 8 x 16 byte block; lane i gets column i)
    v4i fa, fb;
    const int q = i16 >> 1, p = i16 & 1;
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      int elem = 16 * (g >> 1) + 8 * t + q;
      int byte = 16 * (g & 1) + 8 * p;
      v2i ra = __builtin_amdgcn_ds_read_tr8_b64_v2i32((lds_v2i*)&img[w][0][elem][byte]);
      v2i rb = __builtin_amdgcn_ds_read_tr8_b64_v2i32((lds_v2i*)&img[w][1][elem][byte]);
      fa[2 * t] = ra.x; fa[2 * t + 1] = ra.y;
      fb[2 * t] = rb.x; fb[2 * t + 1] = rb.y;
    }
    acc = __builtin_amdgcn_mfma_i32_32x32x32_i8(fa, fb, acc, 0, 0, 0);
    __builtin_amdgcn_wave_barrier();
  }
  __syncthreads();
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    int row = (r & 3) + 8 * (r >> 2) + 4 * (l >> 5), col = l & 31;
    atomicAdd((unsigned long long*)&T[row + col], (unsigned long long)(long long)acc[r]);
  }
  __syncthreads();
  if (threadIdx.x < 63) part[(size_t)blockIdx.x * 63 + threadIdx.x] = T[threadIdx.x];
}

__global__ void k_fill(uint32_t* x, size_t n, uint64_t seed) {
  size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint64_t s = seed ^ (i * 0x9E3779B97F4A7C15ull);
  for (int k = 0; k < 8; ++k) {
    s += 0x9E3779B97F4A7C15ull;
    uint64_t z = s;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    z ^= z >> 31;
    x[i * 8 + k] = (uint32_t)z;
  }
  x[i * 8 + 7] &= 0x3fffffffu;  // < 2^254 (the BN254 range)
}

typedef __int128 i128;
static void normalize(std::vector<i128>& W) {  // signed carry propagation over 32-bit words
  for (size_t i = 0; i + 1 < W.size(); ++i) {
    i128 v = W[i];
    i128 lo = v & 0xffffffff;
    W[i] = lo;
    W[i + 1] += (v - lo) >> 32;
  }
}

int main() {
  // ---- 1
  {
    int8_t A[32][32], B[32][32];
    srand(7);
    for (int i = 0; i < 32; ++i)
      for (int k = 0; k < 32; ++k) A[i][k] = (int8_t)(rand() & 0xff), B[i][k] = (int8_t)(rand() & 0xff);
    int ref[32][32];
    for (int i = 0; i < 32; ++i)
      for (int j = 0; j < 32; ++j) {
        int s = 0;
        for (int k = 0; k < 32; ++k) s += A[i][k] * B[k][j];
        ref[i][j] = s;
      }
    v4i *da, *db;
    v16i* dc;
    CK(hipMalloc(&da, 64 * 16));
    CK(hipMalloc(&db, 64 * 16));
    CK(hipMalloc(&dc, 64 * 64));
    for (int hyp = 0; hyp < 2; ++hyp) {
      int8_t fa[64][16], fb[64][16];
      for (int l = 0; l < 64; ++l)
        for (int j = 0; j < 16; ++j) {
          int k = hyp == 0 ? 16 * (l >> 5) + j : 8 * (l >> 5) + (j & 7) + 16 * (j >> 3);
          fa[l][j] = A[l & 31][k];
          fb[l][j] = B[k][l & 31];
        }
      CK(hipMemcpy(da, fa, sizeof fa, hipMemcpyHostToDevice));
      CK(hipMemcpy(db, fb, sizeof fb, hipMemcpyHostToDevice));
      k_mfma_probe<<<1, 64>>>(da, db, dc);
      int out[64][16];
      CK(hipMemcpy(out, dc, sizeof out, hipMemcpyDeviceToHost));
      int bad = 0;
      for (int l = 0; l < 64; ++l)
        for (int r = 0; r < 16; ++r) {
          int row = (r & 3) + 8 * (r >> 2) + 4 * (l >> 5), col = l & 31;
          bad += out[l][r] != ref[row][col];
        }
      printf("mfma_i32_32x32x32_i8 operand map H%d (%s): %d of 1024 outputs wrong\n", hyp,
             hyp == 0 ? "lane l: k = 16(l>>5)+j" : "lane l: k = 8(l>>5)+(j&7)+16(j>>3)", bad);
    }
  }
  // ---- 2
  {
    v2i* d;
    CK(hipMalloc(&d, 64 * 8));
    for (int mode = 0; mode < 2; ++mode) {
      k_tr8_probe<<<1, 64>>>(d, mode);
      unsigned char h[64][8];
      CK(hipMemcpy(h, d, sizeof h, hipMemcpyDeviceToHost));
      printf("ds_read_b64_tr_b8, lane l address = %s: lane: 8 bytes (LDS byte offsets)\n",
             mode == 0 ? "8*l" : "8*(l^1)");
      for (int l = 0; l < 64; ++l) {
        printf("  %2d:", l);
        for (int b = 0; b < 8; ++b) printf(" %3d", h[l][b]);
        printf("%s", (l & 3) == 3 ? "\n" : " |");
      }
    }
  }
  // ---- 4
  {
    int* d;
    CK(hipMalloc(&d, 128 * 4));
    k_swap_probe<<<1, 64>>>(d);
    int h[128];
    CK(hipMemcpy(h, d, sizeof h, hipMemcpyDeviceToHost));
    int ok = 1;
    for (int l = 0; l < 64; ++l) {
      const int partner = l ^ 32, want0 = l < 32 ? l : partner, want1 = l < 32 ? partner : l;
      ok &= h[2 * l] == want0 && h[2 * l + 1] == want1;
    }
    printf("permlane32_swap(x, x) = {lanes<32: own, else partner ; lanes<32: partner, else own}: %s (lane 0: %d %d, lane 40: %d %d)\n",
           ok ? "yes" : "NO", h[0], h[1], h[80], h[81]);
  }
  // ---- 3
  {
    const size_t n = (size_t)1 << 24;
    uint32_t *A, *S;
    CK(hipMalloc(&A, n * 32));
    CK(hipMalloc(&S, n * 32));
    k_fill<<<(n + 255) / 256, 256>>>(A, n, 11);
    k_fill<<<(n + 255) / 256, 256>>>(S, n, 22);
    const int blocks = 2048;
    long long* part;
    CK(hipMalloc(&part, blocks * 63 * 8));
    // exactness at 2^16 elements
    const size_t ns = 1 << 16;
    k_dot<0><<<blocks, 256>>>(A, S, ns, part);
    CK(hipDeviceSynchronize());
    std::vector<long long> hp(blocks * 63);
    CK(hipMemcpy(hp.data(), part, hp.size() * 8, hipMemcpyDeviceToHost));
    std::vector<i128> got(20, 0), want(20, 0);
    for (int b = 0; b < blocks; ++b)
      for (int d = 0; d < 63; ++d) got[d / 4] += (i128)hp[b * 63 + d] << (8 * (d % 4));
    std::vector<uint32_t> ha(ns * 8), hs(ns * 8);
    CK(hipMemcpy(ha.data(), A, ns * 32, hipMemcpyDeviceToHost));
    CK(hipMemcpy(hs.data(), S, ns * 32, hipMemcpyDeviceToHost));
    for (size_t j = 0; j < ns; ++j)
      for (int a = 0; a < 8; ++a)
        for (int b = 0; b < 8; ++b) want[a + b] += (i128)((uint64_t)ha[j * 8 + a] * hs[j * 8 + b]);
    normalize(got);
    normalize(want);
    int ok = got == want;
    printf("k_dot exact sum of 2^16 products (tr_b8 hypothesis): %s\n", ok ? "MATCH" : "MISMATCH");
    // timing at 2^24 elements per table (1 GiB read)
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (int it = 0; it < 3; ++it) k_dot<0><<<blocks, 256>>>(A, S, n, part);
    CK(hipEventRecord(e0));
    const int iters = 10;
    for (int it = 0; it < iters; ++it) k_dot<0><<<blocks, 256>>>(A, S, n, part);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    ms /= iters;
    printf("k_dot 2^24 x 2 tables: %.1f us, %.2f TB/s\n", ms * 1e3, n * 64.0 / (ms * 1e-3) / 1e12);
  }
  // ---- 5
  {
    const size_t Q = (size_t)1 << 20;
    uint4 *hin[4], *hout[4];
    for (int t = 0; t < 4; ++t) {
      CK(hipMalloc(&hin[t], 16 * Q * 32));
      CK(hipMalloc(&hout[t], 4 * Q * 32));
      CK(hipMemset(hin[t], t + 1, 16 * Q * 32));
    }
    const uint4** din;
    uint4** dout;
    CK(hipMalloc(&din, sizeof hin));
    CK(hipMalloc(&dout, sizeof hout));
    CK(hipMemcpy(din, hin, sizeof hin, hipMemcpyHostToDevice));
    CK(hipMemcpy(dout, hout, sizeof hout, hipMemcpyHostToDevice));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (int grid : {512, 768, 1024, 2048}) {
      for (int it = 0; it < 2; ++it) k_dm_pattern<<<grid, 256>>>(din, dout, Q);
      CK(hipEventRecord(e0));
      for (int it = 0; it < 5; ++it) k_dm_pattern<<<grid, 256>>>(din, dout, Q);
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      ms /= 5;
      const double bytes = 4.0 * (16 * Q + 4 * Q) * 32;
      printf("k_dm_pattern Q=2^20 grid %d: %.1f us, %.2f TB/s (%.2f GB)\n", grid, ms * 1e3, bytes / (ms * 1e-3) / 1e12, bytes / 1e9);
    }
  }
  // ---- 6
  {
    const size_t O = (size_t)1 << 18;
    uint4 *hin[4], *hout[4];
    for (int t = 0; t < 4; ++t) {
      CK(hipMalloc(&hin[t], 64 * O * 32));
      CK(hipMalloc(&hout[t], 8 * O * 32));
      CK(hipMemset(hin[t], t + 1, 64 * O * 32));
    }
    const uint4** din;
    uint4** dout;
    CK(hipMalloc(&din, sizeof hin));
    CK(hipMalloc(&dout, sizeof hout));
    CK(hipMemcpy(din, hin, sizeof hin, hipMemcpyHostToDevice));
    CK(hipMemcpy(dout, hout, sizeof hout, hipMemcpyHostToDevice));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (int grid : {256, 512, 1024, 2048}) {
      for (int it = 0; it < 2; ++it) k_t33_pattern<0><<<grid, 256>>>(din, dout, O);
      CK(hipEventRecord(e0));
      for (int it = 0; it < 5; ++it) k_t33_pattern<0><<<grid, 256>>>(din, dout, O);
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      ms /= 5;
      const double bytes = 4.0 * (64 * O + 8 * O) * 32;
      printf("k_t33_pattern O=2^18 grid %d: %.1f us, %.2f TB/s (%.2f GB)\n", grid, ms * 1e3, bytes / (ms * 1e-3) / 1e12, bytes / 1e9);
    }
    for (int grid : {256, 512, 1024}) {
      for (int it = 0; it < 2; ++it) k_t33_pattern64<<<grid, 256>>>(din, dout, O);
      CK(hipEventRecord(e0));
      for (int it = 0; it < 5; ++it) k_t33_pattern64<<<grid, 256>>>(din, dout, O);
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      ms /= 5;
      const double bytes = 4.0 * (64 * O + 8 * O) * 32;
      printf("k_t33_pattern64 (64 octants x one corner per fold) grid %d: %.1f us, %.2f TB/s\n", grid, ms * 1e3, bytes / (ms * 1e-3) / 1e12);
    }
    for (int mode = 0; mode < 3; ++mode) {
      const int grid = 512;
      auto run = [&] {
        if (mode == 0) k_t33_pattern_st<0><<<grid, 256>>>(din, dout, O);
        else if (mode == 1) k_t33_pattern_st<1><<<grid, 256>>>(din, dout, O);
        else k_t33_pattern_st<2><<<grid, 256>>>(din, dout, O);
      };
      for (int it = 0; it < 2; ++it) run();
      CK(hipEventRecord(e0));
      for (int it = 0; it < 5; ++it) run();
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      ms /= 5;
      const double rb = 4.0 * 64 * O * 32, wb = mode ? 4.0 * 8 * O * 32 : 0.0;
      printf("k_t33_pattern %s grid %d: %.1f us, %.2f TB/s (%.2f GB)\n",
             mode == 0 ? "reads only" : (mode == 1 ? "nontemporal stores" : "paired-lane contiguous stores"),
             grid, ms * 1e3, (rb + wb) / (ms * 1e-3) / 1e12, (rb + wb) / 1e9);
    }
    for (int mode = 0; mode < 2; ++mode) {
      const int grid = 512;
      auto run = [&] {
        if (mode == 0) k_t33_pattern_ntld<0><<<grid, 256>>>(din, dout, O);
        else k_t33_pattern_ntld<1><<<grid, 256>>>(din, dout, O);
      };
      for (int it = 0; it < 2; ++it) run();
      CK(hipEventRecord(e0));
      for (int it = 0; it < 5; ++it) run();
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      ms /= 5;
      const double bytes = 4.0 * (64 * O + 8 * O) * 32;
      printf("k_t33_pattern nontemporal loads, %s stores grid %d: %.1f us, %.2f TB/s\n", mode ? "nontemporal" : "plain",
             grid, ms * 1e3, bytes / (ms * 1e-3) / 1e12);
    }
    for (int t = 0; t < 4; ++t) {
      CK(hipFree(hin[t]));
      CK(hipFree(hout[t]));
    }
  }
  return 0;
}
