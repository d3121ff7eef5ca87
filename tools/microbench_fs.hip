// Device Fiat-Shamir step (csrc/fs.hpp) on gfx950: correctness of the
// wave-cooperative Keccak-f against the host permutation and of a chain of
// FS steps against a host restatement (byte-wise sponge, INV2 multiply),
// plus their single-wave latencies.
// hipcc -O3 --offload-arch=gfx950 tools/microbench_fs.hip -o tools/mb_fs
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <string.h>

#include "../zk-research-implementations_amd/csrc/fs.hpp"
#include "../zk-research-implementations_amd/csrc/keccak.hpp"

using namespace zk;
using F = Bn254Fr;
#define CK(x) do { hipError_t ck_ = (x); if (ck_ != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(ck_), __LINE__); return 1; } } while (0)

__global__ void k_perm(uint64_t* st, int iters, unsigned long long* cyc) {
  __shared__ uint64_t lds[96];
  const uint32_t lane = threadIdx.x;
  uint64_t a = lane < 25 ? st[lane] : 0;
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < iters; ++i) a = keccak_f_lanes(a, lane, lds, lds + 32);
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  if (lane < 25) st[lane] = a;
  if (lane == 0) cyc[0] = t1 - t0;
}

// chain: step k consumes e[2k], e[2k+1] and recs[k], writes recs[k+1]
__global__ void k_chain(const Fe* e, FsRec* recs, int n, uint32_t mode, unsigned long long* cyc) {
  __shared__ uint64_t lds[96];
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int k = 0; k < n; ++k) {
    Fe ek[2] = {e[2 * k], e[2 * k + 1]};
    fs_step_wave<F>(mode, ek, false, recs + k, recs + k + 1, lds);
    __builtin_amdgcn_s_waitcnt(0);
    __threadfence_block();
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) cyc[0] = t1 - t0;
}

static uint64_t sm = 0x1234567;
static uint32_t rnd32() { sm += 0x9e3779b97f4a7c15ull; uint64_t z = sm; z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull; z = (z ^ (z >> 27)) * 0x94d049bb133111ebull; return (uint32_t)(z ^ (z >> 31)); }
static Fe rnd_fe() { Fe x; for (int i = 0; i < 8; ++i) x.v[i] = rnd32(); x.v[7] &= 0x0fffffff; return fe_reduce_once<F>(x); }

static void host_step(uint32_t mode, const Fe* e, const FsRec& prev, FsRec& out) {
  Keccak256 h;
  uint8_t d[32];
  memcpy(d, prev.digest, 32);
  h.update(d, 32);
  Fe c[3] = {e[0], e[1], fe_zero<F>()};
  int m = 2;
  if (mode == FS_GKR) {
    const Fe e0 = e[0], e2 = e[1], e1 = fe_sub<F>(prev.claim, e0);
    c[0] = e0;
    c[2] = fe_mul<F>(fe_add<F>(fe_sub<F>(e0, fe_dbl<F>(e1)), e2), fe_inv2<F>());
    c[1] = fe_sub<F>(fe_sub<F>(e1, e0), c[2]);
    m = 3;
    while (m > 0 && fe_is_zero<F>(c[m - 1])) --m;
  }
  for (int i = 0; i < m; ++i) { Fe cc = fe_from_mont<F>(c[i]); h.update(reinterpret_cast<uint8_t*>(cc.v), 32); }
  h.finalize_reset(d);
  Fe r; memcpy(r.v, d, 32);
  for (int i = 0; i < 5; ++i) r = fe_reduce_once<F>(r);
  memset(&out, 0, sizeof out);
  out.r = fe_to_mont<F>(r);
  out.claim = mode == FS_GKR ? fe_add<F>(c[0], fe_mul<F>(out.r, fe_add<F>(c[1], fe_mul<F>(out.r, c[2])))) : fe_zero<F>();
  memcpy(out.digest, d, 32);
  for (int i = 0; i < 3; ++i) out.coeff[i] = i < m ? c[i] : fe_zero<F>();
  out.ncoeff = m;
}

int main() {
  int bad = 0;
  // 1) permutation
  uint64_t h[25], ref[25];
  for (int i = 0; i < 25; ++i) ref[i] = h[i] = ((uint64_t)rnd32() << 32) | rnd32();
  const int iters = 200;
  for (int k = 0; k < iters; ++k) Keccak256::permute(ref);
  uint64_t* d; unsigned long long* dc; unsigned long long cyc;
  CK(hipMalloc(&d, 200)); CK(hipMalloc(&dc, 8));
  CK(hipMemcpy(d, h, 200, hipMemcpyHostToDevice));
  k_perm<<<1, 64>>>(d, iters, dc);
  CK(hipDeviceSynchronize());
  CK(hipMemcpy(h, d, 200, hipMemcpyDeviceToHost)); CK(hipMemcpy(&cyc, dc, 8, hipMemcpyDeviceToHost));
  const bool pok = !memcmp(h, ref, 200);
  bad |= !pok;
  printf("lane keccak-f: %s, %.0f s_memtime ticks per permutation\n", pok ? "matches host" : "MISMATCH", cyc / (double)iters);
  // 2) chained FS steps, both modes; zero coefficients exercised too
  for (uint32_t mode = 0; mode < 2; ++mode) {
    const int n = 64;
    Fe e[2 * n];
    for (int i = 0; i < 2 * n; ++i) e[i] = rnd_fe();
    FsRec hr[n + 1];
    memset(hr, 0, sizeof hr);
    hr[0].claim = rnd_fe();
    for (int i = 0; i < 8; ++i) hr[0].digest[i] = rnd32();
    e[2 * 5] = e[2 * 5 + 1] = fe_zero<F>();  // mode 0: c = (0, claim', ...) variants
    for (int k = 0; k < n; ++k) {
      if (mode == 0 && k == 9) { e[2 * k] = hr[k].claim; e[2 * k + 1] = hr[k].claim; }  // e1 = 0 -> c2 = 0? exercises trims
      host_step(mode, e + 2 * k, hr[k], hr[k + 1]);
    }
    Fe* de; FsRec* dr;
    CK(hipMalloc(&de, sizeof e)); CK(hipMalloc(&dr, sizeof hr));
    CK(hipMemcpy(de, e, sizeof e, hipMemcpyHostToDevice));
    CK(hipMemcpy(dr, hr, sizeof(FsRec), hipMemcpyHostToDevice));
    k_chain<<<1, 64>>>(de, dr, n, mode, dc);
    CK(hipDeviceSynchronize());
    FsRec got[n + 1];
    CK(hipMemcpy(got, dr, sizeof got, hipMemcpyDeviceToHost)); CK(hipMemcpy(&cyc, dc, 8, hipMemcpyDeviceToHost));
    int mism = 0, trims = 0;
    for (int k = 1; k <= n; ++k) {
      trims += hr[k].ncoeff < 3;
      if (memcmp(&got[k], &hr[k], offsetof(FsRec, ncoeff) + 4)) { if (!mism) printf("  first mismatch at step %d\n", k); ++mism; }
    }
    bad |= mism != 0;
    printf("fs step mode %u: %s (%d steps, %d trimmed), %.0f s_memtime ticks per step\n", mode,
           mism ? "MISMATCH" : "matches host", n, trims, cyc / (double)n);
  }
  return bad;
}
