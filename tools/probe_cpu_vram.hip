// Can the host CPU store into fine-grained device memory (so a kernel can poll
// its own HBM instead of reading pinned host memory over PCIe)? Each probe runs
// in a forked child: a CPU fault only ends that child.
// hipcc -O3 --offload-arch=gfx950 tools/probe_cpu_vram.hip -o tools/mb_probe
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <sys/wait.h>
#include <unistd.h>
#include <chrono>

__global__ void k_wait(volatile uint32_t* p, uint32_t want, unsigned long long* out) {
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  while (__hip_atomic_load((uint32_t*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != want)
    if (__builtin_amdgcn_s_memrealtime() - t0 > 100000000ull) break;  // 1 s exit
  out[0] = __builtin_amdgcn_s_memrealtime();
}

static int probe(const char* name, unsigned flags) {
  pid_t pid = fork();
  if (pid == 0) {
    uint32_t* p = nullptr;
    if (hipExtMallocWithFlags((void**)&p, 4096, flags) != hipSuccess) { printf("%-12s alloc failed\n", name); fflush(stdout); _exit(2); }
    unsigned long long* out;
    (void)hipHostMalloc((void**)&out, 64, hipHostMallocMapped | hipHostMallocCoherent);
    (void)hipMemset(p, 0, 4096);
    (void)hipDeviceSynchronize();
    *(volatile uint32_t*)p = 5;  // CPU store into VRAM (faults here if unmapped)
    __atomic_thread_fence(__ATOMIC_SEQ_CST);
    uint32_t back = 0;
    (void)hipMemcpy(&back, p, 4, hipMemcpyDeviceToHost);
    // latency: kernel spins on p; host stores 7 after a delay
    out[0] = 0;
    k_wait<<<1, 64>>>(p, 7, out);
    usleep(20000);
    const auto t0 = std::chrono::steady_clock::now();
    *(volatile uint32_t*)p = 7;
    __builtin_ia32_sfence();  // drain the write-combining buffer of the BAR mapping
    while (__atomic_load_n(&out[0], __ATOMIC_ACQUIRE) == 0) {
      if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(2)) break;
    }
    const double us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
    (void)hipDeviceSynchronize();
    printf("%-12s cpu store ok, readback %u, store->kernel saw->host saw %.2f us\n", name, back, us);
    fflush(stdout);
    _exit(0);
  }
  int st = 0;
  waitpid(pid, &st, 0);
  if (WIFSIGNALED(st)) printf("%-12s child died with signal %d (no CPU mapping)\n", name, WTERMSIG(st));
  return 0;
}

int main() {
  setvbuf(stdout, nullptr, _IONBF, 0);
  probe("finegrained", hipDeviceMallocFinegrained);
  probe("uncached", hipDeviceMallocUncached);
  // reference: pinned host memory polled by the kernel
  pid_t pid = fork();
  if (pid == 0) {
    uint32_t* p; unsigned long long* out;
    (void)hipHostMalloc((void**)&p, 4096, hipHostMallocMapped | hipHostMallocCoherent);
    (void)hipHostMalloc((void**)&out, 64, hipHostMallocMapped | hipHostMallocCoherent);
    *p = 0; out[0] = 0;
    k_wait<<<1, 64>>>(p, 7, out);
    usleep(20000);
    const auto t0 = std::chrono::steady_clock::now();
    __atomic_store_n(p, 7u, __ATOMIC_RELEASE);
    while (__atomic_load_n(&out[0], __ATOMIC_ACQUIRE) == 0)
      if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(2)) break;
    const double us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
    (void)hipDeviceSynchronize();
    printf("%-12s store->kernel saw->host saw %.2f us\n", "pinned-host", us);
    fflush(stdout);
    _exit(0);
  }
  int st; waitpid(pid, &st, 0);
  return 0;
}
