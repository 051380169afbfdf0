// Probe: host -> GPU -> host ping-pong latency of a persistent polling wave, with the
// request mailbox in (a) pinned host memory (GPU polls across PCIe) or (b) fine-grained
// device memory written by the host through the BAR (GPU polls its own memory).
// The reply always goes to pinned host memory.  Bounded spins everywhere.
// Build: hipcc --offload-arch=gfx950 -O2 tools/mailbox_probe.hip -o /tmp/mailbox_probe
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                  \
  do {                                                                         \
    hipError_t e_ = (x);                                                       \
    if (e_ != hipSuccess) {                                                    \
      std::printf("%s failed: %s\n", #x, hipGetErrorString(e_));              \
      std::exit(1);                                                            \
    }                                                                          \
  } while (0)

__global__ void pong(const unsigned long long* req, unsigned long long* rep, int n, long long timeout_ticks) {
  if (threadIdx.x != 0) return;
  const long long t0 = (long long)__builtin_amdgcn_s_memrealtime();
  for (int i = 1; i <= n; ++i) {
    unsigned long long v = 0;
    for (;;) {
      v = __hip_atomic_load(req, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      if (v >= (unsigned long long)i) break;
      if ((long long)__builtin_amdgcn_s_memrealtime() - t0 > timeout_ticks) return;   // bounded
    }
    __hip_atomic_store(rep, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

static double run(unsigned long long* req_host_view, unsigned long long* req_dev_view, bool wc_fence, int n) {
  unsigned long long* rep;
  CK(hipHostMalloc((void**)&rep, 64, hipHostMallocMapped | hipHostMallocCoherent));
  *rep = 0;
  __atomic_store_n(req_host_view, 0ull, __ATOMIC_SEQ_CST);
  unsigned long long* rep_d;
  CK(hipHostGetDevicePointer((void**)&rep_d, rep, 0));
  hipLaunchKernelGGL(pong, dim3(1), dim3(64), 0, 0, req_dev_view, rep_d, n, 100000000LL * 20);   // 20 s cap
  CK(hipGetLastError());
  std::vector<double> lat;
  for (int i = 1; i <= n; ++i) {
    const auto t0 = std::chrono::steady_clock::now();
    __atomic_store_n(req_host_view, (unsigned long long)i, __ATOMIC_RELAXED);
    if (wc_fence) __builtin_ia32_sfence();
    long spins = 0;
    while (__atomic_load_n(rep, __ATOMIC_ACQUIRE) < (unsigned long long)i) {
      if (++spins > 2000000000L) {
        std::printf("timeout at %d\n", i);
        std::exit(2);
      }
    }
    const auto t1 = std::chrono::steady_clock::now();
    lat.push_back(std::chrono::duration<double, std::micro>(t1 - t0).count());
    const auto t2 = std::chrono::steady_clock::now();
    while (std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t2).count() < 20.0) {
    }
  }
  CK(hipDeviceSynchronize());
  CK(hipHostFree(rep));
  std::sort(lat.begin() + 100, lat.end());
  const size_t m = lat.size() - 100;
  std::printf("  p50 %.2f us  p10 %.2f  p90 %.2f  p99 %.2f\n", lat[100 + m / 2], lat[100 + m / 10],
              lat[100 + m * 9 / 10], lat[100 + m * 99 / 100]);
  return lat[100 + m / 2];
}

int main() {
  const int n = 5000;
  // (a) pinned host mailbox
  unsigned long long* hreq;
  CK(hipHostMalloc((void**)&hreq, 64, hipHostMallocMapped | hipHostMallocCoherent));
  unsigned long long* hreq_d;
  CK(hipHostGetDevicePointer((void**)&hreq_d, hreq, 0));
  std::printf("host-memory mailbox (GPU polls over PCIe):\n");
  run(hreq, hreq_d, false, n);
  // (b) device mailbox, host writes through the BAR
  for (unsigned flag : {(unsigned)hipDeviceMallocFinegrained, (unsigned)hipDeviceMallocUncached}) {
    void* dreq = nullptr;
    hipError_t e = hipExtMallocWithFlags(&dreq, 4096, flag);
    if (e != hipSuccess) {
      std::printf("flag %u: alloc failed: %s\n", flag, hipGetErrorString(e));
      continue;
    }
    hipPointerAttribute_t at{};
    CK(hipPointerGetAttributes(&at, dreq));
    std::printf("device mailbox flag %u: type %d hostPointer %p devicePointer %p\n", flag, (int)at.type,
                at.hostPointer, at.devicePointer);
    unsigned long long* hv = (unsigned long long*)(at.hostPointer ? at.hostPointer : dreq);
    // host access check: write, read back through a device copy
    __atomic_store_n(hv, 0x1234ull, __ATOMIC_SEQ_CST);
    __builtin_ia32_sfence();
    unsigned long long back = 0;
    CK(hipMemcpy(&back, dreq, 8, hipMemcpyDeviceToHost));
    std::printf("  host write visible to device copy: %s\n", back == 0x1234ull ? "yes" : "NO");
    if (back != 0x1234ull) continue;
    run(hv, (unsigned long long*)dreq, true, n);
    CK(hipFree(dreq));
  }
  std::printf("done\n");
  return 0;
}
