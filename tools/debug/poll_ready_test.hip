// Standalone check of sml_serve_dev.h poll_ready on the GPU: the host publishes tagged
// words (LL framing) into host-mapped memory one event at a time; one wave polls with
// poll_ready and echoes (status, word, head) per event into a host-mapped result array.
// Every device wait is bounded (rounds + s_memrealtime timeout).
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstring>
#include <thread>

#include "sml_serve_dev.h"

using namespace sml::serve_dev;

struct Out {
  uint32_t st[64];
  uint64_t w[64][2];
  uint64_t hd[64];
};

__global__ void poll_kernel(const uint64_t* req, const uint64_t* head, Out* out, int nev, int D, uint64_t timeout) {
  const int lane = threadIdx.x;
  const uint64_t dontcare = ~((1ull << D) - 1ull);
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  for (int e = 0; e < nev; ++e) {
    const uint32_t want = (uint32_t)(e + 1);
    const uint64_t* wp = req + (size_t)e * 32 + (lane & 31);
    uint64_t w = 0, hd = 0;
    uint32_t st = 0;
    for (;;) {
      st = poll_ready(wp, head, want, (uint64_t)e + 4, dontcare, 64, w, hd);
      if (st != 0) break;
      if (__builtin_amdgcn_s_memrealtime() - t0 > timeout) break;
    }
    if (lane == 0) {
      out->st[e] = st;
      out->hd[e] = hd;
    }
    if (lane < 2) out->w[e][lane] = w;
    if (st == 0) return;
  }
}

int main() {
  const int nev = 8, D = 18;
  uint64_t *req, *head, *req_d, *head_d;
  Out *out, *out_d;
  hipHostMalloc((void**)&req, nev * 32 * 8, hipHostMallocMapped | hipHostMallocCoherent);
  hipHostMalloc((void**)&head, 8, hipHostMallocMapped | hipHostMallocCoherent);
  hipHostMalloc((void**)&out, sizeof(Out), hipHostMallocMapped | hipHostMallocCoherent);
  std::memset(req, 0, nev * 32 * 8);
  std::memset(out, 0, sizeof(Out));
  *head = 0;
  hipHostGetDevicePointer((void**)&req_d, req, 0);
  hipHostGetDevicePointer((void**)&head_d, head, 0);
  hipHostGetDevicePointer((void**)&out_d, out, 0);
  hipLaunchKernelGGL(poll_kernel, dim3(1), dim3(64), 0, 0, req_d, head_d, out_d, nev, D, 300000000ull);
  for (int e = 0; e < nev; ++e) {
    std::this_thread::sleep_for(std::chrono::milliseconds(20));
    for (int j = 0; j < D; ++j)
      __atomic_store_n(&req[e * 32 + j], ((uint64_t)(e + 1) << 32) | (uint64_t)(1000 * e + j), __ATOMIC_RELEASE);
    __atomic_store_n(head, (uint64_t)(e + 1), __ATOMIC_RELEASE);
  }
  hipDeviceSynchronize();
  int bad = 0;
  for (int e = 0; e < nev; ++e) {
    const uint64_t w0 = out->w[e][0], w1 = out->w[e][1];
    const bool ok = out->st[e] == 1 && w0 == (((uint64_t)(e + 1) << 32) | (uint64_t)(1000 * e)) &&
                    w1 == (((uint64_t)(e + 1) << 32) | (uint64_t)(1000 * e + 1));
    bad += !ok;
    std::printf("event %d: st=%u w0=%016llx w1=%016llx head=%llu %s\n", e, out->st[e], (unsigned long long)w0,
                (unsigned long long)w1, (unsigned long long)out->hd[e], ok ? "ok" : "BAD");
  }
  std::printf("%s\n", bad ? "FAIL" : "PASS");
  return bad ? 1 : 0;
}
