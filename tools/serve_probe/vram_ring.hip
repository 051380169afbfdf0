// Probe: where should the persistent scorer's REQUEST ring live?
//   host -- fine-grained pinned host memory (hipHostMalloc coherent): the GPU polls it
//           across PCIe (the current ae_serve.hip design);
//   vram -- fine-grained device memory that the CPU writes through the PCIe BAR
//           (HSA pool allocation + hsa_amd_agents_allow_access for the CPU agent): the
//           host's store is a posted write, the GPU polls its own memory;
//   *_sfence -- the same with a store fence after each host store (the BAR mapping is
//           write-combining: round 3's first probe saw 8.7 ms p50 without it).
// One resident wave echoes each tagged request word into a host-memory result word; the
// host measures store -> echo seen.  Every device spin is bounded (s_memrealtime).
#include <hip/hip_runtime.h>
#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <vector>

#define CK(x)                                                                 \
  do {                                                                        \
    auto e_ = (x);                                                            \
    if (e_ != 0) {                                                            \
      std::fprintf(stderr, "%s failed (%d) at %d\n", #x, (int)e_, __LINE__); \
      return 1;                                                               \
    }                                                                         \
  } while (0)

__global__ void echo_kernel(const uint64_t* req, uint64_t* res, int n, unsigned long long timeout_ticks, int* status) {
  if (threadIdx.x != 0) return;
  for (int i = 0; i < n; ++i) {
    const uint32_t want = (uint32_t)(i + 1);
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    uint64_t v = 0;
    for (;;) {
      asm volatile("global_load_dwordx2 %0, %1, off sc0 sc1\n s_waitcnt vmcnt(0)" : "=v"(v) : "v"(req) : "memory");
      if ((uint32_t)(v >> 32) == want) break;
      if (__builtin_amdgcn_s_memrealtime() - t0 > timeout_ticks) {
        *status = 1;
        return;
      }
    }
    __hip_atomic_store(res, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

struct Pools {
  hsa_agent_t gpu{}, cpu{};
  hsa_amd_memory_pool_t fine{};
  bool have_fine = false;
  int gpu_seen = 0;
};

static hsa_status_t pool_cb(hsa_amd_memory_pool_t pool, void* data) {
  auto* P = static_cast<Pools*>(data);
  hsa_amd_segment_t seg;
  hsa_amd_memory_pool_get_info(pool, HSA_AMD_MEMORY_POOL_INFO_SEGMENT, &seg);
  if (seg != HSA_AMD_SEGMENT_GLOBAL) return HSA_STATUS_SUCCESS;
  uint32_t flags = 0;
  hsa_amd_memory_pool_get_info(pool, HSA_AMD_MEMORY_POOL_INFO_GLOBAL_FLAGS, &flags);
  if ((flags & HSA_AMD_MEMORY_POOL_GLOBAL_FLAG_FINE_GRAINED) && !P->have_fine) {
    P->fine = pool;
    P->have_fine = true;
  }
  return HSA_STATUS_SUCCESS;
}

static hsa_status_t agent_cb(hsa_agent_t a, void* data) {
  auto* P = static_cast<Pools*>(data);
  hsa_device_type_t t;
  hsa_agent_get_info(a, HSA_AGENT_INFO_DEVICE, &t);
  if (t == HSA_DEVICE_TYPE_CPU && P->cpu.handle == 0) P->cpu = a;
  if (t == HSA_DEVICE_TYPE_GPU && P->gpu_seen++ == 0) {
    P->gpu = a;
    hsa_amd_agent_iterate_memory_pools(a, pool_cb, P);
  }
  return HSA_STATUS_SUCCESS;
}

static int run(const char* name, uint64_t* req_host_view, const uint64_t* req_dev_view, uint64_t* res_host,
               uint64_t* res_dev, int* status_d, int n, std::vector<double>& lat, bool fence = false) {
  *reinterpret_cast<volatile uint64_t*>(res_host) = 0;
  *reinterpret_cast<volatile uint64_t*>(req_host_view) = 0;
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  hipLaunchKernelGGL(echo_kernel, dim3(1), dim3(64), 0, s, req_dev_view, res_dev, n, 500000000ull, status_d);
  CK(hipGetLastError());
  lat.clear();
  for (int i = 0; i < n; ++i) {
    const uint64_t w = ((uint64_t)(uint32_t)(i + 1) << 32) | 0x3f800000u;
    auto t0 = std::chrono::steady_clock::now();
    __atomic_store_n(req_host_view, w, __ATOMIC_RELEASE);
    // a BAR mapping is write-combining: without a store fence the word can sit in the
    // core's WC buffer until it is evicted (milliseconds)
    if (fence) __builtin_ia32_sfence();
    uint64_t spins = 0;
    while (__atomic_load_n(res_host, __ATOMIC_ACQUIRE) != w) {
      if (++spins > 2000000000ull) {
        std::fprintf(stderr, "%s: host timeout at %d\n", name, i);
        break;
      }
    }
    auto t1 = std::chrono::steady_clock::now();
    lat.push_back(std::chrono::duration<double, std::micro>(t1 - t0).count());
    auto until = t1 + std::chrono::microseconds(50);
    while (std::chrono::steady_clock::now() < until) {
    }
  }
  CK(hipStreamSynchronize(s));
  CK(hipStreamDestroy(s));
  std::vector<double> v(lat.begin() + 100, lat.end());
  std::sort(v.begin(), v.end());
  std::printf("{\"ring\": \"%s\", \"n\": %zu, \"p50_us\": %.3f, \"p99_us\": %.3f, \"min_us\": %.3f}\n", name, v.size(),
              v[v.size() / 2], v[v.size() * 99 / 100], v[0]);
  return 0;
}

int main(int argc, char** argv) {
  const int n = argc > 1 ? std::atoi(argv[1]) : 5000;
  CK(hipSetDevice(0));
  CK(hipFree(nullptr));
  uint64_t *res_host, *res_dev, *req_h, *req_hd;
  int* status_d;
  CK(hipHostMalloc((void**)&res_host, 4096, hipHostMallocMapped | hipHostMallocCoherent));
  CK(hipHostGetDevicePointer((void**)&res_dev, res_host, 0));
  CK(hipMalloc((void**)&status_d, sizeof(int)));
  CK(hipMemset(status_d, 0, sizeof(int)));
  std::vector<double> lat;
  // host ring
  CK(hipHostMalloc((void**)&req_h, 4096, hipHostMallocMapped | hipHostMallocCoherent));
  CK(hipHostGetDevicePointer((void**)&req_hd, req_h, 0));
  if (run("host", req_h, req_hd, res_host, res_dev, status_d, n, lat)) return 1;
  // VRAM ring through HSA
  CK(hsa_init());
  Pools P;
  CK(hsa_iterate_agents(agent_cb, &P));
  if (!P.have_fine) {
    std::printf("{\"ring\": \"vram\", \"error\": \"no fine-grained VRAM pool\"}\n");
    return 0;
  }
  void* vr = nullptr;
  CK(hsa_amd_memory_pool_allocate(P.fine, 4096, 0, &vr));
  hsa_agent_t agents[2] = {P.gpu, P.cpu};
  const hsa_status_t acc = hsa_amd_agents_allow_access(2, agents, nullptr, vr);
  if (acc != HSA_STATUS_SUCCESS) {
    std::printf("{\"ring\": \"vram\", \"error\": \"allow_access(cpu) = %d\"}\n", (int)acc);
    return 0;
  }
  if (run("vram", (uint64_t*)vr, (const uint64_t*)vr, res_host, res_dev, status_d, n, lat)) return 1;
  if (run("vram_sfence", (uint64_t*)vr, (const uint64_t*)vr, res_host, res_dev, status_d, n, lat, true)) return 1;
  if (run("host_sfence", req_h, req_hd, res_host, res_dev, status_d, n, lat, true)) return 1;
  int st = 0;
  CK(hipMemcpy(&st, status_d, sizeof(int), hipMemcpyDeviceToHost));
  std::printf("{\"device_timeouts\": %d}\n", st);
  hsa_amd_memory_pool_free(vr);
  return 0;
}
