// Host-callable small all-reduce over the peer-to-peer granule exchange (runtime/p2p.h).
//
// For buckets of a few KB (the autoencoder's 1536-float padded gradient image + metrics)
// an RCCL ring all-reduce is latency-bound (~10-30 us per call).  This is one
// launch per call: every thread publishes its elements as {tag, value} granules into its
// slot of every peer's receive buffer (one posted xGMI write each, all links at once),
// polls the matching granules of its own buffer, and sums the world's values in rank
// order (identical on every rank: bit-identical replicas).  Spins are bounded by a
// wall-clock timeout (s_memrealtime, 100 MHz); a timed-out poll sets *status and exits.
#include "sml_common.h"
#include "sml_p2p.h"

#include "../runtime/p2p.h"

namespace {

constexpr int kThreads = 256;

__global__ __launch_bounds__(kThreads) void p2p_allreduce_kernel(float* __restrict__ x, int64_t n,
                                                                 uint64_t* const* __restrict__ peers, int world,
                                                                 int rank, int64_t slots, uint32_t tag, int parity,
                                                                 int* status, long long timeout_ticks) {
  const int64_t stride = (int64_t)gridDim.x * kThreads;
  const long long t0 = (long long)__builtin_amdgcn_s_memrealtime();
  for (int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x; i < n; i += stride) {
    const float mine = x[i];
    for (int r = 0; r < world; ++r)
      if (r != rank) sml::p2p_put(peers[r] + sml::p2p_index(parity, rank, world, slots, i), tag, mine);
    const uint64_t* own = peers[rank];
    float acc = 0.f;
    bool failed = false;
    for (int r = 0; r < world; ++r) {   // rank order: the same float sum on every rank
      float v = mine;
      if (r != rank) {
        const uint64_t* g = own + sml::p2p_index(parity, r, world, slots, i);
        while (!sml::p2p_try(g, tag, v)) {
          __builtin_amdgcn_s_sleep(1);
          if ((long long)__builtin_amdgcn_s_memrealtime() - t0 > timeout_ticks) {
            failed = true;
            break;
          }
        }
      }
      acc += v;
      if (failed) break;
    }
    if (failed) {
      __hip_atomic_store(status, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      return;
    }
    x[i] = acc;
  }
}

}  // namespace

namespace sml {

hipError_t p2p_allreduce_launch(float* x, int64_t n, uint64_t** peers, int world, int rank, int64_t slots,
                                uint32_t tag, int parity, int* status, long long timeout_ticks, hipStream_t stream) {
  if (n < 0 || n > slots || world < 1 || rank < 0 || rank >= world || (parity != 0 && parity != 1))
    return hipErrorInvalidValue;
  if (n == 0) return hipSuccess;
  const int64_t blocks = (n + kThreads - 1) / kThreads;
  const int grid = (int)(blocks < 64 ? blocks : 64);
  hipLaunchKernelGGL(p2p_allreduce_kernel, dim3(grid), dim3(kThreads), 0, stream, x, n, peers, world, rank,
                     slots, tag, parity, status, timeout_ticks);
  return hipGetLastError();
}

}  // namespace sml
