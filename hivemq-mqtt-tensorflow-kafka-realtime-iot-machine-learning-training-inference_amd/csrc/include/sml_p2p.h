// Device side of the peer-to-peer granule exchange (runtime/p2p.h).
//
// A granule is one naturally aligned 8-byte word {tag (high 32 bits), fp32 value (low 32)}
// written by ONE system-scope store: the value is its own flag, so a poll that sees the
// current tag also sees the value (no fence, no separate flag write).  The receive
// buffers are uncached (hipDeviceMallocUncached), so a peer's posted xGMI write becomes
// visible to the local poll without cache maintenance.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace sml {

// tags: 1-based counters folded into 30 bits (0 = never written); the persistent trainer
// tags by optimizer iteration, the host-callable all-reduce by call count with the top
// bit set, so the two uses of one exchange can never accept each other's granules
inline constexpr uint32_t p2p_tag(int64_t epoch) { return (uint32_t)(epoch & 0x3fffffff) + 1u; }
inline constexpr uint32_t p2p_call_tag(int64_t call) { return 0x80000000u | p2p_tag(call); }

#if defined(__HIPCC__)
// granule index in a receive buffer: [parity][source rank][slot]
__device__ __forceinline__ int64_t p2p_index(int parity, int src, int world, int64_t slots, int64_t slot) {
  return ((int64_t)parity * world + src) * slots + slot;
}

__device__ __forceinline__ void p2p_put(uint64_t* g, uint32_t tag, float v) {
  const uint64_t w = ((uint64_t)tag << 32) | (uint64_t)__float_as_uint(v);
  __hip_atomic_store(g, w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// one poll; true (and the value) once the granule carries `tag`
__device__ __forceinline__ bool p2p_try(const uint64_t* g, uint32_t tag, float& v) {
  const uint64_t w = __hip_atomic_load(const_cast<uint64_t*>(g), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  v = __uint_as_float((uint32_t)w);
  return (uint32_t)(w >> 32) == tag;
}

#endif  // __HIPCC__

}  // namespace sml
