// Device-side helpers shared by the persistent per-event scorers (ae_serve.hip,
// lstm_serve.hip): cache-bypassing system-scope traffic to the host-mapped request /
// result rings (LL framing, sml_ops.h).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace sml {
namespace serve_dev {

// Host-mapped traffic uses RELAXED system-scope atomics: they compile to
// cache-bypassing (sc0 sc1) loads / stores, so polling never invalidates and
// publishing never writes back the whole L2 (which an acquire / release at
// system scope would do on every iteration).  Ordering of the result stores
// before the completion counter is enforced with s_waitcnt vmcnt(0).
__device__ __forceinline__ uint64_t ld_sys(const uint64_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ uint32_t ld_sys32(const uint32_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ void st_sys(uint64_t* p, uint64_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ void st_sys32(uint32_t* p, uint32_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ void wait_stores() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

// One poll: this lane's tagged word of the next request slot and the host's head
// counter, as cache-bypassing loads issued without a wait (the caller waits with a
// counted s_waitcnt tied to the outputs, so several polls can be in flight).
__device__ __forceinline__ void poll_issue(uint64_t& w, uint64_t& hd, const uint64_t* wp, const uint64_t* hp) {
  asm volatile("global_load_dwordx2 %0, %1, off sc0 sc1" : "=v"(w) : "v"(wp) : "memory");
  asm volatile("global_load_dwordx2 %0, %1, off sc0 sc1" : "=v"(hd) : "v"(hp) : "memory");
}

// Two tagged request words (16 bytes) with one cache-bypassing load, issued without a
// wait so a whole row's loads are in flight together (relaxed atomic loads are
// serialised by the compiler: one PCIe round trip per word).  Each 8-byte word is
// checked against its own tag, so the pair need not be read atomically.
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ u32x4 ld_sys_pair_issue(const uint64_t* p) {
  u32x4 v;
  asm volatile("global_load_dwordx4 %0, %1, off sc0 sc1" : "=v"(v) : "v"(p) : "memory");
  return v;
}

__device__ __forceinline__ uint64_t tagged(uint32_t tag, float v) {
  return ((uint64_t)tag << 32) | (uint64_t)__float_as_uint(v);
}
__device__ __forceinline__ uint64_t tagged_u(uint32_t tag, uint32_t v) { return ((uint64_t)tag << 32) | (uint64_t)v; }

}  // namespace serve_dev
}  // namespace sml
