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

// One request slot's first 32 tagged words (16 x 16-byte cache-bypassing loads from one
// base address) in ONE asm statement that also waits for them: no loaded register is
// visible to compiler code before its data landed.  Each 8-byte word is checked against
// its own tag by the caller, so the 16-byte loads need not be atomic.
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ void ld_sys_row32(const uint64_t* p, u32x4 (&q)[16]) {
  asm volatile(
      "global_load_dwordx4 %0, %16, off offset:0 sc0 sc1\n"
      "global_load_dwordx4 %1, %16, off offset:16 sc0 sc1\n"
      "global_load_dwordx4 %2, %16, off offset:32 sc0 sc1\n"
      "global_load_dwordx4 %3, %16, off offset:48 sc0 sc1\n"
      "global_load_dwordx4 %4, %16, off offset:64 sc0 sc1\n"
      "global_load_dwordx4 %5, %16, off offset:80 sc0 sc1\n"
      "global_load_dwordx4 %6, %16, off offset:96 sc0 sc1\n"
      "global_load_dwordx4 %7, %16, off offset:112 sc0 sc1\n"
      "global_load_dwordx4 %8, %16, off offset:128 sc0 sc1\n"
      "global_load_dwordx4 %9, %16, off offset:144 sc0 sc1\n"
      "global_load_dwordx4 %10, %16, off offset:160 sc0 sc1\n"
      "global_load_dwordx4 %11, %16, off offset:176 sc0 sc1\n"
      "global_load_dwordx4 %12, %16, off offset:192 sc0 sc1\n"
      "global_load_dwordx4 %13, %16, off offset:208 sc0 sc1\n"
      "global_load_dwordx4 %14, %16, off offset:224 sc0 sc1\n"
      "global_load_dwordx4 %15, %16, off offset:240 sc0 sc1\n"
      "s_waitcnt vmcnt(0)\n"
      : "=&v"(q[0]), "=&v"(q[1]), "=&v"(q[2]), "=&v"(q[3]), "=&v"(q[4]), "=&v"(q[5]), "=&v"(q[6]), "=&v"(q[7]),
        "=&v"(q[8]), "=&v"(q[9]), "=&v"(q[10]), "=&v"(q[11]), "=&v"(q[12]), "=&v"(q[13]), "=&v"(q[14]),
        "=&v"(q[15])
      : "v"(p)
      : "memory");
}

__device__ __forceinline__ uint64_t tagged(uint32_t tag, float v) {
  return ((uint64_t)tag << 32) | (uint64_t)__float_as_uint(v);
}
__device__ __forceinline__ uint64_t tagged_u(uint32_t tag, uint32_t v) { return ((uint64_t)tag << 32) | (uint64_t)v; }

}  // namespace serve_dev
}  // namespace sml
