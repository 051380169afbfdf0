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

// Pipelined poll of the next request slot, entirely inside ONE asm statement.
// Three polls (this lane's tagged word + the host's head counter) are kept in flight,
// spaced ~1/3 of a PCIe round trip, and each one consumed is re-issued at once, so an
// event is seen ~RTT/3 after its row lands.  Why one statement: with the loads issued by
// one asm and waited by another, the compiler is free to copy a load's destination
// register in between (a loop-carried phi copy) -- reading the register before the data
// landed.  Here the in-flight loads target fixed clobbered registers v[240:251] that no
// compiler code touches, and every load has landed (vmcnt 0) when the statement ends.
// Returns 1: all lanes not in `dontcare` see tag == want (row in `w`, head in `hd`);
// 2: head > lim (backlog); 0: `rounds` rounds without either (caller checks stop/idle).
__device__ __forceinline__ uint32_t poll_ready(const uint64_t* wp, const uint64_t* hp, uint32_t want, uint64_t lim,
                                               uint64_t dontcare, uint32_t rounds, uint64_t& w, uint64_t& hd) {
  uint32_t st, n;
#define SML_POLL_ISSUE(W, H) \
  "global_load_dwordx2 v[" #W "], %[wp], off sc0 sc1\n" \
  "global_load_dwordx2 v[" #H "], %[hp], off sc0 sc1\n"
#define SML_POLL_CHECK(W_HI, H, K) \
  "s_waitcnt vmcnt(4)\n" \
  "v_cmp_lt_u64 vcc, %[lim], v[" #H "]\n" \
  "s_cmp_lg_u64 vcc, 0\n" \
  "s_cbranch_scc1 .Lsml_poll_b" #K "_%=\n" \
  "v_cmp_eq_u32 vcc, %[want], v" #W_HI "\n" \
  "s_or_b64 vcc, vcc, %[dc]\n" \
  "s_cmp_eq_u64 vcc, -1\n" \
  "s_cbranch_scc1 .Lsml_poll_r" #K "_%=\n"
#define SML_POLL_OUT(K, W, H, S) \
  ".Lsml_poll_r" #K "_%=:\n" \
  "s_mov_b32 %[st], 1\n" \
  "s_branch .Lsml_poll_m" #K "_%=\n" \
  ".Lsml_poll_b" #K "_%=:\n" \
  "s_mov_b32 %[st], 2\n" \
  ".Lsml_poll_m" #K "_%=:\n" \
  "v_mov_b64 %[w], v[" #W "]\n" \
  "v_mov_b64 %[hd], v[" #H "]\n" \
  "s_branch .Lsml_poll_e_%=\n"
  asm volatile(
      "s_mov_b32 %[n], %[rounds]\n"
      SML_POLL_ISSUE(240:241, 242:243)
      "s_sleep 8\n"
      SML_POLL_ISSUE(244:245, 246:247)
      "s_sleep 8\n"
      SML_POLL_ISSUE(248:249, 250:251)
      ".Lsml_poll_l_%=:\n"
      SML_POLL_CHECK(241, 242:243, 0)
      SML_POLL_ISSUE(240:241, 242:243)
      SML_POLL_CHECK(245, 246:247, 1)
      SML_POLL_ISSUE(244:245, 246:247)
      SML_POLL_CHECK(249, 250:251, 2)
      SML_POLL_ISSUE(248:249, 250:251)
      "s_sub_u32 %[n], %[n], 1\n"
      "s_cmp_lg_u32 %[n], 0\n"
      "s_cbranch_scc1 .Lsml_poll_l_%=\n"
      "s_mov_b32 %[st], 0\n"
      "v_mov_b64 %[w], 0\n"
      "v_mov_b64 %[hd], 0\n"
      "s_branch .Lsml_poll_e_%=\n"
      SML_POLL_OUT(0, 240:241, 242:243, 0)
      SML_POLL_OUT(1, 244:245, 246:247, 1)
      SML_POLL_OUT(2, 248:249, 250:251, 2)
      ".Lsml_poll_e_%=:\n"
      "s_waitcnt vmcnt(0)\n"
      : [st] "=&s"(st), [n] "=&s"(n), [w] "=&v"(w), [hd] "=&v"(hd)
      : [wp] "v"(wp), [hp] "v"(hp), [want] "v"(want), [lim] "v"(lim), [dc] "s"(dontcare), [rounds] "s"(rounds)
      : "memory", "vcc", "scc", "v240", "v241", "v242", "v243", "v244", "v245", "v246", "v247", "v248", "v249",
        "v250", "v251");
#undef SML_POLL_ISSUE
#undef SML_POLL_CHECK
#undef SML_POLL_OUT
  return st;
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
