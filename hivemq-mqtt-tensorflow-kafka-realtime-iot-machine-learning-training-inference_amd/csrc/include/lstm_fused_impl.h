// Shared device helpers for the fused LSTM layer kernels (lstm_fused.hip: backward,
// lstm_fused_fwd.hip: forward).  Included by exactly those two translation units; the
// two are separate files because they want different MFMA register forms (the forward
// keeps its gate accumulators in VGPRs, the backward its weight-gradient accumulators
// in AGPRs -- see the build marker at the top of lstm_fused.hip).
#pragma once
#include <cstdlib>

#include "sml_common.h"
#include "sml_ops.h"

namespace sml_lstm {

using namespace sml;

constexpr int WAVES = 4;

__device__ __forceinline__ float act_f(int a, float z) { return a == ACT_RELU ? relu_fast(z) : tanh_fast(z); }
__device__ __forceinline__ float act_d(int a, float z, float y) {
  return a == ACT_RELU ? (z > 0.f ? 1.f : 0.f) : fmaf(-y, y, 1.0f);
}

__device__ __forceinline__ bf16x4 ld_bf16x4(const __bf16* p) { return *reinterpret_cast<const bf16x4*>(p); }
__device__ __forceinline__ f32x4 unpack4(bf16x4 v) {
  f32x4 r;
#pragma unroll
  for (int j = 0; j < 4; ++j) r[j] = bf16_to_f32((unsigned short)v[j]);
  return r;
}

// The lane id through an empty asm: the compiler cannot treat addresses built from it
// as loop-invariant, so LDS operand reads are not hoisted into (scarce) registers.
__device__ __forceinline__ int opaque_lane(int lane) {
  asm volatile("" : "+v"(lane));
  return lane;
}

// Four consecutive row elements p[k0 .. k0+3], XV floats per load, in two halves:
// load_row4 issues the loads from clamped in-row addresses (never out of bounds, never
// under a lane mask) and mask_row4 zeroes the columns past IN.  The mask is applied
// where the value is CONSUMED: a select right after the load would make the wave wait
// for the load there, which is what the prefetch exists to avoid.
template <int XV>
__device__ __forceinline__ f32x4 load_row4(const float* p, int k0, int IN) {
  if constexpr (XV == 4) {
    return *reinterpret_cast<const f32x4*>(p + (k0 < IN ? k0 : 0));
  } else if constexpr (XV == 2) {
    const f32x2_t lo = *reinterpret_cast<const f32x2_t*>(p + (k0 < IN ? k0 : 0));
    const f32x2_t hi = *reinterpret_cast<const f32x2_t*>(p + (k0 + 2 < IN ? k0 + 2 : 0));
    return f32x4{lo[0], lo[1], hi[0], hi[1]};
  } else {
    f32x4 r;
#pragma unroll
    for (int j = 0; j < 4; ++j) r[j] = p[k0 + j < IN ? k0 + j : 0];
    return r;
  }
}
__device__ __forceinline__ f32x4 mask_row4(f32x4 r, int k0, int IN) {
#pragma unroll
  for (int j = 0; j < 4; ++j) r[j] = k0 + j < IN ? r[j] : 0.f;
  return r;
}

// bf16 rows (inter-layer activations): XV elements per load, 8 / 4 / 2 bytes
typedef short s16x2_t __attribute__((ext_vector_type(2)));
template <int XV>
__device__ __forceinline__ bf16x4 load_row4(const __bf16* p, int k0, int IN) {
  if constexpr (XV == 4) {
    return *reinterpret_cast<const bf16x4*>(p + (k0 < IN ? k0 : 0));
  } else if constexpr (XV == 2) {
    const s16x2_t lo = *reinterpret_cast<const s16x2_t*>(p + (k0 < IN ? k0 : 0));
    const s16x2_t hi = *reinterpret_cast<const s16x2_t*>(p + (k0 + 2 < IN ? k0 + 2 : 0));
    return bf16x4{lo[0], lo[1], hi[0], hi[1]};
  } else {
    const short* q = reinterpret_cast<const short*>(p);
    bf16x4 r;
#pragma unroll
    for (int j = 0; j < 4; ++j) r[j] = q[k0 + j < IN ? k0 + j : 0];
    return r;
  }
}

// the MFMA B operand of a raw row piece: columns past IN zeroed, bf16
__device__ __forceinline__ bf16x4 row_operand(f32x4 raw, int k0, int IN) { return pack4(mask_row4(raw, k0, IN)); }
__device__ __forceinline__ bf16x4 row_operand(bf16x4 raw, int k0, int IN) {
#pragma unroll
  for (int j = 0; j < 4; ++j) raw[j] = k0 + j < IN ? raw[j] : (short)0;
  return raw;
}

// The same operand with the mask as bits: lane-fixed keep words (0xFFFF per kept bf16 column,
// row_keep) and the constant-1 bias columns merged in one v_bfi_b32 per register -- the per-element
// selects of row_operand are 4 VALU per piece and step in the fused recurrences' hot loops.
typedef unsigned u32x2_t __attribute__((ext_vector_type(2)));
__device__ __forceinline__ u32x2_t row_keep(int k0, int IN) {
  u32x2_t k;
  k[0] = (k0 < IN ? 0xFFFFu : 0u) | (k0 + 1 < IN ? 0xFFFF0000u : 0u);
  k[1] = (k0 + 2 < IN ? 0xFFFFu : 0u) | (k0 + 3 < IN ? 0xFFFF0000u : 0u);
  return k;
}
__device__ __forceinline__ bf16x4 row_operand_k(f32x4 raw, u32x2_t keep, bf16x4 ones) {
  const u32x2_t p = __builtin_bit_cast(u32x2_t, pack4(raw)), o = __builtin_bit_cast(u32x2_t, ones);
  u32x2_t r;
#pragma unroll
  for (int i = 0; i < 2; ++i) r[i] = (p[i] & keep[i]) | (o[i] & ~keep[i]);
  return __builtin_bit_cast(bf16x4, r);
}
__device__ __forceinline__ bf16x4 row_operand_k(bf16x4 raw, u32x2_t keep, bf16x4 ones) {
  const u32x2_t p = __builtin_bit_cast(u32x2_t, raw), o = __builtin_bit_cast(u32x2_t, ones);
  u32x2_t r;
#pragma unroll
  for (int i = 0; i < 2; ++i) r[i] = (p[i] & keep[i]) | (o[i] & ~keep[i]);
  return __builtin_bit_cast(bf16x4, r);
}

// x element type -> raw register type of a 4-element row piece
template <typename XT> struct RowRaw { using type = f32x4; };
template <> struct RowRaw<__bf16> { using type = bf16x4; };

// (U, KT bucket, x row vector width, x element type) -> kernel instance
template <typename F>
hipError_t dispatch(int U, int IN, int xv, bool x_bf16, F&& f) {
  const int KT = (IN + 15) / 16;
  auto with_t = [&](auto u, auto k, auto v) {
    if (x_bf16) return f(u, k, v, (const __bf16*)nullptr);
    return f(u, k, v, (const float*)nullptr);
  };
#define SML_UK(u, k)                                                                                          \
  if (U == u && KT <= k) {                                                                                    \
    using UC = std::integral_constant<int, u>;                                                                \
    using KC = std::integral_constant<int, k>;                                                                \
    if (xv == 4) return with_t(UC{}, KC{}, std::integral_constant<int, 4>{});                                 \
    if (xv == 2) return with_t(UC{}, KC{}, std::integral_constant<int, 2>{});                                 \
    return with_t(UC{}, KC{}, std::integral_constant<int, 1>{});                                              \
  }
  SML_UK(16, 1) SML_UK(16, 2) SML_UK(16, 4)
  SML_UK(32, 1) SML_UK(32, 2)
  // U = 64: scalar row loads only (a third of the instances; the per-step x load is not what
  // bounds a U = 64 layer)
  if (U == 64 && KT <= 2) {
    using UC = std::integral_constant<int, 64>;
    if (KT <= 1) return with_t(UC{}, std::integral_constant<int, 1>{}, std::integral_constant<int, 1>{});
    return with_t(UC{}, std::integral_constant<int, 2>{}, std::integral_constant<int, 1>{});
  }
#undef SML_UK
  return hipErrorInvalidValue;
}

// Bias modes of the fused kernels (BM), chosen per layer by bias_mode():
//   BM_PLAIN 0: bias in registers (forward) / LDS (backward recompute); db summed per step.
//   BM_BX    1 ("bias columns", needs IN + 2 <= 16*KT, e.g. the 18 car features in 32
//            K-slots): the x MFMA operand carries a constant 1.0 in columns IN and IN + 1 and
//            the W^T fragments carry the bias there, split as bf16 hi + lo (hi + lo equals the
//            fp32 bias to 2^-16 relative).  The gate pre-activations come out of the MFMAs
//            with the bias included -- no bias registers, no accumulator initialisation --
//            and in the backward the same constant column makes dW^T column IN the bias
//            gradient (no per-step db adds).  Forward and backward recompute use identical
//            operands, so the recomputed pre-activations stay bit-identical.
//   BM_DB    2 (needs IN + 1 <= 16*KT): only the backward changes -- a constant-1 x column
//            with zero weights, whose dW^T column is db; the bias itself stays as in PLAIN.
// In BX and DB db is the sum of bf16-rounded dz (the dW / dU precision) instead of fp32.
// SML_LSTM_BIASCOL=0 / 1 / d selects PLAIN / BX / DB where the layer admits it (A/B;
// default BX, else DB, else PLAIN).
// SML_LSTM_BIASCOL=m (A/B): the backward in BX mode under a plain forward -- the recomputed
// pre-activations then differ from the forward's by the bias's fp32 rounding (not bit-identical).
constexpr int BM_PLAIN = 0, BM_BX = 1, BM_DB = 2;
inline char bias_env() {
  static const char m = [] {
    const char* e = std::getenv("SML_LSTM_BIASCOL");
    return e && e[0] ? e[0] : '1';
  }();
  return m;
}
inline int bias_mode(int IN, int KT) {
  const char m = bias_env();
  if (m == '0') return BM_PLAIN;
  if (m != 'd' && IN + 2 <= 16 * KT) return BM_BX;
  return IN + 1 <= 16 * KT ? BM_DB : BM_PLAIN;
}
// the forward's bias mode: the backward's, except under SML_LSTM_BIASCOL=m
inline int bias_mode_fwd(int IN, int KT) { return bias_env() == 'm' ? BM_PLAIN : bias_mode(IN, KT); }

// lane (c, g)'s constant-1 bits for x tile kt (BX / DB): bf16 1.0 at columns IN, IN + 1
// (in DB column IN + 1, if it exists, also has zero weights: one more padding column)
__device__ __forceinline__ bf16x4 ones_at_bias(int kt, int g, int IN) {
  bf16x4 r;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int f = 16 * kt + 4 * g + j;
    r[j] = (f == IN || f == IN + 1) ? (short)0x3F80 : (short)0;
  }
  return r;
}

// W^T fragment element (gate m, feature f) in BX mode: the weight, or the bias hi / lo parts
__device__ __forceinline__ float wt_elem_bx(const float* W, const float* b, int G4, int IN, int f, int m) {
  if (f < IN) return W[(int64_t)f * G4 + m];
  const float bv = b[m];
  const float hi = bf16_to_f32((unsigned short)(pack2(bv, 0.f) & 0xFFFFu));   // RNE, as the fragment pack
  if (f == IN) return hi;
  if (f == IN + 1) return bv - hi;
  return 0.f;
}

// widest row access (elements, up to 4) that IN and the base pointer's alignment allow
inline int row_vec(const void* p, int IN, int elem_bytes) {
  const uintptr_t u = (uintptr_t)p;
  if ((IN & 3) == 0 && (u & (4 * elem_bytes - 1)) == 0) return 4;
  if ((IN & 1) == 0 && (u & (2 * elem_bytes - 1)) == 0) return 2;
  return 1;
}

}  // namespace sml_lstm
