// Shared device helpers for the streamml gfx950 kernels.
//
// MFMA fragment conventions used throughout (v_mfma_f32_16x16x16_bf16, wave64):
//   lane l, c = l & 15, g = l >> 4
//   A operand  (16x16, 4 bf16/lane): A[m = c][k = 4g + j],  j = 0..3
//   B operand  (16x16, 4 bf16/lane): B[k = 4g + j][n = c]
//   C/D        (16x16, 4 f32/lane) : C[m = 4g + i][n = c],  i = 0..3
//
// "Feature-major" (transposed) orientation: a 16-feature x 16-row activation tile
// P[f][r] held with f = 4g+i on registers and r = c on lanes.  That is both the
// C layout of W^T . X^T and the B layout of the next layer, so layers chain with
// no data movement.  Re-reading the same registers as an A operand gives P^T,
// so one MFMA against the identity converts a tile to "row-major" orientation
// (rows on registers, feature on the lane) which is what the weight-gradient
// MFMA (contraction over rows) consumes.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

// SML_DCHECK: device-side bounds / invariant assert, compiled in only by the checked
// build (python -m streamml._build --checked -> _C_dbg.so, loaded when the process
// runs with SML_KERNEL_CHECKS=1).  A failed check prints the condition and traps the
// wave, so the fault names its cause.  Release builds compile it away.
#if defined(SML_KERNEL_CHECKS) && SML_KERNEL_CHECKS
#define SML_DCHECK(cond)                                                           \
  do {                                                                             \
    if (!(cond)) {                                                                 \
      printf("SML_DCHECK failed: %s (%s:%d)\n", #cond, __FILE__, __LINE__);        \
      __builtin_trap();                                                            \
    }                                                                              \
  } while (0)
#else
#define SML_DCHECK(cond) ((void)0)
#endif

namespace sml {

typedef short bf16x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));
typedef float f32x2_t __attribute__((ext_vector_type(2)));

enum Act : int { ACT_LINEAR = 0, ACT_RELU = 1, ACT_TANH = 2, ACT_SIGMOID = 3 };

__device__ __forceinline__ f32x4 mfma16(bf16x4 a, bf16x4 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(a, b, c, 0, 0, 0);
}

// Two consecutive K=16 tiles in ONE gfx950 v_mfma_f32_16x16x32_bf16: lane (c, g) holds
// k = 4g..4g+3 of tile 0 and of tile 1, i.e. hardware k 8g..8g+7 is the logical
// {16*0 + 4g + e, 16*1 + 4g + e}.  A and B are permuted alike, so the contraction is the
// same sum as mfma16(a0, b0) + mfma16(a1, b1), in half the MFMA issues.
__device__ __forceinline__ f32x4 mfma32(bf16x4 a0, bf16x4 a1, bf16x4 b0, bf16x4 b1, f32x4 c) {
  typedef short s16x8 __attribute__((ext_vector_type(8)));
  typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
  const s16x8 a = __builtin_shufflevector(a0, a1, 0, 1, 2, 3, 4, 5, 6, 7);
  const s16x8 b = __builtin_shufflevector(b0, b1, 0, 1, 2, 3, 4, 5, 6, 7);
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, a), __builtin_bit_cast(bf16x8, b), c, 0,
                                                 0, 0);
}

// The same with the A operand already concatenated (static fragments kept as one 8-short
// vector: no register copies to make the two K halves adjacent at every use).
typedef short s16x8 __attribute__((ext_vector_type(8)));
__device__ __forceinline__ s16x8 cat8(bf16x4 a0, bf16x4 a1) { return __builtin_shufflevector(a0, a1, 0, 1, 2, 3, 4, 5, 6, 7); }
__device__ __forceinline__ f32x4 mfma32a(s16x8 a, bf16x4 b0, bf16x4 b1, f32x4 c) {
  typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
  const s16x8 b = __builtin_shufflevector(b0, b1, 0, 1, 2, 3, 4, 5, 6, 7);
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, a), __builtin_bit_cast(bf16x8, b), c, 0,
                                                 0, 0);
}

__device__ __forceinline__ unsigned pack2(float lo, float hi) {
  f32x2_t v = {lo, hi};
  bf16x2_t b = __builtin_convertvector(v, bf16x2_t);
  return __builtin_bit_cast(unsigned, b);
}

__device__ __forceinline__ bf16x4 pack4(f32x4 v) {
  unsigned lo = pack2(v[0], v[1]);
  unsigned hi = pack2(v[2], v[3]);
  typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
  u32x2 u = {lo, hi};
  return __builtin_bit_cast(bf16x4, u);
}

__device__ __forceinline__ float bf16_to_f32(unsigned short h) {
  return __uint_as_float(((unsigned)h) << 16);
}

__device__ __forceinline__ float rcp_fast(float x) { return __builtin_amdgcn_rcpf(x); }

__device__ __forceinline__ float tanh_fast(float z) {
  // tanh(z) = 1 - 2 / (exp(2z) + 1); exp(2z) = exp2(z * 2*log2(e)).
  // Saturates correctly at +-inf (rcp(inf) = 0).
  const float e = __builtin_amdgcn_exp2f(z * 2.8853900817779268f);
  return fmaf(-2.0f, rcp_fast(e + 1.0f), 1.0f);
}

// max(z, 0) in one v_med3_f32 (fmaxf adds a NaN-canonicalising v_max)
__device__ __forceinline__ float relu_fast(float z) { return __builtin_amdgcn_fmed3f(z, 0.0f, 3.402823466e38f); }

__device__ __forceinline__ float sigmoid_fast(float z) { return rcp_fast(1.0f + __expf(-z)); }

__device__ __forceinline__ float act_fwd(int a, float z) {
  switch (a) {
    case ACT_RELU: return relu_fast(z);
    case ACT_TANH: return tanh_fast(z);
    case ACT_SIGMOID: return sigmoid_fast(z);
    default: return z;
  }
}

// d * act'(.) expressed through the activation output h
__device__ __forceinline__ float act_grad(int a, float h, float d) {
  switch (a) {
    case ACT_RELU: return h > 0.0f ? d : 0.0f;
    case ACT_TANH: return d * fmaf(-h, h, 1.0f);
    case ACT_SIGMOID: return d * h * (1.0f - h);
    default: return d;
  }
}

// derivative expressed through the activation output h
__device__ __forceinline__ float act_bwd(int a, float h) {
  switch (a) {
    case ACT_RELU: return h > 0.0f ? 1.0f : 0.0f;
    case ACT_TANH: return 1.0f - h * h;
    case ACT_SIGMOID: return h * (1.0f - h);
    default: return 1.0f;
  }
}

// identity B operand: B[k = 4g+j][n = c] = (4g+j == c)
__device__ __forceinline__ bf16x4 identity_b(int c, int g) {
  bf16x4 r;
#pragma unroll
  for (int j = 0; j < 4; ++j) r[j] = (4 * g + j == c) ? (short)0x3F80 : (short)0;
  return r;
}

// transpose a feature-major bf16 tile to row-major orientation (C layout, f32)
__device__ __forceinline__ f32x4 transpose_tile(bf16x4 t, bf16x4 ident) {
  f32x4 z = {0.f, 0.f, 0.f, 0.f};
  return mfma16(t, ident, z);
}

// Lane exchange across 16-lane rows / 32-lane halves with the gfx950 VALU
// permlane swaps (no LDS traffic).  xor16(v) returns v of lane (l ^ 16),
// xor32(v) returns v of lane (l ^ 32).
__device__ __forceinline__ float xor16(float v, int lane) {
  const unsigned u = __float_as_uint(v);
  const auto r = __builtin_amdgcn_permlane16_swap(u, u, false, false);
  return __uint_as_float(((lane >> 4) & 1) ? r[0] : r[1]);
}
__device__ __forceinline__ float xor32(float v, int lane) {
  const unsigned u = __float_as_uint(v);
  const auto r = __builtin_amdgcn_permlane32_swap(u, u, false, false);
  return __uint_as_float(lane >= 32 ? r[0] : r[1]);
}
__device__ __forceinline__ int xor16i(int v, int lane) { return __float_as_int(xor16(__int_as_float(v), lane)); }
__device__ __forceinline__ int xor32i(int v, int lane) { return __float_as_int(xor32(__int_as_float(v), lane)); }

typedef __attribute__((address_space(3))) bf16x4 lds_bf16x4;

// 16x16 bf16 tile transpose through LDS (gfx950 ds_read_b64_tr_b16).
// In : feature-major tile, lane (c, g) holds P[f = 4g+i][r = c], i = 0..3.
// Out: row-major tile,     lane (c, g) holds P[f = c][r = 4g+q], q = 0..3,
//      i.e. the MFMA A operand P^T[m = feature][k = row] / B operand
//      P[k = row][n = feature] that a contraction over rows needs.
// The wave-private 512-byte image is [r][f] (32-byte rows): the write is one
// 8-byte ds_write per lane; the read is one ds_read_b64_tr_b16 per lane, lane
// 4q+p of each 16-lane group addressing row 4g+q, columns 4p..4p+3.
// LDS ops of one wave complete in order, so no wait is needed between the write
// and the transposed read beyond the one the compiler places before the use.
// XOR swizzle: the 8-byte column of row r is stored at column (col ^ ((r >> 2) & 3)).  With plain
// 32-byte rows the write put lanes c, c + 4, c + 8, c + 12 of a 16-lane group on the same banks
// (4-way conflict on every ds_write_b64: SQ_LDS_BANK_CONFLICT 3.6-5.9 cycles per LDS instruction
// in the LSTM backward, profiles/r06); swizzled, the write and the transposed read are both
// conflict-free, and every lane still reads the same 8 bytes, so the result is bit-identical.
__device__ __forceinline__ int tr_wr_off(int c, int g) { return c * 32 + 8 * (g ^ ((c >> 2) & 3)); }
__device__ __forceinline__ int tr_rd_off(int c, int g) { return (4 * g + (c >> 2)) * 32 + 8 * ((c & 3) ^ g); }
__device__ __forceinline__ bf16x4 lds_transpose(bf16x4 v, char* wave_scratch, int c, int g) {
  lds_bf16x4* wr = (lds_bf16x4*)(wave_scratch + tr_wr_off(c, g));
  *wr = v;
  lds_bf16x4* rd = (lds_bf16x4*)(wave_scratch + tr_rd_off(c, g));
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16(rd);
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

}  // namespace sml
