// Fused LSTM recurrence kernels for gfx950 (MI355X).
//
// Reference model (LSTM-TensorFlow-IO-Kafka/cardata-v2.py:177-183): stacked Keras
// LSTMs, activation='relu', recurrent_activation='sigmoid', gate order i,f,c,o
// (kernel [in,4u], recurrent_kernel [u,4u], bias [4u]).  TF disables cuDNN for
// relu LSTMs; here the recurrence is a hand-written kernel:
//
//   Zx = X.W + b for every timestep is ONE library GEMM [B*T,in]x[in,4u] (done by
//   the caller); only  z_t = Zx_t + h_{t-1}.U  stays on the sequential path.
//
// One wave owns 16 sequences for the whole time loop; h and c stay in VGPRs.
// Feature-major MFMA orientation (lane c = sequence, registers = gate features):
//   z^T[4u,16] = U^T[4u,u] . h^T[u,16]    (u/16 k-steps x u/4 M-tiles of 16x16x16 bf16)
// so the C tile of gate block m is exactly the B operand layout needed when
// h_t feeds the next step, and i,f,c~,o of one unit land in the same lane/register.
//
// BPTT kernel: walks t = T-1..0 computing dz_t (pre-activation gate grads) and
// the recurrent dh via  dh^T[u,16] = U[u,4u] . dz^T[4u,16]; dz is written out so
// dW = X^T.dz, dU = H_{t-1}^T.dz, db = sum dz, dX = dz.W^T are large library
// GEMMs over B*T rows (no per-step weight-gradient traffic on the serial path).
#include "sml_common.h"

using namespace sml;

namespace {

constexpr int WAVES = 4;

__device__ __forceinline__ float sig(float z) { return sigmoid_fast(z); }

__device__ __forceinline__ float act_f(int a, float z) { return a == ACT_RELU ? relu_fast(z) : tanh_fast(z); }
// derivative of the cell activation, given its input z and output y
__device__ __forceinline__ float act_d(int a, float z, float y) {
  return a == ACT_RELU ? (z > 0.f ? 1.f : 0.f) : fmaf(-y, y, 1.0f);
}

template <int U>
struct LstmArgs {
  const float* zx;     // [B, T, 4U]  x.W + b (row-major)
  const float* Uw;     // [U, 4U]     Keras recurrent_kernel
  const float* h0;     // [B, U] or null
  const float* c0;     // [B, U] or null
  float* hseq;         // [B, T, U]
  float* cseq;         // [B, T, U]
  float* gates;        // [B, T, 4U]  post-activation i, f, c~, o
  int64_t B;
  int T;
  int act;             // cell / candidate activation (relu or tanh)
};

template <int U>
__global__ __launch_bounds__(WAVES * 64) void lstm_fwd_kernel(LstmArgs<U> a) {
  constexpr int G4 = 4 * U;     // gate features
  constexpr int MT = G4 / 16;   // M tiles of the gate vector
  constexpr int UB = U / 16;    // unit blocks (k-steps over h)
  const int lane = threadIdx.x & 63;
  const int wid = threadIdx.x >> 6;
  const int c = lane & 15, g = lane >> 4;
  const int64_t s0 = ((int64_t)blockIdx.x * WAVES + wid) * 16;
  if (s0 >= a.B) return;  // wave-uniform
  const int64_t seq = s0 + c;
  const bool valid = seq < a.B;
  const int64_t sq = valid ? seq : a.B - 1;  // clamped for loads

  // U^T fragments: A[m = gate 16mt + c][k = unit 16s + 4g + j] = U[unit][gate]
  bf16x4 ut[MT][UB];
#pragma unroll
  for (int mt = 0; mt < MT; ++mt)
#pragma unroll
    for (int s = 0; s < UB; ++s)
#pragma unroll
      for (int j = 0; j < 4; ++j)
        ut[mt][s][j] = __builtin_bit_cast(short, (__bf16)a.Uw[(16 * s + 4 * g + j) * G4 + 16 * mt + c]);

  f32x4 h[UB], cs[UB];
#pragma unroll
  for (int b = 0; b < UB; ++b)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int u = 16 * b + 4 * g + i;
      h[b][i] = a.h0 ? a.h0[sq * U + u] : 0.f;
      cs[b][i] = a.c0 ? a.c0[sq * U + u] : 0.f;
    }
  bf16x4 hb[UB];
#pragma unroll
  for (int b = 0; b < UB; ++b) hb[b] = pack4(h[b]);

  const float* zrow = a.zx + sq * (int64_t)a.T * G4;
  f32x4 znext[MT];
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) znext[mt] = *reinterpret_cast<const f32x4*>(zrow + 16 * mt + 4 * g);

  for (int t = 0; t < a.T; ++t) {
    f32x4 z[MT];
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) z[mt] = znext[mt];
    if (t + 1 < a.T) {  // prefetch next step's input projection
#pragma unroll
      for (int mt = 0; mt < MT; ++mt)
        znext[mt] = *reinterpret_cast<const f32x4*>(zrow + (int64_t)(t + 1) * G4 + 16 * mt + 4 * g);
    }
#pragma unroll
    for (int mt = 0; mt < MT; ++mt)
#pragma unroll
      for (int s = 0; s < UB; ++s) z[mt] = mfma16(ut[mt][s], hb[s], z[mt]);

    const int64_t base_g = (sq * a.T + t) * (int64_t)G4;
    const int64_t base_u = (sq * a.T + t) * (int64_t)U;
#pragma unroll
    for (int b = 0; b < UB; ++b) {
      f32x4 gi, gf, gc, go;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        gi[i] = sig(z[b][i]);
        gf[i] = sig(z[UB + b][i]);
        gc[i] = act_f(a.act, z[2 * UB + b][i]);
        go[i] = sig(z[3 * UB + b][i]);
        cs[b][i] = fmaf(gf[i], cs[b][i], gi[i] * gc[i]);
        h[b][i] = go[i] * act_f(a.act, cs[b][i]);
      }
      if (valid) {
        const int off = 16 * b + 4 * g;
        *reinterpret_cast<f32x4*>(a.gates + base_g + off) = gi;
        *reinterpret_cast<f32x4*>(a.gates + base_g + U + off) = gf;
        *reinterpret_cast<f32x4*>(a.gates + base_g + 2 * U + off) = gc;
        *reinterpret_cast<f32x4*>(a.gates + base_g + 3 * U + off) = go;
        *reinterpret_cast<f32x4*>(a.cseq + base_u + off) = cs[b];
        *reinterpret_cast<f32x4*>(a.hseq + base_u + off) = h[b];
      }
      hb[b] = pack4(h[b]);
    }
  }
}

template <int U>
struct LstmBwdArgs {
  const float* dh;     // [B, T, U] gradient w.r.t. the h sequence
  const float* gates;  // [B, T, 4U] post-activation
  const float* cseq;   // [B, T, U]
  const float* c0;     // [B, U] or null
  const float* Uw;     // [U, 4U]
  float* dz;           // [B, T, 4U] pre-activation gate gradients
  float* dh0;          // [B, U] or null: gradient w.r.t. the initial h
  float* dc0;          // [B, U] or null
  int64_t B;
  int T;
  int act;
};

template <int U>
__global__ __launch_bounds__(WAVES * 64) void lstm_bwd_kernel(LstmBwdArgs<U> a) {
  constexpr int G4 = 4 * U;
  constexpr int MT = G4 / 16;
  constexpr int UB = U / 16;
  const int lane = threadIdx.x & 63;
  const int wid = threadIdx.x >> 6;
  const int c = lane & 15, g = lane >> 4;
  const int64_t s0 = ((int64_t)blockIdx.x * WAVES + wid) * 16;
  if (s0 >= a.B) return;
  const int64_t seq = s0 + c;
  const bool valid = seq < a.B;
  const int64_t sq = valid ? seq : a.B - 1;

  // U fragments: A[m = unit 16b + c][k = gate 16kt + 4g + j] = U[unit][gate]
  bf16x4 uf[UB][MT];
#pragma unroll
  for (int b = 0; b < UB; ++b)
#pragma unroll
    for (int kt = 0; kt < MT; ++kt)
#pragma unroll
      for (int j = 0; j < 4; ++j)
        uf[b][kt][j] = __builtin_bit_cast(short, (__bf16)a.Uw[(16 * b + c) * G4 + 16 * kt + 4 * g + j]);

  const f32x4 zero4 = {0.f, 0.f, 0.f, 0.f};
  f32x4 dhr[UB], dcn[UB];
#pragma unroll
  for (int b = 0; b < UB; ++b) dhr[b] = dcn[b] = zero4;

  for (int t = a.T - 1; t >= 0; --t) {
    const int64_t bg = (sq * a.T + t) * (int64_t)G4;
    const int64_t bu = (sq * a.T + t) * (int64_t)U;
    f32x4 dzt[MT];
#pragma unroll
    for (int b = 0; b < UB; ++b) {
      const int off = 16 * b + 4 * g;
      const f32x4 gi = *reinterpret_cast<const f32x4*>(a.gates + bg + off);
      const f32x4 gf = *reinterpret_cast<const f32x4*>(a.gates + bg + U + off);
      const f32x4 gc = *reinterpret_cast<const f32x4*>(a.gates + bg + 2 * U + off);
      const f32x4 go = *reinterpret_cast<const f32x4*>(a.gates + bg + 3 * U + off);
      const f32x4 ct = *reinterpret_cast<const f32x4*>(a.cseq + bu + off);
      f32x4 cp;
      if (t > 0) cp = *reinterpret_cast<const f32x4*>(a.cseq + bu - U + off);
      else if (a.c0) cp = *reinterpret_cast<const f32x4*>(a.c0 + sq * U + off);
      else cp = zero4;
      const f32x4 dho = valid ? *reinterpret_cast<const f32x4*>(a.dh + bu + off) : zero4;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float dh = dho[i] + dhr[b][i];
        const float ac = act_f(a.act, ct[i]);
        const float dc = dcn[b][i] + dh * go[i] * act_d(a.act, ct[i], ac);
        dzt[b][i] = dc * gc[i] * gi[i] * (1.f - gi[i]);                     // d z_i
        dzt[UB + b][i] = dc * cp[i] * gf[i] * (1.f - gf[i]);                // d z_f
        const float gcd = a.act == ACT_RELU ? (gc[i] > 0.f ? 1.f : 0.f) : fmaf(-gc[i], gc[i], 1.f);
        dzt[2 * UB + b][i] = dc * gi[i] * gcd;                              // d z_c~
        dzt[3 * UB + b][i] = dh * ac * go[i] * (1.f - go[i]);               // d z_o
        dcn[b][i] = dc * gf[i];
      }
    }
    if (!valid) {
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) dzt[mt] = zero4;
    }
    bf16x4 dzb[MT];
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) {
      if (valid) *reinterpret_cast<f32x4*>(a.dz + bg + 16 * mt + 4 * g) = dzt[mt];
      dzb[mt] = pack4(dzt[mt]);
    }
    // recurrent gradient for step t-1: dh^T = U . dz^T
#pragma unroll
    for (int b = 0; b < UB; ++b) {
      f32x4 acc = zero4;
#pragma unroll
      for (int kt = 0; kt < MT; ++kt) acc = mfma16(uf[b][kt], dzb[kt], acc);
      dhr[b] = acc;
    }
  }
  if (valid) {
#pragma unroll
    for (int b = 0; b < UB; ++b) {
      const int off = 16 * b + 4 * g;
      if (a.dh0) *reinterpret_cast<f32x4*>(a.dh0 + sq * U + off) = dhr[b];
      if (a.dc0) *reinterpret_cast<f32x4*>(a.dc0 + sq * U + off) = dcn[b];
    }
  }
}

// ---------------------------------------------------------------------------
// U = 128: the recurrent weight no longer fits one wave (4U x U bf16 = 256 VGPRs of
// fragments), so FOUR waves share each 16-sequence tile.  Wave w owns units 32w..32w+31
// (unit blocks 2w, 2w+1): the i / f / c~ / o gate tiles of those units (8 of the 32 gate
// tiles) with their U^T fragments over all 8 unit k-steps in registers (128 VGPRs).  Per
// step each wave computes its 8 gate tiles (64 MFMAs), updates its units' h / c, and
// publishes its two bf16 h blocks through a double-buffered LDS image that every wave
// reads back as the next step's B operand: one barrier per step.  The backward mirrors
// it: each wave forms dz for its own gate tiles, the bf16 dz tiles meet in LDS, and
// dh for the wave's units = U[units][all gates] . dz^T (64 MFMAs).
// ---------------------------------------------------------------------------
constexpr int SU = 128, SG4 = 4 * SU, SMT = SG4 / 16, SUB = SU / 16;

__global__ __launch_bounds__(256) void lstm_fwd_split_kernel(LstmArgs<SU> a) {
  __shared__ bf16x4 hbuf[2][SUB][64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int c = lane & 15, g = lane >> 4;
  const int64_t s0 = (int64_t)blockIdx.x * 16;   // block-uniform
  const int64_t seq = s0 + c;
  const bool valid = seq < a.B;
  const int64_t sq = valid ? seq : a.B - 1;
  // local tile li = 2q + j: gate q of unit block b = 2w + j, global gate tile q * SUB + b
  bf16x4 ut[8][SUB];
#pragma unroll
  for (int li = 0; li < 8; ++li) {
    const int mt = (li >> 1) * SUB + 2 * w + (li & 1);
#pragma unroll
    for (int s = 0; s < SUB; ++s)
#pragma unroll
      for (int j = 0; j < 4; ++j)
        ut[li][s][j] = __builtin_bit_cast(short, (__bf16)a.Uw[(16 * s + 4 * g + j) * SG4 + 16 * mt + c]);
  }
  f32x4 h[2], cs[2];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int u = 16 * (2 * w + j) + 4 * g + i;
      h[j][i] = a.h0 ? a.h0[sq * SU + u] : 0.f;
      cs[j][i] = a.c0 ? a.c0[sq * SU + u] : 0.f;
    }
    hbuf[0][2 * w + j][lane] = pack4(h[j]);
  }
  const float* zrow = a.zx + sq * (int64_t)a.T * SG4;
  f32x4 znext[8];
#pragma unroll
  for (int li = 0; li < 8; ++li) {
    const int mt = (li >> 1) * SUB + 2 * w + (li & 1);
    znext[li] = *reinterpret_cast<const f32x4*>(zrow + 16 * mt + 4 * g);
  }
  __syncthreads();
  for (int t = 0; t < a.T; ++t) {
    const int cur = t & 1;
    f32x4 z[8];
#pragma unroll
    for (int li = 0; li < 8; ++li) z[li] = znext[li];
    if (t + 1 < a.T) {
#pragma unroll
      for (int li = 0; li < 8; ++li) {
        const int mt = (li >> 1) * SUB + 2 * w + (li & 1);
        znext[li] = *reinterpret_cast<const f32x4*>(zrow + (int64_t)(t + 1) * SG4 + 16 * mt + 4 * g);
      }
    }
    bf16x4 hb[SUB];
#pragma unroll
    for (int s = 0; s < SUB; ++s) hb[s] = hbuf[cur][s][lane];
#pragma unroll
    for (int li = 0; li < 8; ++li)
#pragma unroll
      for (int s = 0; s < SUB; ++s) z[li] = mfma16(ut[li][s], hb[s], z[li]);
    const int64_t base_g = (sq * a.T + t) * (int64_t)SG4;
    const int64_t base_u = (sq * a.T + t) * (int64_t)SU;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      f32x4 gi, gf, gc, go;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        gi[i] = sig(z[0 + j][i]);
        gf[i] = sig(z[2 + j][i]);
        gc[i] = act_f(a.act, z[4 + j][i]);
        go[i] = sig(z[6 + j][i]);
        cs[j][i] = fmaf(gf[i], cs[j][i], gi[i] * gc[i]);
        h[j][i] = go[i] * act_f(a.act, cs[j][i]);
      }
      const int off = 16 * (2 * w + j) + 4 * g;
      if (valid) {
        *reinterpret_cast<f32x4*>(a.gates + base_g + off) = gi;
        *reinterpret_cast<f32x4*>(a.gates + base_g + SU + off) = gf;
        *reinterpret_cast<f32x4*>(a.gates + base_g + 2 * SU + off) = gc;
        *reinterpret_cast<f32x4*>(a.gates + base_g + 3 * SU + off) = go;
        *reinterpret_cast<f32x4*>(a.cseq + base_u + off) = cs[j];
        *reinterpret_cast<f32x4*>(a.hseq + base_u + off) = h[j];
      }
      hbuf[cur ^ 1][2 * w + j][lane] = pack4(h[j]);   // read after this step's barrier
    }
    __syncthreads();
  }
}

__global__ __launch_bounds__(256) void lstm_bwd_split_kernel(LstmBwdArgs<SU> a) {
  __shared__ bf16x4 dzbuf[2][SMT][64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int c = lane & 15, g = lane >> 4;
  const int64_t s0 = (int64_t)blockIdx.x * 16;
  const int64_t seq = s0 + c;
  const bool valid = seq < a.B;
  const int64_t sq = valid ? seq : a.B - 1;
  // U fragments of the wave's two unit blocks over all gate k-tiles:
  // A[m = unit 16b + c][k = gate 16kt + 4g + jj] = U[unit][gate]
  bf16x4 uf[2][SMT];
#pragma unroll
  for (int j = 0; j < 2; ++j)
#pragma unroll
    for (int kt = 0; kt < SMT; ++kt)
#pragma unroll
      for (int jj = 0; jj < 4; ++jj)
        uf[j][kt][jj] = __builtin_bit_cast(short, (__bf16)a.Uw[(16 * (2 * w + j) + c) * SG4 + 16 * kt + 4 * g + jj]);
  const f32x4 zero4 = {0.f, 0.f, 0.f, 0.f};
  f32x4 dhr[2] = {zero4, zero4}, dcn[2] = {zero4, zero4};
  for (int t = a.T - 1; t >= 0; --t) {
    const int cur = t & 1;
    const int64_t bg = (sq * a.T + t) * (int64_t)SG4;
    const int64_t bu = (sq * a.T + t) * (int64_t)SU;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int b = 2 * w + j;
      const int off = 16 * b + 4 * g;
      const f32x4 gi = *reinterpret_cast<const f32x4*>(a.gates + bg + off);
      const f32x4 gf = *reinterpret_cast<const f32x4*>(a.gates + bg + SU + off);
      const f32x4 gc = *reinterpret_cast<const f32x4*>(a.gates + bg + 2 * SU + off);
      const f32x4 go = *reinterpret_cast<const f32x4*>(a.gates + bg + 3 * SU + off);
      const f32x4 ct = *reinterpret_cast<const f32x4*>(a.cseq + bu + off);
      f32x4 cp;
      if (t > 0) cp = *reinterpret_cast<const f32x4*>(a.cseq + bu - SU + off);
      else if (a.c0) cp = *reinterpret_cast<const f32x4*>(a.c0 + sq * SU + off);
      else cp = zero4;
      const f32x4 dho = valid ? *reinterpret_cast<const f32x4*>(a.dh + bu + off) : zero4;
      f32x4 dzt[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float dh = dho[i] + dhr[j][i];
        const float ac = act_f(a.act, ct[i]);
        const float dc = dcn[j][i] + dh * go[i] * act_d(a.act, ct[i], ac);
        dzt[0][i] = dc * gc[i] * gi[i] * (1.f - gi[i]);
        dzt[1][i] = dc * cp[i] * gf[i] * (1.f - gf[i]);
        const float gcd = a.act == ACT_RELU ? (gc[i] > 0.f ? 1.f : 0.f) : fmaf(-gc[i], gc[i], 1.f);
        dzt[2][i] = dc * gi[i] * gcd;
        dzt[3][i] = dh * ac * go[i] * (1.f - go[i]);
        dcn[j][i] = dc * gf[i];
      }
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        if (!valid) dzt[q] = zero4;
        const int mt = q * SUB + b;
        if (valid) *reinterpret_cast<f32x4*>(a.dz + bg + 16 * mt + 4 * g) = dzt[q];
        dzbuf[cur][mt][lane] = pack4(dzt[q]);
      }
    }
    __syncthreads();
    // recurrent gradient for step t-1 of the wave's units: dh^T = U . dz^T over all gates
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      f32x4 acc = zero4;
#pragma unroll
      for (int kt = 0; kt < SMT; ++kt) acc = mfma16(uf[j][kt], dzbuf[cur][kt][lane], acc);
      dhr[j] = acc;
    }
  }
  if (valid) {
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int off = 16 * (2 * w + j) + 4 * g;
      if (a.dh0) *reinterpret_cast<f32x4*>(a.dh0 + sq * SU + off) = dhr[j];
      if (a.dc0) *reinterpret_cast<f32x4*>(a.dc0 + sq * SU + off) = dcn[j];
    }
  }
}

}  // namespace

namespace sml {

hipError_t lstm_fwd_launch(const float* zx, const float* Uw, const float* h0, const float* c0, float* hseq,
                           float* cseq, float* gates, int64_t B, int T, int U, int act, hipStream_t stream) {
  const int grid = (int)((B + 16 * WAVES - 1) / (16 * WAVES));
  if (U == 16) {
    LstmArgs<16> a{zx, Uw, h0, c0, hseq, cseq, gates, B, T, act};
    hipLaunchKernelGGL(lstm_fwd_kernel<16>, dim3(grid), dim3(WAVES * 64), 0, stream, a);
  } else if (U == 32) {
    LstmArgs<32> a{zx, Uw, h0, c0, hseq, cseq, gates, B, T, act};
    hipLaunchKernelGGL(lstm_fwd_kernel<32>, dim3(grid), dim3(WAVES * 64), 0, stream, a);
  } else if (U == 64) {
    LstmArgs<64> a{zx, Uw, h0, c0, hseq, cseq, gates, B, T, act};
    hipLaunchKernelGGL(lstm_fwd_kernel<64>, dim3(grid), dim3(WAVES * 64), 0, stream, a);
  } else if (U == SU) {   // four waves per 16-sequence tile
    LstmArgs<SU> a{zx, Uw, h0, c0, hseq, cseq, gates, B, T, act};
    hipLaunchKernelGGL(lstm_fwd_split_kernel, dim3((unsigned)((B + 15) / 16)), dim3(256), 0, stream, a);
  } else {
    return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

hipError_t lstm_bwd_launch(const float* dh, const float* gates, const float* cseq, const float* c0, const float* Uw,
                           float* dz, float* dh0, float* dc0, int64_t B, int T, int U, int act, hipStream_t stream) {
  const int grid = (int)((B + 16 * WAVES - 1) / (16 * WAVES));
  if (U == 16) {
    LstmBwdArgs<16> a{dh, gates, cseq, c0, Uw, dz, dh0, dc0, B, T, act};
    hipLaunchKernelGGL(lstm_bwd_kernel<16>, dim3(grid), dim3(WAVES * 64), 0, stream, a);
  } else if (U == 32) {
    LstmBwdArgs<32> a{dh, gates, cseq, c0, Uw, dz, dh0, dc0, B, T, act};
    hipLaunchKernelGGL(lstm_bwd_kernel<32>, dim3(grid), dim3(WAVES * 64), 0, stream, a);
  } else if (U == 64) {
    LstmBwdArgs<64> a{dh, gates, cseq, c0, Uw, dz, dh0, dc0, B, T, act};
    hipLaunchKernelGGL(lstm_bwd_kernel<64>, dim3(grid), dim3(WAVES * 64), 0, stream, a);
  } else if (U == SU) {
    LstmBwdArgs<SU> a{dh, gates, cseq, c0, Uw, dz, dh0, dc0, B, T, act};
    hipLaunchKernelGGL(lstm_bwd_split_kernel, dim3((unsigned)((B + 15) / 16)), dim3(256), 0, stream, a);
  } else {
    return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

}  // namespace sml
