// Fused LSTM layer forward (the backward and the design notes are in lstm_fused.hip):
// x.W + recurrence + cell-state save in ONE launch, one wave per 16 sequences.
#include "lstm_fused_impl.h"

using namespace sml;
using namespace sml_lstm;

namespace {

struct FusedFwdArgs {
  const void* x;       // [B, T, IN] fp32 (model input) or bf16 (a lower LSTM layer's h); sequence b
                       // starts x_seq elements after sequence b-1 (T*IN: contiguous; IN: the
                       // sliding windows of cardata-v2.py:199-206 read in place from the base rows)
  const float* W;      // [IN, 4U]
  const float* Uw;     // [U, 4U]
  const float* b;      // [4U]
  const float* h0;     // [B, U] or null
  const float* c0;     // [B, U] or null
  __bf16* hseq;        // [B16, T, U] bf16, B16 = B rounded up to 16 (rows past B are scratch).
                       // bf16 loses nothing downstream: every consumer (the next layer's x,
                       // this layer's backward, a Dense head) feeds it to bf16 MFMAs
  __bf16* cseq;        // [B/16, T, U/16, 64, 4]   cell state, bf16, fragment-native (backward only)
  int64_t B;
  int T, IN, act;
  int64_t x_seq;
};

// BX: bias columns (lstm_fused_impl.h bias_mode BM_BX): the bias enters through constant-1 x columns
// IN, IN + 1 and the W^T fragment, so no bias registers (32 VGPRs at U = 32) and no
// accumulator initialisation -- identical operands to the backward's gate recompute.
template <int U, int KT, int XV, typename XT, int ACT, bool BX = false, int PF = 2>
__global__ __launch_bounds__(WAVES * 64, 1) void lstm_fused_fwd_kernel(FusedFwdArgs a) {
  using XR = typename RowRaw<XT>::type;
  constexpr int G4 = 4 * U, MT = G4 / 16, UB = U / 16;
  const int lane = threadIdx.x & 63, c = lane & 15, g = lane >> 4;
  const int64_t s0 = ((int64_t)blockIdx.x * WAVES + (threadIdx.x >> 6)) * 16;
  if (s0 >= a.B) return;  // wave-uniform
  const int64_t seq = s0 + c;
  const bool valid = seq < a.B;
  const int64_t sq = valid ? seq : a.B - 1;
  const int IN = a.IN, T = a.T;

  // A fragments: W^T[m = gate][k = feature], U^T[m = gate][k = unit]
  bf16x4 wt[MT][KT], ut[MT][UB];
  f32x4 bias[MT];
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) {
#pragma unroll
    for (int kt = 0; kt < KT; ++kt) {
      f32x4 t4;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int k = 16 * kt + 4 * g + j;
        t4[j] = BX ? wt_elem_bx(a.W, a.b, G4, IN, k, 16 * mt + c) : (k < IN ? a.W[(int64_t)k * G4 + 16 * mt + c] : 0.f);
      }
      wt[mt][kt] = pack4(t4);
    }
#pragma unroll
    for (int s = 0; s < UB; ++s) {
      f32x4 t4;
#pragma unroll
      for (int j = 0; j < 4; ++j) t4[j] = a.Uw[(16 * s + 4 * g + j) * G4 + 16 * mt + c];
      ut[mt][s] = pack4(t4);
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) bias[mt][i] = BX ? 0.f : a.b[16 * mt + 4 * g + i];
  }
  bf16x4 onex[KT];   // BX: the constant-1 bits of x columns IN, IN + 1
#pragma unroll
  for (int kt = 0; kt < KT; ++kt) onex[kt] = BX ? ones_at_bias(kt, g, IN) : bf16x4{0, 0, 0, 0};
  f32x4 h[UB], cs[UB];
  bf16x4 hb[UB];
#pragma unroll
  for (int b = 0; b < UB; ++b) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int u = 16 * b + 4 * g + i;
      h[b][i] = a.h0 ? a.h0[sq * U + u] : 0.f;
      cs[b][i] = a.c0 ? a.c0[sq * U + u] : 0.f;
    }
    hb[b] = pack4(h[b]);
  }
  // x_t^T as B operand: B[k = feature 16kt + 4g + j][n = sequence c]
  const XT* xrow = static_cast<const XT*>(a.x) + sq * a.x_seq;
  auto load_x = [&](int t, XR* v) {
    const XT* p = xrow + (int64_t)t * IN;
#pragma unroll
    for (int kt = 0; kt < KT; ++kt) v[kt] = load_row4<XV>(p, 16 * kt + 4 * g, IN);
  };
  const int64_t wv = (int64_t)blockIdx.x * WAVES + (threadIdx.x >> 6);
  SML_DCHECK(wv * 16 < a.B + 15 && seq < (a.B + 15) / 16 * 16);   // inside the padded h / c buffers
  __bf16* cw = a.cseq + wv * T * (int64_t)(UB * 256) + lane * 4;
  // x prefetch PF steps ahead in a register ring; the loop is unrolled by PF so every
  // ring slot is a fixed register set (a rotating copy would wait for the newest load).
  // vmcnt also counts the h / c stores, in issue order: at PF = 2 the loop waited for
  // vmcnt(0) -- every load and store of the previous two steps -- once per trip

  XR xr[PF][KT];
#pragma unroll
  for (int p = 0; p < PF; ++p) load_x(p < T ? p : T - 1, xr[p]);
  auto fwd_step = [&](int t, XR* xin) {
    bf16x4 xb[KT];
#pragma unroll
    for (int kt = 0; kt < KT; ++kt) {
      xb[kt] = row_operand(xin[kt], 16 * kt + 4 * g, IN);
      if constexpr (BX) xb[kt] |= onex[kt];
    }
    load_x(t + PF < T ? t + PF : T - 1, xin);   // in flight for PF steps
    f32x4 z[MT];
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) {
      // z = b + [W ; U]^T . [x_t ; h_{t-1}]^T: the KT + UB K-tiles taken in pairs on the
      // 16x16x32 MFMA (the backward's gate recompute uses the identical pairing)
      z[mt] = BX ? f32x4{0.f, 0.f, 0.f, 0.f} : bias[mt];
      constexpr int NK = KT + UB;
#pragma unroll
      for (int k = 0; k + 1 < NK; k += 2)
        z[mt] = mfma32(k < KT ? wt[mt][k] : ut[mt][k - KT], k + 1 < KT ? wt[mt][k + 1] : ut[mt][k + 1 - KT],
                       k < KT ? xb[k] : hb[k - KT], k + 1 < KT ? xb[k + 1] : hb[k + 1 - KT], z[mt]);
      // odd tile count: the last tile against a zero tile, still on 16x16x32 -- a 16x16x16
      // whose SrcC is a 16x16x32 result miscomputed here (ROCm 7.2, gfx950; measured)
      if constexpr (NK & 1) z[mt] = mfma32(ut[mt][UB - 1], bf16x4{0, 0, 0, 0}, hb[UB - 1], bf16x4{0, 0, 0, 0}, z[mt]);
    }
    // hseq and cseq are padded to whole waves: padding lanes write their own rows,
    // so no store sits under a lane mask (a masked store makes the number of
    // outstanding memory ops path-dependent and the compiler then waits for all)
    __bf16* ht = a.hseq + (seq * T + t) * (int64_t)U + 4 * g;
    __bf16* ct = cw + (int64_t)t * (UB * 256);
#pragma unroll
    for (int b = 0; b < UB; ++b) {
      f32x4 gi, gf, gc, go;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        gi[i] = sigmoid_fast(z[b][i]);
        gf[i] = sigmoid_fast(z[UB + b][i]);
        gc[i] = act_f(ACT, z[2 * UB + b][i]);
        go[i] = sigmoid_fast(z[3 * UB + b][i]);
        cs[b][i] = fmaf(gf[i], cs[b][i], gi[i] * gc[i]);
        h[b][i] = go[i] * act_f(ACT, cs[b][i]);
      }
      hb[b] = pack4(h[b]);
      *reinterpret_cast<bf16x4*>(ct + b * 256) = pack4(cs[b]);
      *reinterpret_cast<bf16x4*>(ht + 16 * b) = hb[b];
    }
  };
  int t0 = 0;
  for (; t0 + PF <= T; t0 += PF) {   // whole groups: straight-line, fixed ring slots
#pragma unroll
    for (int p = 0; p < PF; ++p) fwd_step(t0 + p, xr[p]);
  }
#pragma unroll
  for (int p = 0; p < PF - 1; ++p)    // remainder (T % PF steps)
    if (t0 + p < T) fwd_step(t0 + p, xr[p]);
}

template <int U, int KT, int XV, typename XT>
hipError_t launch_fwd(const FusedFwdArgs& a, hipStream_t st) {
  const int grid = (int)((a.B + 16 * WAVES - 1) / (16 * WAVES));
  auto go = [&](auto bxc, auto pfc) {
    constexpr bool BXV = decltype(bxc)::value;
    constexpr int PF = decltype(pfc)::value;
    if (a.act == ACT_RELU)
      hipLaunchKernelGGL((lstm_fused_fwd_kernel<U, KT, XV, XT, ACT_RELU, BXV, PF>), dim3(grid), dim3(WAVES * 64), 0, st,
                         a);
    else
      hipLaunchKernelGGL((lstm_fused_fwd_kernel<U, KT, XV, XT, ACT_TANH, BXV, PF>), dim3(grid), dim3(WAVES * 64), 0, st,
                         a);
  };
  // x prefetch distance 2 (4 measured within noise and costs registers: profiles/r04)
  if (bias_mode_fwd(a.IN, KT) == BM_BX) go(std::true_type{}, std::integral_constant<int, 2>{});   // as the backward
  else go(std::false_type{}, std::integral_constant<int, 2>{});
  return hipGetLastError();
}

}  // namespace

namespace sml {

hipError_t lstm_fused_fwd_launch(const void* x, bool x_bf16, const float* W, const float* Uw, const float* b,
                                 const float* h0, const float* c0, void* hseq_bf16, void* cseq_bf16, int64_t B, int T,
                                 int IN, int U, int act, int64_t x_seq, hipStream_t stream) {
  FusedFwdArgs a{x, W, Uw, b, h0, c0, (__bf16*)hseq_bf16, (__bf16*)cseq_bf16, B, T, IN, act,
                 x_seq > 0 ? x_seq : (int64_t)T * IN};
  return dispatch(U, IN, row_vec(x, IN, x_bf16 ? 2 : 4), x_bf16, [&](auto u, auto k, auto v, auto xt) {
    using XT = std::remove_const_t<std::remove_pointer_t<decltype(xt)>>;
    return launch_fwd<decltype(u)::value, decltype(k)::value, decltype(v)::value, XT>(a, stream);
  });
}

}  // namespace sml
