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
  // LF (U >= 64): the MT x (KT + UB) weight fragments (160-192 registers) live in LDS, shared by the
  // workgroup's waves and read per step through an opaque lane index; the registers held the scratch
  // spills of the register-fragment build
  constexpr bool LF = U >= 64;
  constexpr int NK = KT + UB;
  __shared__ __attribute__((aligned(16))) bf16x4 lfw[LF ? MT * NK * 64 : 1];
  if constexpr (LF) {
    const int w = threadIdx.x >> 6;
    for (int tile = w; tile < MT * NK; tile += WAVES) {   // tile (mt, k): W^T (k < KT) | U^T
      const int mt = tile / NK, k = tile % NK;
      f32x4 t4;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        if (k < KT) {
          const int f = 16 * k + 4 * g + j;
          t4[j] = BX ? wt_elem_bx(a.W, a.b, G4, a.IN, f, 16 * mt + c) : (f < a.IN ? a.W[(int64_t)f * G4 + 16 * mt + c] : 0.f);
        } else {
          t4[j] = a.Uw[(16 * (k - KT) + 4 * g + j) * G4 + 16 * mt + c];
        }
      }
      lfw[tile * 64 + lane] = pack4(t4);
    }
    __syncthreads();   // before any wave leaves
  }
  const int64_t s0 = ((int64_t)blockIdx.x * WAVES + (threadIdx.x >> 6)) * 16;
  if (s0 >= a.B) return;  // wave-uniform
  const int64_t seq = s0 + c;
  const bool valid = seq < a.B;
  const int64_t sq = valid ? seq : a.B - 1;
  const int IN = a.IN, T = a.T;

  // A fragments: W^T[m = gate][k = feature], U^T[m = gate][k = unit]
  constexpr int MR = LF ? 1 : MT;   // register fragments (none under LF)
  bf16x4 wt[MR][KT], ut[MR][UB];
  f32x4 bias[MT];
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) {
    if constexpr (LF) {
#pragma unroll
      for (int i = 0; i < 4; ++i) bias[mt][i] = BX ? 0.f : a.b[16 * mt + 4 * g + i];
      continue;
    } else {
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
    const int ol = opaque_lane(lane);   // LF: per step, so the fragment reads stay in the loop
    auto fr = [&](int mt, int k) -> bf16x4 {   // A fragment of K tile k (x side k < KT, then h side)
      if constexpr (LF) return lfw[(mt * NK + k) * 64 + ol];
      else return k < KT ? wt[mt][k] : ut[mt][k - KT];
    };
    f32x4 z[MT];
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) {
      // z = b + [W ; U]^T . [x_t ; h_{t-1}]^T: the KT + UB K-tiles taken in pairs on the
      // 16x16x32 MFMA (the backward's gate recompute uses the identical pairing)
      z[mt] = BX ? f32x4{0.f, 0.f, 0.f, 0.f} : bias[mt];
#pragma unroll
      for (int k = 0; k + 1 < NK; k += 2)
        z[mt] = mfma32(fr(mt, k), fr(mt, k + 1), k < KT ? xb[k] : hb[k - KT], k + 1 < KT ? xb[k + 1] : hb[k + 1 - KT],
                       z[mt]);
      // odd tile count: the last tile against a zero tile, still on 16x16x32 -- a 16x16x16
      // whose SrcC is a 16x16x32 result miscomputed here (ROCm 7.2, gfx950; measured)
      if constexpr (NK & 1) z[mt] = mfma32(fr(mt, NK - 1), bf16x4{0, 0, 0, 0}, hb[UB - 1], bf16x4{0, 0, 0, 0}, z[mt]);
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

// ---------------------------------------------------------------------------------------
// Two stacked LSTM layers in ONE forward launch (the seq-50 two-layer stack of BASELINE
// config 3: LSTM(32, relu, seq) -> LSTM(16, relu), LSTM-TensorFlow-IO-Kafka/cardata-v2.py:
// 172-183 with look_back 50).  Each wave carries its 16 sequences through layer 1 AND layer 2
// at every time step: layer 1's h_t leaves the step as the bf16 B operand of layer 2's x.W
// MFMAs straight from registers -- the lane (c, g) holds units 16b + 4g + j of sequence c,
// which IS the B layout of layer 2's K tile b -- so the second layer never re-reads layer 1's
// h sequence from HBM (210 MB per 65 536-window step) and the two recurrences' dependency
// chains interleave in one instruction stream (layer 2 alone issued 13 % of its cycles, 54 %
// dependency stalls: profiles/r04/SUMMARY.md sec. 3).  Layer 1's h / c and layer 2's h / c are
// still saved (bf16) for the backward, which recomputes the gates from them: every operand,
// operand pairing and bias mode is the single-layer kernels', so the saved sequences are
// bit-identical to two lstm_fused_fwd launches.
struct FusedFwd2Args {
  const float* x;                       // [B, T, IN1] fp32 (x_seq elements between sequences)
  const float *W1, *U1, *b1, *W2, *U2, *b2;
  __bf16 *hseq1, *cseq1, *hseq2, *cseq2;   // padded to whole 16-sequence waves
  __bf16* hlast2;                          // HF: layer 2's h_T as [B16, U2] rows (the head's input)
  int64_t B;
  int T, IN1, act1, act2;
  int64_t x_seq;
};

template <int U, int KT, bool BX>
__device__ __forceinline__ void load_layer_frags(const float* W, const float* Uw, const float* b, int IN, int c, int g,
                                                 bf16x4 (&wt)[4 * U / 16][KT], bf16x4 (&ut)[4 * U / 16][U / 16],
                                                 f32x4 (&bias)[4 * U / 16]) {
  constexpr int G4 = 4 * U, MT = G4 / 16, UB = U / 16;
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) {
#pragma unroll
    for (int kt = 0; kt < KT; ++kt) {
      f32x4 t4;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int k = 16 * kt + 4 * g + j;
        t4[j] = BX ? wt_elem_bx(W, b, G4, IN, k, 16 * mt + c) : (k < IN ? W[(int64_t)k * G4 + 16 * mt + c] : 0.f);
      }
      wt[mt][kt] = pack4(t4);
    }
#pragma unroll
    for (int s = 0; s < UB; ++s) {
      f32x4 t4;
#pragma unroll
      for (int j = 0; j < 4; ++j) t4[j] = Uw[(16 * s + 4 * g + j) * G4 + 16 * mt + c];
      ut[mt][s] = pack4(t4);
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) bias[mt][i] = BX ? 0.f : b[16 * mt + 4 * g + i];
  }
}

// z = b + [W ; U]^T . [x_t ; h_{t-1}]^T with the single-layer kernel's K-tile pairing
template <int MT, int KT, int UB, bool BX>
__device__ __forceinline__ void gate_preacts(const bf16x4 (&wt)[MT][KT], const bf16x4 (&ut)[MT][UB],
                                             const f32x4 (&bias)[MT], const bf16x4 (&xb)[KT], const bf16x4 (&hb)[UB],
                                             f32x4 (&z)[MT]) {
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) {
    z[mt] = BX ? f32x4{0.f, 0.f, 0.f, 0.f} : bias[mt];
    constexpr int NK = KT + UB;
#pragma unroll
    for (int k = 0; k + 1 < NK; k += 2)
      z[mt] = mfma32(k < KT ? wt[mt][k] : ut[mt][k - KT], k + 1 < KT ? wt[mt][k + 1] : ut[mt][k + 1 - KT],
                     k < KT ? xb[k] : hb[k - KT], k + 1 < KT ? xb[k + 1] : hb[k + 1 - KT], z[mt]);
    if constexpr (NK & 1) z[mt] = mfma32(ut[mt][UB - 1], bf16x4{0, 0, 0, 0}, hb[UB - 1], bf16x4{0, 0, 0, 0}, z[mt]);
  }
}

// The same sum with the x-side K pair's A fragment (W^T tiles 0 and 1, concatenated) read from LDS
// (fwd2 with two tiles per wave: the registers go to the second tile's state; the x-side MFMAs are
// off the recurrence's critical path, so the read's latency is not).  KT must be 2.
template <int MT, int UB, bool BX>
__device__ __forceinline__ void gate_preacts_lx(const s16x8* lx, int ol, const bf16x4 (&ut)[MT][UB],
                                                const f32x4 (&bias)[MT], const bf16x4 (&xb)[2], const bf16x4 (&hb)[UB],
                                                f32x4 (&z)[MT]) {
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) {
    z[mt] = BX ? f32x4{0.f, 0.f, 0.f, 0.f} : bias[mt];
    z[mt] = mfma32a(lx[mt * 64 + ol], xb[0], xb[1], z[mt]);
    constexpr int NK = 2 + UB;
#pragma unroll
    for (int k = 2; k + 1 < NK; k += 2) z[mt] = mfma32(ut[mt][k - 2], ut[mt][k - 1], hb[k - 2], hb[k - 1], z[mt]);
    if constexpr (NK & 1) z[mt] = mfma32(ut[mt][UB - 1], bf16x4{0, 0, 0, 0}, hb[UB - 1], bf16x4{0, 0, 0, 0}, z[mt]);
  }
}

// Timing probes of the stacked forward (SML_LSTM_FWD2_PROBE, A/B only -- bits 1 and 4 give WRONG
// values and exist to price an instruction class): 1 = sigmoid without the -log2(e) multiply (what a
// pre-scaled W^T would cost), 2 = the three sigmoids of a unit through ONE reciprocal (exact up to
// rounding; z clamped at -20 so the product cannot overflow), 4 = x operand without the column mask /
// bias-column OR; 8 = h stored fragment-native (512 contiguous bytes per wave and tile, as c) instead
// of [B, T, U] rows; 16 / 32 = h / c not stored (upper bounds of the store cost).
// ht / ct: wave-uniform bases of the step's h / c stores, hoff / coff: this lane's byte offsets (the
// stores take the global_store saddr form: no 64-bit per-lane pointers carried through the time loop)
template <int U, int ACT, int PROBE>
__device__ __forceinline__ void cell_update_p(const f32x4 (&z)[4 * U / 16], f32x4 (&h)[U / 16], f32x4 (&cs)[U / 16],
                                              bf16x4 (&hb)[U / 16], char* ht, unsigned hoff, char* ct, unsigned coff) {
  constexpr int UB = U / 16;
#pragma unroll
  for (int b = 0; b < UB; ++b) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      float gi, gf, go;
      if constexpr (PROBE & 2) {
        const float A = 1.0f + __expf(-fmaxf(z[b][i], -20.f));
        const float Bf = 1.0f + __expf(-fmaxf(z[UB + b][i], -20.f));
        const float C = 1.0f + __expf(-fmaxf(z[3 * UB + b][i], -20.f));
        const float AB = A * Bf;
        const float r = rcp_fast(AB * C);
        gi = r * (Bf * C);
        gf = r * (A * C);
        go = r * AB;
      } else if constexpr (PROBE & 1) {
        gi = rcp_fast(1.0f + __builtin_amdgcn_exp2f(-z[b][i]));
        gf = rcp_fast(1.0f + __builtin_amdgcn_exp2f(-z[UB + b][i]));
        go = rcp_fast(1.0f + __builtin_amdgcn_exp2f(-z[3 * UB + b][i]));
      } else {
        gi = sigmoid_fast(z[b][i]);
        gf = sigmoid_fast(z[UB + b][i]);
        go = sigmoid_fast(z[3 * UB + b][i]);
      }
      const float gc = act_f(ACT, z[2 * UB + b][i]);
      cs[b][i] = fmaf(gf, cs[b][i], gi * gc);
      h[b][i] = go * act_f(ACT, cs[b][i]);
    }
    hb[b] = pack4(h[b]);
    if constexpr (!(PROBE & 32)) *reinterpret_cast<bf16x4*>(ct + coff + b * 512) = pack4(cs[b]);
    if constexpr (!(PROBE & 16)) *reinterpret_cast<bf16x4*>(ht + hoff + ((PROBE & 8) ? b * 512 : 32 * b)) = hb[b];
  }
}

template <int U, int ACT>
__device__ __forceinline__ void cell_update(const f32x4 (&z)[4 * U / 16], f32x4 (&h)[U / 16], f32x4 (&cs)[U / 16],
                                            bf16x4 (&hb)[U / 16], __bf16* ht, __bf16* ct) {
  constexpr int UB = U / 16;
#pragma unroll
  for (int b = 0; b < UB; ++b) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const float gi = sigmoid_fast(z[b][i]);
      const float gf = sigmoid_fast(z[UB + b][i]);
      const float gc = act_f(ACT, z[2 * UB + b][i]);
      const float go = sigmoid_fast(z[3 * UB + b][i]);
      cs[b][i] = fmaf(gf, cs[b][i], gi * gc);
      h[b][i] = go * act_f(ACT, cs[b][i]);
    }
    hb[b] = pack4(h[b]);
    *reinterpret_cast<bf16x4*>(ct + b * 256) = pack4(cs[b]);
    *reinterpret_cast<bf16x4*>(ht + 16 * b) = hb[b];
  }
}

// NT: 16-sequence tiles per wave (2: two independent recurrences interleaved in one instruction
// stream, sharing the weight fragments -- 2 048 waves for the 4 096 tiles of B = 65 536, one residency
// round at two waves per SIMD instead of two rounds of one-tile waves).  The saved layouts are the
// one-tile kernel's (cseq indexed by 16-sequence tile), so the backward is unchanged.
// HF: h1 / h2 stored fragment-native ([B/16, T, U/16, 64 lanes, 4], like c: one 512-byte store per
// wave and tile instead of 16 row pieces 64 / 32 bytes long) for the backward kernels' fragment mode
// (lstm_fused.hip FR), and layer 2's h_T once more as rows for the head.
template <int U1, int KT1, int XV, int ACT1, bool BX1, int U2, int ACT2, int PF = 2, int NT = 1, int PROBE = 0,
          bool HF = false>
__global__ __launch_bounds__(WAVES * 64, 1) void lstm_fused_fwd2_kernel(FusedFwd2Args a) {
  constexpr int MT1 = 4 * U1 / 16, UB1 = U1 / 16, MT2 = 4 * U2 / 16, UB2 = U2 / 16, KT2 = UB1;
  const int lane = threadIdx.x & 63, c = lane & 15, g = lane >> 4;
  // wave-uniform (SGPR) tile index: every per-step address is an SGPR base plus a per-lane 32-bit offset
  const int64_t wv0 = ((int64_t)blockIdx.x * WAVES + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6)) * NT;
  const int IN1 = a.IN1, T = a.T;
  // NT = 2: the x-side A fragments of both layers live in LDS (shared by the workgroup's waves)
  constexpr bool LX = NT > 1;
  static_assert(!LX || (KT1 == 2 && KT2 == 2), "LDS x fragments: one K pair per layer");
  __shared__ __attribute__((aligned(16))) s16x8 lx1[LX ? MT1 * 64 : 1], lx2[LX ? MT2 * 64 : 1];

  bf16x4 wt1[MT1][KT1], ut1[MT1][UB1], wt2[MT2][KT2], ut2[MT2][UB2];
  f32x4 bias1[MT1], bias2[MT2];
  load_layer_frags<U1, KT1, BX1>(a.W1, a.U1, a.b1, IN1, c, g, wt1, ut1, bias1);
  load_layer_frags<U2, KT2, false>(a.W2, a.U2, a.b2, U1, c, g, wt2, ut2, bias2);   // x = h1: no spare columns
  if constexpr (LX) {
    if (threadIdx.x < 64) {
#pragma unroll
      for (int mt = 0; mt < MT1; ++mt) lx1[mt * 64 + lane] = cat8(wt1[mt][0], wt1[mt][1]);
#pragma unroll
      for (int mt = 0; mt < MT2; ++mt) lx2[mt * 64 + lane] = cat8(wt2[mt][0], wt2[mt][1]);
    }
    __syncthreads();   // before any wave leaves
  }
  if (wv0 * 16 >= a.B) return;  // wave-uniform
  bf16x4 onex[KT1];
  u32x2_t xkeep[KT1];   // the x operand's kept columns (row_operand_k: one v_bfi per register)
#pragma unroll
  for (int kt = 0; kt < KT1; ++kt) {
    onex[kt] = BX1 ? ones_at_bias(kt, g, IN1) : bf16x4{0, 0, 0, 0};
    xkeep[kt] = row_keep(16 * kt + 4 * g, IN1);
  }
  f32x4 h1[NT][UB1], c1[NT][UB1], h2[NT][UB2], c2[NT][UB2];
  bf16x4 hb1[NT][UB1], hb2[NT][UB2];
  int xo[NT][KT1][4];   // per-lane byte offsets of the x row pieces (tile row 0, step 0 = the uniform base)
#pragma unroll
  for (int k = 0; k < NT; ++k) {
#pragma unroll
    for (int b = 0; b < UB1; ++b) {
      h1[k][b] = c1[k][b] = f32x4{0.f, 0.f, 0.f, 0.f};
      hb1[k][b] = bf16x4{0, 0, 0, 0};
    }
#pragma unroll
    for (int b = 0; b < UB2; ++b) {
      h2[k][b] = c2[k][b] = f32x4{0.f, 0.f, 0.f, 0.f};
      hb2[k][b] = bf16x4{0, 0, 0, 0};
    }
    // a tile past B (the last wave's second tile) runs on clamped rows and stores into the
    // buffers' padding (allocated to whole waves of NT tiles)
    const int64_t wv = wv0 + k;
    const int64_t seq = wv * 16 + c;
    const int cl = seq < a.B ? c : (int)(a.B - 1 - wv * 16);   // rows past B read row B - 1 (< 0: idle tile)
    SML_DCHECK(seq < (a.B + 16 * NT - 1) / (16 * NT) * (16 * NT));
#pragma unroll
    for (int kt = 0; kt < KT1; ++kt)
#pragma unroll
      for (int j = 0; j < 4; ++j) {   // clamped in-row columns, as load_row4
        const int k0 = 16 * kt + 4 * g + (XV == 2 ? (j & 2) : (XV == 4 ? 0 : j));
        xo[k][kt][j] = (int)((cl * a.x_seq + (k0 < IN1 ? k0 : 0)) * 4);
      }
  }
  // byte offsets of this lane in the h / c stores: fragment-native 8 bytes per lane, rows 2 x (T U) per
  // sequence + 8 per unit group
  const unsigned fo = lane * 8, ro1 = (c * T * U1 + 4 * g) * 2, ro2 = (c * T * U2 + 4 * g) * 2;
  auto tile_row = [&](int k) { return (wv0 + k) * 16; };   // uniform
  auto load_x = [&](int t, f32x4 (*v)[KT1]) {
#pragma unroll
    for (int k = 0; k < NT; ++k) {
      const char* x0 = reinterpret_cast<const char*>(a.x) + (tile_row(k) * a.x_seq + (int64_t)t * IN1) * 4;
#pragma unroll
      for (int kt = 0; kt < KT1; ++kt) {
        if constexpr (XV == 4) {
          v[k][kt] = *reinterpret_cast<const f32x4*>(x0 + xo[k][kt][0]);
        } else if constexpr (XV == 2) {
          const f32x2_t lo = *reinterpret_cast<const f32x2_t*>(x0 + xo[k][kt][0]);
          const f32x2_t hi = *reinterpret_cast<const f32x2_t*>(x0 + xo[k][kt][2]);
          v[k][kt] = f32x4{lo[0], lo[1], hi[0], hi[1]};
        } else {
#pragma unroll
          for (int j = 0; j < 4; ++j) v[k][kt][j] = *reinterpret_cast<const float*>(x0 + xo[k][kt][j]);
        }
      }
    }
  };
  // step t's store bases (uniform): c fragment-native; h fragment-native (HF / PROBE 8) or rows
  auto cbase = [&](__bf16* base, int k, int t, int ub) {
    return reinterpret_cast<char*>(base) + ((wv0 + k) * T + t) * (int64_t)(ub * 512);
  };
  auto hbase = [&](__bf16* base, int k, int t, int u, int ub, bool frag) {
    return frag ? cbase(base, k, t, ub) : reinterpret_cast<char*>(base) + (tile_row(k) * T + t) * (int64_t)(u * 2);
  };
  f32x4 xr[PF][NT][KT1];
#pragma unroll
  for (int p = 0; p < PF; ++p) load_x(p < T ? p : T - 1, xr[p]);
  auto step = [&](int t, f32x4 (*xin)[KT1]) {
    bf16x4 xb[NT][KT1];
#pragma unroll
    for (int k = 0; k < NT; ++k)
#pragma unroll
      for (int kt = 0; kt < KT1; ++kt) {
        if constexpr (PROBE & 4) {
          xb[k][kt] = pack4(xin[k][kt]);
        } else {
          xb[k][kt] = row_operand_k(xin[k][kt], xkeep[kt], onex[kt]);
        }
      }
    load_x(t + PF < T ? t + PF : T - 1, xin);
    const int ol = opaque_lane(lane);   // per step: the LDS fragment reads stay in the loop
    f32x4 z1[NT][MT1];
#pragma unroll
    for (int k = 0; k < NT; ++k) {
      if constexpr (LX) gate_preacts_lx<MT1, UB1, BX1>(lx1, ol, ut1, bias1, xb[k], hb1[k], z1[k]);
      else gate_preacts<MT1, KT1, UB1, BX1>(wt1, ut1, bias1, xb[k], hb1[k], z1[k]);
    }
    constexpr bool HFR = (PROBE & 8) || HF;
#pragma unroll
    for (int k = 0; k < NT; ++k)
      cell_update_p<U1, ACT1, PROBE | (HF ? 8 : 0)>(z1[k], h1[k], c1[k], hb1[k], hbase(a.hseq1, k, t, U1, UB1, HFR),
                                                     HFR ? fo : ro1, cbase(a.cseq1, k, t, UB1), fo);
    // layer 2: x_t = layer 1's h_t, already the B operand (hb1)
    f32x4 z2[NT][MT2];
#pragma unroll
    for (int k = 0; k < NT; ++k) {
      if constexpr (LX) gate_preacts_lx<MT2, UB2, false>(lx2, ol, ut2, bias2, hb1[k], hb2[k], z2[k]);
      else gate_preacts<MT2, KT2, UB2, false>(wt2, ut2, bias2, hb1[k], hb2[k], z2[k]);
    }
#pragma unroll
    for (int k = 0; k < NT; ++k)
      cell_update_p<U2, ACT2, PROBE | (HF ? 8 : 0)>(z2[k], h2[k], c2[k], hb2[k], hbase(a.hseq2, k, t, U2, UB2, HFR),
                                                     HFR ? fo : ro2, cbase(a.cseq2, k, t, UB2), fo);
  };
  int t0 = 0;
  for (; t0 + PF <= T; t0 += PF) {
#pragma unroll
    for (int p = 0; p < PF; ++p) step(t0 + p, xr[p]);
  }
#pragma unroll
  for (int p = 0; p < PF - 1; ++p)
    if (t0 + p < T) step(t0 + p, xr[p]);
  if constexpr (HF) {   // h2 of the last step, as rows (the Dense head reads h_T)
#pragma unroll
    for (int k = 0; k < NT; ++k) {
      const int64_t seq = (wv0 + k) * 16 + c;
#pragma unroll
      for (int b = 0; b < UB2; ++b) *reinterpret_cast<bf16x4*>(a.hlast2 + seq * U2 + 16 * b + 4 * g) = hb2[k][b];
    }
  }
}

inline int fwd2_tiles() {   // SML_LSTM_FWD2_NT=1|2: 16-sequence tiles per wave of the stacked forward
  static const int v = [] {
    const char* e = std::getenv("SML_LSTM_FWD2_NT");
    return e && e[0] == '2' ? 2 : 1;   // 2 measured 0.4-0.9 % slower (profiles/r05/lstm/ab_fwd2_nt.txt)
  }();
  return v;
}

template <int XV>
hipError_t launch_fwd2(const FusedFwd2Args& a, hipStream_t st) {
  const bool bx = bias_mode_fwd(a.IN1, 2) == BM_BX;
  if (bias_mode_fwd(32, 2) == BM_BX) return hipErrorInvalidValue;   // layer 2 (IN 32) has no spare columns
  const int nt = fwd2_tiles();
  const int grid = (int)((a.B + 16 * WAVES * nt - 1) / (16 * WAVES * nt));
  static const int probe = [] {
    const char* e = std::getenv("SML_LSTM_FWD2_PROBE");
    return e ? std::atoi(e) : 0;
  }();
  if (probe && nt == 1 && XV == 2 && bx && a.act1 == ACT_RELU && a.act2 == ACT_RELU && a.hlast2 == nullptr) {   // the bench shape only
    auto go = [&](auto k) {
      hipLaunchKernelGGL((lstm_fused_fwd2_kernel<32, 2, XV, ACT_RELU, true, 16, ACT_RELU, 2, 1, decltype(k)::value>),
                         dim3(grid), dim3(WAVES * 64), 0, st, a);
    };
    if (probe == 1) go(std::integral_constant<int, 1>{});
    else if (probe == 2) go(std::integral_constant<int, 2>{});
    else if (probe == 4) go(std::integral_constant<int, 4>{});
    else if (probe == 8) go(std::integral_constant<int, 8>{});
    else if (probe == 16) go(std::integral_constant<int, 16>{});
    else if (probe == 32) go(std::integral_constant<int, 32>{});
    else if (probe == 48) go(std::integral_constant<int, 48>{});
    else go(std::integral_constant<int, 5>{});
    return hipGetLastError();
  }
#define SML_F2(A1, A2, BXV)                                                                                  \
  do {                                                                                                       \
    if (a.hlast2 != nullptr)                                                                                 \
      hipLaunchKernelGGL((lstm_fused_fwd2_kernel<32, 2, XV, A1, BXV, 16, A2, 2, 1, 0, true>), dim3(grid),   \
                         dim3(WAVES * 64), 0, st, a);                                                        \
    else if (nt == 2)                                                                                        \
      hipLaunchKernelGGL((lstm_fused_fwd2_kernel<32, 2, XV, A1, BXV, 16, A2, 1, 2>), dim3(grid), dim3(WAVES * 64), \
                         0, st, a);                                                                          \
    else                                                                                                     \
      hipLaunchKernelGGL((lstm_fused_fwd2_kernel<32, 2, XV, A1, BXV, 16, A2, 2, 1>), dim3(grid), dim3(WAVES * 64), \
                         0, st, a);                                                                          \
  } while (0)
  if (a.act1 == ACT_RELU && a.act2 == ACT_RELU) {
    if (bx) SML_F2(ACT_RELU, ACT_RELU, true);
    else SML_F2(ACT_RELU, ACT_RELU, false);
  } else if (a.act1 == ACT_TANH && a.act2 == ACT_TANH) {
    if (bx) SML_F2(ACT_TANH, ACT_TANH, true);
    else SML_F2(ACT_TANH, ACT_TANH, false);
  } else {
    return hipErrorInvalidValue;   // mixed activations: two single-layer launches
  }
#undef SML_F2
  return hipGetLastError();
}

}  // namespace

namespace sml {

int lstm_fused_fwd2_rows(int64_t B) {   // sequences the h / c buffers of the stacked forward must hold
  const int64_t per = 16 * fwd2_tiles();
  return (int)((B + per - 1) / per * per);
}

bool lstm_fused_fwd2_supported(int IN1, int U1, int U2, int act1, int act2) {
  return U1 == 32 && U2 == 16 && IN1 >= 1 && IN1 <= 32 && act1 == act2 && (act1 == ACT_RELU || act1 == ACT_TANH);
}

hipError_t lstm_fused_fwd2_launch(const float* x, const float* W1, const float* U1, const float* b1, const float* W2,
                                  const float* U2, const float* b2, void* hseq1, void* cseq1, void* hseq2, void* cseq2,
                                  void* hlast2, int64_t B, int T, int IN1, int act1, int act2, int64_t x_seq,
                                  hipStream_t stream) {
  FusedFwd2Args a{x, W1, U1, b1, W2, U2, b2, (__bf16*)hseq1, (__bf16*)cseq1, (__bf16*)hseq2, (__bf16*)cseq2,
                  (__bf16*)hlast2, B, T, IN1, act1, act2, x_seq > 0 ? x_seq : (int64_t)T * IN1};
  const int xv = row_vec(x, IN1, 4);
  if (xv == 4) return launch_fwd2<4>(a, stream);
  if (xv == 2) return launch_fwd2<2>(a, stream);
  return launch_fwd2<1>(a, stream);
}


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
