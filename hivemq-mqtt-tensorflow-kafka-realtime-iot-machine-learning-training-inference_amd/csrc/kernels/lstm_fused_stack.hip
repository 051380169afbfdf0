// sml-build: agpr-accumulators
//
// Backward of two stacked LSTM layers in ONE launch: the seq-50 two-layer stack of BASELINE
// config 3 (LSTM(32, seq) -> LSTM(16) -> Dense(18); LSTM-TensorFlow-IO-Kafka/cardata-v2.py:
// 172-209 at look_back 50).  lstm_fused.hip runs one launch per layer: layer 2's backward
// writes dX -- layer 1's incoming dh, 65 536 x 50 x 32 bf16 = 210 MB per step -- and layer
// 1's backward reads it back; both read the layer-1 h sequence (layer 2 as its x, layer 1 as
// its h_{t-1}).  Here every wave walks time backwards through BOTH layers for its 16
// sequences: at step t, layer 2's BPTT step produces dX_t in registers, in the C layout of
// layer 1's dh_t (lane (c, g): features 16kt + 4g + i of sequence c = units 16b + 4g + i), and
// layer 1's step t consumes it at once.  h1_{t-1}, read as layer 1's h_{t-1} at step t, is
// carried in registers to be layer 2's x at step t - 1: each saved tensor is read once.
//
// Per layer the step is lstm_fused.hip's one-step loop (gate recompute with the forward's
// operands and pairing, dz, the dh chain on 16x16x32 MFMAs, weight gradients contracted one
// step behind through LDS transposes into AGPR accumulators, one slab per workgroup over a
// persistent grid).  dX is rounded to bf16 before layer 1 uses it, exactly as the two-launch
// path stores it, so layer 1 sees the same dh.  Layer 1 takes the bias-column mode (its 18
// inputs leave two spare K slots), layer 2 (32 inputs = h1) the plain one: the forward's.
// Layer 2 runs one step AHEAD of layer 1 (its step t - 1 does not depend on layer 1's step t),
// so both layers' work sits in one loop body.
//
// Measured (MI355X, seq-50 config, profiles/r05/lstm/ab_r05g_bwd2.txt): correct, but SLOWER than
// the two launches -- 501 us vs 243 + 236 us; 88.8 vs 91.7 M windows/s.  Both layers' registers
// (256 VGPR + 221 AGPR) leave one wave per SIMD to carry two serial dependency chains, where the
// two-launch path runs layer 2 at two waves per SIMD and layer 1 on its two-step pair loop; the
// 420 MB of dX traffic saved is worth less than that.  Opt-in (SML_LSTM_BWD2=1) for the A/B.
#include <cstdlib>

#include "lstm_fused_impl.h"

using namespace sml;
using namespace sml_lstm;

namespace {

// One layer's backward state and step (lstm_fused.hip's kernel body as a device object).
template <int U, int KT, typename XT, int ACT, bool DX, int RF, int BM>
struct BwdLayer {
  static constexpr bool BX = BM == BM_BX, DB = BM != BM_PLAIN;
  using XR = typename RowRaw<XT>::type;
  static constexpr int G4 = 4 * U, MT = G4 / 16, UB = U / 16, LDW = 16 * KT;
  static constexpr int S = G4 * (LDW + U + 1);
  static constexpr int NKT = KT + UB, NTR = MT + KT + UB, KTN = KT;
  static constexpr bool RFU = RF & 1, RFW = RF & 2, RFX = DX && (RF & 4);

  bf16x4* wfwd;   // [MT * NKT][64]  W^T | U^T, forward orientation (gate recompute)
  bf16x4* ufl;    // [UB * MT][64]   U (dh chain)
  bf16x4* wfl;    // [KT * MT][64]   W (dX)
  float* sbias;   // [G4]
  float* slab;    // [S]
  char* scr;      // this wave's transpose scratch [NTR][512]
  int IN;

  bf16x4 rfw[RFW ? MT * NKT : 1], rfu[RFU ? UB * MT : 1], rfx[RFX ? KT * MT : 1];
  f32x4 accW[MT][KT], accU[MT][UB], accb[MT];
  f32x4 dhr[UB], dcn[UB], ctc[UB];
  bf16x4 pdz[MT], pxb[KT], phb[UB];
  bf16x4 onex[KT];

  // fragments into LDS (every thread of the workgroup takes part)
  __device__ void stage(const float* W, const float* Uw, const float* b, int w, int lane, int c, int g) {
    for (int i = threadIdx.x; i < G4; i += WAVES * 64) sbias[i] = b[i];
    for (int tile = w; tile < MT * NKT; tile += WAVES) {
      const int mt = tile / NKT, k = tile % NKT;
      f32x4 t4;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        if (k < KT) {
          const int f = 16 * k + 4 * g + j;
          t4[j] = BX ? wt_elem_bx(W, b, G4, IN, f, 16 * mt + c) : (f < IN ? W[(int64_t)f * G4 + 16 * mt + c] : 0.f);
        } else {
          t4[j] = Uw[(16 * (k - KT) + 4 * g + j) * G4 + 16 * mt + c];
        }
      }
      wfwd[tile * 64 + lane] = pack4(t4);
    }
    for (int tile = w; tile < UB * MT; tile += WAVES) {
      const int bb = tile / MT, kt = tile % MT;
      f32x4 t4;
#pragma unroll
      for (int j = 0; j < 4; ++j) t4[j] = Uw[(16 * bb + c) * G4 + 16 * kt + 4 * g + j];
      ufl[tile * 64 + lane] = pack4(t4);
    }
    if constexpr (DX) {
      for (int tile = w; tile < KT * MT; tile += WAVES) {
        const int kt = tile / MT, mt = tile % MT;
        const int f = 16 * kt + c;
        f32x4 t4;
#pragma unroll
        for (int j = 0; j < 4; ++j) t4[j] = f < IN ? W[(int64_t)f * G4 + 16 * mt + 4 * g + j] : 0.f;
        wfl[tile * 64 + lane] = pack4(t4);
      }
    }
  }

  __device__ void init_regs(int lane, int g) {
    const f32x4 zero4 = {0.f, 0.f, 0.f, 0.f};
    if constexpr (RFW) {
#pragma unroll
      for (int i = 0; i < MT * NKT; ++i) rfw[i] = wfwd[i * 64 + lane];
    }
    if constexpr (RFU) {
#pragma unroll
      for (int i = 0; i < UB * MT; ++i) rfu[i] = ufl[i * 64 + lane];
    }
    if constexpr (RFX) {
#pragma unroll
      for (int i = 0; i < KT * MT; ++i) rfx[i] = wfl[i * 64 + lane];
    }
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) {
#pragma unroll
      for (int kt = 0; kt < KT; ++kt) accW[mt][kt] = zero4;
#pragma unroll
      for (int kb = 0; kb < UB; ++kb) accU[mt][kb] = zero4;
      accb[mt] = zero4;
    }
#pragma unroll
    for (int kt = 0; kt < KT; ++kt) onex[kt] = DB ? ones_at_bias(kt, g, IN) : bf16x4{0, 0, 0, 0};
  }

  // a fresh recurrence and weight-gradient pipeline per tile (the accumulators carry on);
  // cw: this wave's cell-state rows (fragment-native, lane offset included)
  __device__ void begin(const __bf16* cw, int T, bool active) {
    const f32x4 zero4 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int b = 0; b < UB; ++b) {
      dhr[b] = dcn[b] = zero4;
      ctc[b] = active ? unpack4(ld_bf16x4(cw + (int64_t)(T - 1) * (UB * 256) + b * 256)) : zero4;
    }
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) pdz[mt] = pack4(zero4);
#pragma unroll
    for (int kt = 0; kt < KT; ++kt) pxb[kt] = pack4(zero4);
#pragma unroll
    for (int s = 0; s < UB; ++s) phb[s] = pack4(zero4);
  }

  // the previous step's weight gradients: dz^T (A) against x / h (B) over the 16 sequences
  __device__ void wgrad(int c, int g) {
    bf16x4 hB[UB], xB[KT];
#pragma unroll
    for (int kb = 0; kb < UB; ++kb) hB[kb] = lds_transpose(phb[kb], scr + (MT + KT + kb) * 512, c, g);
#pragma unroll
    for (int kt = 0; kt < KT; ++kt) xB[kt] = lds_transpose(pxb[kt], scr + (MT + kt) * 512, c, g);
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) {
      const bf16x4 adz = lds_transpose(pdz[mt], scr + mt * 512, c, g);
#pragma unroll
      for (int kt = 0; kt < KT; ++kt) accW[mt][kt] = mfma16(adz, xB[kt], accW[mt][kt]);
#pragma unroll
      for (int kb = 0; kb < UB; ++kb) accU[mt][kb] = mfma16(adz, hB[kb], accU[mt][kb]);
    }
  }

  // one BPTT step: x_t, h_{t-1}, c_{t-1} of this lane's sequence, the incoming dh_t (fp32 values
  // of bf16 numbers), take_dh = whether it counts; dX_t^T into dxo (DX)
  __device__ void step(const XR (&xt)[KT], const bf16x4 (&hp)[UB], const bf16x4 (&cprev)[UB],
                       const f32x4 (&dhi)[UB], bool take_dh, int lane, int c, int g, f32x4 (&dxo)[KT]) {
    const f32x4 zero4 = {0.f, 0.f, 0.f, 0.f};
    const int ol = opaque_lane(lane);
    auto fw = [&](int i) { if constexpr (RFW) return rfw[i]; else return wfwd[i * 64 + ol]; };
    auto fu = [&](int i) { if constexpr (RFU) return rfu[i]; else return ufl[i * 64 + ol]; };
    auto fx = [&](int i) { if constexpr (RFX) return rfx[i]; else return wfl[i * 64 + ol]; };
    bf16x4 xb[KT], hb[UB];
#pragma unroll
    for (int kt = 0; kt < KT; ++kt) {
      xb[kt] = row_operand(xt[kt], 16 * kt + 4 * g, IN);
      if constexpr (DB) xb[kt] |= onex[kt];
    }
#pragma unroll
    for (int s = 0; s < UB; ++s) hb[s] = hp[s];
    f32x4 z[MT];
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) {
      z[mt] = BX ? zero4 : *reinterpret_cast<const f32x4*>(sbias + 16 * mt + (ol >> 4) * 4);
#pragma unroll
      for (int k = 0; k + 1 < NKT; k += 2)
        z[mt] = mfma32(fw(mt * NKT + k), fw(mt * NKT + k + 1), k < KT ? xb[k] : hb[k - KT],
                       k + 1 < KT ? xb[k + 1] : hb[k + 1 - KT], z[mt]);
      if constexpr (NKT & 1)
        z[mt] = mfma32(fw(mt * NKT + NKT - 1), bf16x4{0, 0, 0, 0}, hb[UB - 1], bf16x4{0, 0, 0, 0}, z[mt]);
    }
    wgrad(c, g);   // the previous (later) step's weight gradients, between the MFMA and VALU work
    f32x4 dzt[MT];
#pragma unroll
    for (int b = 0; b < UB; ++b) {
      const f32x4 cp = unpack4(cprev[b]);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float gi = sigmoid_fast(z[b][i]), gf = sigmoid_fast(z[UB + b][i]);
        const float gc = act_f(ACT, z[2 * UB + b][i]), go = sigmoid_fast(z[3 * UB + b][i]);
        const float dh = (take_dh ? dhi[b][i] : 0.f) + dhr[b][i];
        const float ct = ctc[b][i];
        const float ac = act_f(ACT, ct);
        const float dhgo = dh * go;
        const float dc = ACT == ACT_RELU ? (ct > 0.f ? dcn[b][i] + dhgo : dcn[b][i])
                                         : fmaf(dhgo, fmaf(-ac, ac, 1.f), dcn[b][i]);
        const float di = dc * gi;
        const float df = dc * gf;
        dzt[b][i] = (dc * gc) * fmaf(-gi, gi, gi);
        dzt[UB + b][i] = fmaf(-df, gf, df) * cp[i];
        dzt[2 * UB + b][i] = ACT == ACT_RELU ? (gc > 0.f ? di : 0.f) : di * fmaf(-gc, gc, 1.f);
        dzt[3 * UB + b][i] = (dh * ac) * fmaf(-go, go, go);
        dcn[b][i] = df;
      }
      ctc[b] = cp;
    }
    bf16x4 dzb[MT];
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) {
      dzb[mt] = pack4(dzt[mt]);
      if constexpr (!DB) accb[mt] += dzt[mt];
    }
#pragma unroll
    for (int b = 0; b < UB; ++b) {
      f32x4 acc = zero4;
#pragma unroll
      for (int kt = 0; kt < MT; kt += 2) acc = mfma32(fu(b * MT + kt), fu(b * MT + kt + 1), dzb[kt], dzb[kt + 1], acc);
      dhr[b] = acc;
    }
    if constexpr (DX) {
#pragma unroll
      for (int kt = 0; kt < KT; ++kt) {
        f32x4 acc = zero4;
#pragma unroll
        for (int mt = 0; mt < MT; mt += 2)
          acc = mfma32(fx(kt * MT + mt), fx(kt * MT + mt + 1), dzb[mt], dzb[mt + 1], acc);
        dxo[kt] = acc;
      }
    }
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) pdz[mt] = dzb[mt];
#pragma unroll
    for (int kt = 0; kt < KT; ++kt) pxb[kt] = xb[kt];
#pragma unroll
    for (int s = 0; s < UB; ++s) phb[s] = hb[s];
  }

  // the 4 waves add their accumulators into the workgroup slab in a fixed order (every
  // thread of the workgroup calls this), then the slab goes out
  __device__ void write_slab(bool any_active, int w, int c, int g, float* out) {
    if constexpr (!DB) {
#pragma unroll
      for (int mt = 0; mt < MT; ++mt)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          float v = accb[mt][i];
#pragma unroll
          for (int o = 1; o < 16; o <<= 1) v += __shfl_xor(v, o, 64);
          accb[mt][i] = v;
        }
    }
    for (int turn = 0; turn < WAVES; ++turn) {
      __syncthreads();
      if (turn == w && any_active) {
#pragma unroll
        for (int mt = 0; mt < MT; ++mt)
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const int m = 16 * mt + 4 * g + i;
#pragma unroll
            for (int kt = 0; kt < KT; ++kt) slab[m * LDW + 16 * kt + c] += accW[mt][kt][i];
#pragma unroll
            for (int kb = 0; kb < UB; ++kb) slab[G4 * LDW + m * U + 16 * kb + c] += accU[mt][kb][i];
            if (!DB && c == 0) slab[G4 * LDW + G4 * U + m] += accb[mt][i];
          }
      }
    }
    __syncthreads();
    if constexpr (DB) {
      for (int m = threadIdx.x; m < G4; m += WAVES * 64) {
        slab[G4 * LDW + G4 * U + m] = slab[m * LDW + IN];
        slab[m * LDW + IN] = 0.f;
        if (IN + 1 < LDW) slab[m * LDW + IN + 1] = 0.f;
      }
      __syncthreads();
    }
    for (int i = threadIdx.x; i < S; i += WAVES * 64) out[i] = slab[i];
  }
};

struct Bwd2Args {
  const float* x;          // [B, T, IN1] fp32, x_seq elements between sequences
  const __bf16* h1;        // [B, T, 32] bf16 (layer 1's output = layer 2's x)
  const __bf16* c1;        // layer 1's cell state, fragment-native (lstm_fused_fwd)
  const __bf16* h2;        // [B, T, 16]
  const __bf16* c2;
  const __bf16* dh2;       // [B, 16] (h_T only) or [B, T, 16]
  const float *W1, *U1, *b1, *W2, *U2, *b2;
  float* partials1;        // [gridDim.x, S1]
  float* partials2;        // [gridDim.x, S2]
  int64_t B, x_seq;
  int T, IN1, dh2_last_only;
};

template <int XV1, int ACT, int RF1>
__global__ __launch_bounds__(WAVES * 64, 1) void lstm_fused_bwd2_kernel(Bwd2Args a) {
  using L1T = BwdLayer<32, 2, float, ACT, false, RF1, BM_BX>;
  using L2T = BwdLayer<16, 2, __bf16, ACT, true, 0, BM_PLAIN>;
  __shared__ __attribute__((aligned(16))) char scratch1[WAVES][L1T::NTR * 512];
  __shared__ __attribute__((aligned(16))) char scratch2[WAVES][L2T::NTR * 512];
  __shared__ __attribute__((aligned(16))) float slab1[L1T::S];
  __shared__ __attribute__((aligned(16))) float slab2[L2T::S];
  __shared__ __attribute__((aligned(16))) bf16x4 wfwd1[L1T::MT * L1T::NKT * 64];
  __shared__ __attribute__((aligned(16))) bf16x4 ufl1[L1T::UB * L1T::MT * 64];
  __shared__ __attribute__((aligned(16))) bf16x4 wfwd2[L2T::MT * L2T::NKT * 64];
  __shared__ __attribute__((aligned(16))) bf16x4 ufl2[L2T::UB * L2T::MT * 64];
  __shared__ __attribute__((aligned(16))) bf16x4 wfl2[L2T::KTN * L2T::MT * 64];
  __shared__ __attribute__((aligned(16))) float sbias1[L1T::G4];
  __shared__ __attribute__((aligned(16))) float sbias2[L2T::G4];
  const int lane = threadIdx.x & 63, c = lane & 15, g = lane >> 4;
  const int w = threadIdx.x >> 6;
  const int T = a.T;
  L1T L1;
  L2T L2;
  L1.wfwd = wfwd1; L1.ufl = ufl1; L1.wfl = nullptr; L1.sbias = sbias1; L1.slab = slab1; L1.scr = scratch1[w];
  L1.IN = a.IN1;
  L2.wfwd = wfwd2; L2.ufl = ufl2; L2.wfl = wfl2; L2.sbias = sbias2; L2.slab = slab2; L2.scr = scratch2[w];
  L2.IN = 32;
  for (int i = threadIdx.x; i < L1T::S; i += WAVES * 64) slab1[i] = 0.f;
  for (int i = threadIdx.x; i < L2T::S; i += WAVES * 64) slab2[i] = 0.f;
  L1.stage(a.W1, a.U1, a.b1, w, lane, c, g);
  L2.stage(a.W2, a.U2, a.b2, w, lane, c, g);
  __syncthreads();
  L1.init_regs(lane, g);
  L2.init_regs(lane, g);

  // per-layer step operands; layer 2 runs one step AHEAD of layer 1 (its step t - 1 is
  // independent of layer 1's step t), so both layers' MFMA / VALU / LDS work sits in one
  // straight-line loop body the scheduler can interleave
  struct Op1 {
    f32x4 x[2];            // x_t, features 16kt + 4g + j
    bf16x4 hp[2], cp[2];   // h1_{t-1}, c1_{t-1}
  };
  struct Op2 {
    bf16x4 hp[1], cp[1], dh[1];   // h2_{t-1}, c2_{t-1}, dh2_t
  };
  const int64_t nblk = (a.B + 16 * WAVES - 1) / (16 * WAVES);
  bool any_active = false;
  for (int64_t blk = blockIdx.x; blk < nblk; blk += gridDim.x) {   // block-uniform trip count
    const int64_t wave_id = blk * WAVES + w;
    const int64_t s0 = wave_id * 16;
    const bool active = s0 < a.B;
    const int64_t seq = s0 + c;
    const bool valid = seq < a.B;
    const int64_t sq = valid ? seq : a.B - 1;
    any_active |= active;
    const __bf16* cw1 = a.c1 + wave_id * T * (int64_t)(2 * 256) + lane * 4;
    const __bf16* cw2 = a.c2 + wave_id * T * (int64_t)(1 * 256) + lane * 4;
    L1.begin(cw1, T, active);
    L2.begin(cw2, T, active);
    if (!active) continue;
    const __bf16* h1row = a.h1 + sq * T * 32;
    const __bf16* h2row = a.h2 + sq * T * 16;
    const float* xrow = a.x + sq * a.x_seq;
    const bf16x4 z4 = {0, 0, 0, 0};
    auto load1 = [&](int t, Op1& o) {   // t >= 0
#pragma unroll
      for (int kt = 0; kt < 2; ++kt) o.x[kt] = load_row4<XV1>(xrow + (int64_t)t * a.IN1, 16 * kt + 4 * g, a.IN1);
#pragma unroll
      for (int bb = 0; bb < 2; ++bb) {   // t = 0: zero initial state (Keras' stateless layers)
        o.cp[bb] = t > 0 ? ld_bf16x4(cw1 + (int64_t)(t - 1) * (2 * 256) + bb * 256) : z4;
        o.hp[bb] = t > 0 ? ld_bf16x4(h1row + (int64_t)(t - 1) * 32 + 16 * bb + 4 * g) : z4;
      }
    };
    auto load2 = [&](int t, Op2& o) {   // t >= 0
      const __bf16* dp = a.dh2_last_only ? a.dh2 + sq * 16 : a.dh2 + (sq * T + t) * 16;
      o.dh[0] = ld_bf16x4(dp + 4 * g);
      o.cp[0] = t > 0 ? ld_bf16x4(cw2 + (int64_t)(t - 1) * 256) : z4;
      o.hp[0] = t > 0 ? ld_bf16x4(h2row + (int64_t)(t - 1) * 16 + 4 * g) : z4;
    };
    auto l2_step = [&](int t, const bf16x4 (&x2)[2], const Op2& o, f32x4 (&dx2)[2]) {
      const bool take2 = valid && (!a.dh2_last_only || t == T - 1);
      const f32x4 dh2i[1] = {unpack4(o.dh[0])};
      L2.step(x2, o.hp, o.cp, dh2i, take2, lane, c, g, dx2);
    };
    // prologue: layer 2's step T - 1 (its x is h1_{T-1})
    f32x4 dx2[2];
    {
      bf16x4 x2[2];
#pragma unroll
      for (int bb = 0; bb < 2; ++bb) x2[bb] = ld_bf16x4(h1row + (int64_t)(T - 1) * 32 + 16 * bb + 4 * g);
      Op2 o2;
      load2(T - 1, o2);
      l2_step(T - 1, x2, o2, dx2);
    }
    Op1 n1;
    Op2 n2;
    load1(T - 1, n1);
    if (T >= 2) load2(T - 2, n2);
    for (int t = T - 1; t >= 1; --t) {   // layer 1's step t with layer 2's step t - 1
      const Op1 c1o = n1;
      const Op2 c2o = n2;
      load1(t - 1, n1);
      if (t >= 2) load2(t - 2, n2);
      // layer 1's incoming dh_t: layer 2's dX_t, rounded to bf16 as the two-launch path stores it
      f32x4 dh1i[2];
#pragma unroll
      for (int bb = 0; bb < 2; ++bb) dh1i[bb] = unpack4(pack4(dx2[bb]));
      f32x4 ndx2[2];
      l2_step(t - 1, c1o.hp, c2o, ndx2);   // x of layer 2 at t - 1 = h1_{t-1} = layer 1's h_{t-1} now
      f32x4 unused[2];
      L1.step(c1o.x, c1o.hp, c1o.cp, dh1i, valid, lane, c, g, unused);
#pragma unroll
      for (int bb = 0; bb < 2; ++bb) dx2[bb] = ndx2[bb];
    }
    {   // layer 1's step 0
      f32x4 dh1i[2], unused[2];
#pragma unroll
      for (int bb = 0; bb < 2; ++bb) dh1i[bb] = unpack4(pack4(dx2[bb]));
      L1.step(n1.x, n1.hp, n1.cp, dh1i, valid, lane, c, g, unused);
    }
    L1.wgrad(c, g);   // step 0's weight gradients
    L2.wgrad(c, g);
  }
  L1.write_slab(any_active, w, c, g, a.partials1 + (int64_t)blockIdx.x * L1T::S);
  L2.write_slab(any_active, w, c, g, a.partials2 + (int64_t)blockIdx.x * L2T::S);
}

}  // namespace

namespace sml {

bool lstm_fused_bwd2_supported(int IN1, int U1, int U2, int act1, int act2) {
  return U1 == 32 && U2 == 16 && IN1 >= 1 && IN1 + 2 <= 32 && act1 == act2 && (act1 == ACT_RELU || act1 == ACT_TANH) &&
         bias_mode(IN1, 2) == BM_BX && bias_mode(32, 2) == BM_PLAIN;
}

int lstm_fused_bwd2_grid(int64_t B) { return lstm_fused_slabs(B, 32, false); }

hipError_t lstm_fused_bwd2_launch(const float* x, int64_t x_seq, int IN1, const void* h1, const void* c1, const void* h2,
                                  const void* c2, const void* dh2, int dh2_last_only, const float* W1, const float* U1,
                                  const float* b1, const float* W2, const float* U2, const float* b2, float* partials1,
                                  float* partials2, int64_t B, int T, int act, hipStream_t stream) {
  Bwd2Args a{x, (const __bf16*)h1, (const __bf16*)c1, (const __bf16*)h2, (const __bf16*)c2, (const __bf16*)dh2,
             W1, U1, b1, W2, U2, b2, partials1, partials2, B, x_seq > 0 ? x_seq : (int64_t)T * IN1, T, IN1,
             dh2_last_only};
  const int grid = lstm_fused_bwd2_grid(B);
  const int xv = row_vec(x, IN1, 4);
  static const int rf = [] {   // SML_LSTM_BWD2_RF: layer 1's register fragments (lstm_fused.hip RF bits)
    const char* e = std::getenv("SML_LSTM_BWD2_RF");
    return e ? std::atoi(e) : 0;   // RF 1 (U fragments in registers): 85.4 vs 88.8 M windows/s
  }();
#define SML_B2(XVC, A, RFC) \
  hipLaunchKernelGGL((lstm_fused_bwd2_kernel<XVC, A, RFC>), dim3(grid), dim3(WAVES * 64), 0, stream, a)
#define SML_B2A(XVC, RFC)                      \
  if (act == ACT_RELU) SML_B2(XVC, ACT_RELU, RFC); \
  else SML_B2(XVC, ACT_TANH, RFC)
  // (RF 3, and RF 1 with scalar-row x, spill: not built)
#define SML_B2R(XVC)           \
  if (rf == 1) { SML_B2A(XVC, 1); } \
  else { SML_B2A(XVC, 0); }
  if (xv == 4) { SML_B2R(4) }
  else if (xv == 2) { SML_B2R(2) }
  else { SML_B2A(1, 0); }
#undef SML_B2R
#undef SML_B2A
#undef SML_B2
  return hipGetLastError();
}

}  // namespace sml
