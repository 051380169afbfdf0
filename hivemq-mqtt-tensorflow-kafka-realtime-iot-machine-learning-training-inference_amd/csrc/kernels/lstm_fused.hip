// sml-build: agpr-accumulators
//
// Fully fused LSTM layer kernels for gfx950: ONE launch for the forward pass
// and ONE for the backward pass of a Keras LSTM layer (reference
// LSTM-TensorFlow-IO-Kafka/cardata-v2.py:177-183: activation relu|tanh,
// recurrent_activation sigmoid, gate order i,f,c,o).
//
// Why: at the BASELINE config-3 shapes (B*T = 409 600 rows, 4u = 128 gates) the
// unfused layer moved ~2 GB per training step through HBM (x.W written as Zx and
// re-read, fp32 gates, dz written and re-read by three weight-gradient / dX
// GEMMs).  Fused, a layer reads x, h, c and bf16 gates once per pass:
//
//   forward, per step t (one wave = 16 sequences, h / c in VGPRs):
//     z^T[4u,16] = b + W^T . x_t^T + U^T . h_{t-1}^T     (all on MFMA)
//     gates -> bf16 store (for BPTT), c_t, h_t -> fp32 store
//   backward, per step t = T-1 .. 0:
//     dz_t from (dh_t + U.dz_{t+1}) and the stored gates / cell state
//     dh_{t-1}^T = U . dz_t^T                (critical path, MFMA)
//     dX_t^T     = W . dz_t^T                (MFMA, optional)
//     dW^T += dz_t^T . x_t,  dU^T += dz_t^T . h_{t-1},  db += colsum(dz_t) (fp32)
//       -> register accumulators (AGPRs) over the wave's 16 sequences x T
//          steps; the contraction over sequences needs dz_t^T as an A operand,
//          obtained with one LDS transpose per gate tile (ds_read_b64_tr_b16).
//     Each wave writes one fp32 slab of [dW^T | dU^T | db]; slab_sum_kernel
//     (dense.hip) reduces the slabs deterministically.
//
// Saved-state layout ("fragment-native"): gates and cell state are only ever read
// back by the backward kernel, by the same lane of the same wave that wrote them,
// so they are stored in MFMA C-fragment order, not [B, T, 4U]:
//   gates[wave][t][tile 0..MT)[lane 0..64)[4] bf16,  cseq[wave][t][tile 0..UB)[lane][4]
// Every store / load of a 16-sequence tile is then ONE contiguous 512-byte access per
// wave instead of 16 scattered 32-byte pieces (rows T*4U*2 bytes apart), and the
// buffers are padded to whole waves (16 sequences) so no lane needs a bounds check.
//
// MFMA orientation (v_mfma_f32_16x16x16_bf16, lane c = l & 15, g = l >> 4):
//   C tile mt of z: lane (c, g) holds gate 16mt + 4g + i of sequence s0 + c, so
//   the four gates of unit u sit in tiles q*UB + u/16 of the same lane/register.
// This file is compiled without -amdgpu-mfma-vgpr-form so the weight-gradient
// accumulators can live in AGPRs (launch_bounds(256, 1): 512 registers/lane).
#include "sml_common.h"
#include "sml_ops.h"

using namespace sml;

namespace {

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

struct FusedFwdArgs {
  const float* x;      // [B, T, IN]
  const float* W;      // [IN, 4U]
  const float* Uw;     // [U, 4U]
  const float* b;      // [4U]
  const float* h0;     // [B, U] or null
  const float* c0;     // [B, U] or null
  float* hseq;         // [B, T, U]
  __bf16* cseq;        // [B/16, T, U/16, 64, 4]   cell state, bf16, fragment-native (backward only)
  __bf16* gates;       // [B/16, T, 4U/16, 64, 4]  post-activation i, f, c~, o, fragment-native
  int64_t B;
  int T, IN, act;
  int xvec;            // x row access width in floats (4 / 2 / 1), from IN and x's alignment
};

template <int U, int KT>
__global__ __launch_bounds__(WAVES * 64, 1) void lstm_fused_fwd_kernel(FusedFwdArgs a) {
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
        t4[j] = k < IN ? a.W[(int64_t)k * G4 + 16 * mt + c] : 0.f;
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
    for (int i = 0; i < 4; ++i) bias[mt][i] = a.b[16 * mt + 4 * g + i];
  }
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
  const float* xrow = a.x + sq * (int64_t)T * IN;
  const int xvec = a.xvec;   // wave-uniform
  auto load_x = [&](int t, f32x4* v) {
    const float* p = xrow + (int64_t)t * IN;
#pragma unroll
    for (int kt = 0; kt < KT; ++kt) {
      const int k0 = 16 * kt + 4 * g;
      if (xvec == 4) {                       // one dwordx4 per tile
        v[kt] = k0 < IN ? *reinterpret_cast<const f32x4*>(p + k0) : f32x4{0.f, 0.f, 0.f, 0.f};
      } else if (xvec == 2) {                // two dwordx2 (rows 8-byte aligned)
        const f32x2_t lo = k0 < IN ? *reinterpret_cast<const f32x2_t*>(p + k0) : f32x2_t{0.f, 0.f};
        const f32x2_t hi = k0 + 2 < IN ? *reinterpret_cast<const f32x2_t*>(p + k0 + 2) : f32x2_t{0.f, 0.f};
        v[kt] = f32x4{lo[0], lo[1], hi[0], hi[1]};
      } else {
#pragma unroll
        for (int j = 0; j < 4; ++j) v[kt][j] = k0 + j < IN ? p[k0 + j] : 0.f;
      }
    }
  };
  const int64_t wv = (int64_t)blockIdx.x * WAVES + (threadIdx.x >> 6);
  __bf16* gw = a.gates + wv * T * (int64_t)(MT * 256) + lane * 4;
  __bf16* cw = a.cseq + wv * T * (int64_t)(UB * 256) + lane * 4;
  f32x4 xn[KT];
  load_x(0, xn);
  for (int t = 0; t < T; ++t) {
    bf16x4 xb[KT];
#pragma unroll
    for (int kt = 0; kt < KT; ++kt) xb[kt] = pack4(xn[kt]);
    if (t + 1 < T) load_x(t + 1, xn);   // next step's input, in flight during this step
    f32x4 z[MT];
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) {
      z[mt] = bias[mt];
#pragma unroll
      for (int kt = 0; kt < KT; ++kt) z[mt] = mfma16(wt[mt][kt], xb[kt], z[mt]);
#pragma unroll
      for (int s = 0; s < UB; ++s) z[mt] = mfma16(ut[mt][s], hb[s], z[mt]);
    }
    const int64_t bu = (sq * T + t) * (int64_t)U;
    __bf16* gt = gw + (int64_t)t * (MT * 256);
    __bf16* ct = cw + (int64_t)t * (UB * 256);
#pragma unroll
    for (int b = 0; b < UB; ++b) {
      f32x4 gi, gf, gc, go;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        gi[i] = sigmoid_fast(z[b][i]);
        gf[i] = sigmoid_fast(z[UB + b][i]);
        gc[i] = act_f(a.act, z[2 * UB + b][i]);
        go[i] = sigmoid_fast(z[3 * UB + b][i]);
        cs[b][i] = fmaf(gf[i], cs[b][i], gi[i] * gc[i]);
        h[b][i] = go[i] * act_f(a.act, cs[b][i]);
      }
      // padded lanes (seq >= B) write their own padded slots: no bounds check
      *reinterpret_cast<bf16x4*>(gt + b * 256) = pack4(gi);
      *reinterpret_cast<bf16x4*>(gt + (UB + b) * 256) = pack4(gf);
      *reinterpret_cast<bf16x4*>(gt + (2 * UB + b) * 256) = pack4(gc);
      *reinterpret_cast<bf16x4*>(gt + (3 * UB + b) * 256) = pack4(go);
      *reinterpret_cast<bf16x4*>(ct + b * 256) = pack4(cs[b]);
      if (valid) *reinterpret_cast<f32x4*>(a.hseq + bu + 16 * b + 4 * g) = h[b];
      hb[b] = pack4(h[b]);
    }
  }
}

struct FusedBwdArgs {
  const float* dh;     // [B, T, U]  gradient w.r.t. the h sequence ([B, U] of h_T when dh_last_only)
  const __bf16* gates; // fragment-native, as written by the forward kernel
  const __bf16* cseq;  // fragment-native
  const float* hseq;   // [B, T, U]
  const float* x;      // [B, T, IN]
  const float* h0;     // [B, U] or null
  const float* c0;     // [B, U] or null
  const float* W;      // [IN, 4U]
  const float* Uw;     // [U, 4U]
  float* dx;           // [B, T, IN] or null
  float* dh0;          // [B, U] or null
  float* dc0;          // [B, U] or null
  float* partials;     // [nblocks, S]: dW^T [4U][16KT] | dU^T [4U][U] | db [4U] (one slab per workgroup)
  int64_t B;
  int T, IN, act;
  int dh_last_only;    // return_sequences=False: only h_T received a gradient (no [B, T, U] zeros read)
  int xvec;            // dx row access width in floats (4 / 2 / 1)
};

template <int U, int KT>
__global__ __launch_bounds__(WAVES * 64, 1) void lstm_fused_bwd_kernel(FusedBwdArgs a) {
  constexpr int G4 = 4 * U, MT = G4 / 16, UB = U / 16;
  constexpr int LDW = 16 * KT;
  constexpr int S = G4 * (LDW + U + 1);
  __shared__ __attribute__((aligned(16))) char scratch[WAVES][MT * 512];
  __shared__ __attribute__((aligned(16))) float slab[S];   // the workgroup's combined weight-gradient slab
  const int lane = threadIdx.x & 63, c = lane & 15, g = lane >> 4;
  const int w = threadIdx.x >> 6;
  const int64_t wave_id = (int64_t)blockIdx.x * WAVES + w;
  const int64_t s0 = wave_id * 16;
  const bool active = s0 < a.B;  // waves past B contribute zeros (they still join the slab barriers)
  const int64_t seq = s0 + c;
  const bool valid = seq < a.B;
  const int64_t sq = valid ? seq : a.B - 1;
  const int IN = a.IN, T = a.T;
  char* scr = scratch[w];
  for (int i = threadIdx.x; i < S; i += WAVES * 64) slab[i] = 0.f;

  // A fragments: U[m = unit][k = gate] (for dh), W[m = feature][k = gate] (for dX)
  bf16x4 uf[UB][MT];
#pragma unroll
  for (int b = 0; b < UB; ++b)
#pragma unroll
    for (int kt = 0; kt < MT; ++kt) {
      f32x4 t4;
#pragma unroll
      for (int j = 0; j < 4; ++j) t4[j] = a.Uw[(16 * b + c) * G4 + 16 * kt + 4 * g + j];
      uf[b][kt] = pack4(t4);
    }
  const bool want_dx = a.dx != nullptr;
  bf16x4 wf[KT][MT];
#pragma unroll
  for (int kt = 0; kt < KT; ++kt)
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) {
      f32x4 t4;
      const int f = 16 * kt + c;
#pragma unroll
      for (int j = 0; j < 4; ++j) t4[j] = (want_dx && f < IN) ? a.W[(int64_t)f * G4 + 16 * mt + 4 * g + j] : 0.f;
      wf[kt][mt] = pack4(t4);
    }

  const f32x4 zero4 = {0.f, 0.f, 0.f, 0.f};
  f32x4 accW[MT][KT], accU[MT][UB];
  f32x4 accb[MT];   // db in exact fp32: per lane (sequence c) over time, folded across lanes at the end
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) {
#pragma unroll
    for (int kt = 0; kt < KT; ++kt) accW[mt][kt] = zero4;
#pragma unroll
    for (int kb = 0; kb < UB; ++kb) accU[mt][kb] = zero4;
    accb[mt] = zero4;
  }
  f32x4 dhr[UB], dcn[UB];
#pragma unroll
  for (int b = 0; b < UB; ++b) dhr[b] = dcn[b] = zero4;

  // per-step operands; "C layout" ones indexed by this lane's sequence, the
  // weight-gradient B operands by rows (sequences) s0 + 4g + j
  // c_t is carried from the previous (later) step's c_{t-1} load: every c is read once
  struct Step {
    bf16x4 gi[UB], gf[UB], gc[UB], go[UB];
    bf16x4 cprev[UB];
    f32x4 dho[UB];
    f32x4 hprev[UB];   // B[k = seq 4g + j][n = unit 16kb + c]
    f32x4 xt[KT];      // B[k = seq 4g + j][n = feature 16kt + c]
  };
  const __bf16* gw = a.gates + wave_id * T * (int64_t)(MT * 256) + lane * 4;
  const __bf16* cw = a.cseq + wave_id * T * (int64_t)(UB * 256) + lane * 4;
  const int xvec = a.xvec;   // wave-uniform
  auto load_step = [&](int t, Step& st) {
    const int64_t bu = (sq * T + t) * (int64_t)U;
    const __bf16* gt = gw + (int64_t)t * (MT * 256);
    const __bf16* cp = cw + (int64_t)(t - 1) * (UB * 256);
#pragma unroll
    for (int b = 0; b < UB; ++b) {
      const int off = 16 * b + 4 * g;
      st.gi[b] = ld_bf16x4(gt + b * 256);
      st.gf[b] = ld_bf16x4(gt + (UB + b) * 256);
      st.gc[b] = ld_bf16x4(gt + (2 * UB + b) * 256);
      st.go[b] = ld_bf16x4(gt + (3 * UB + b) * 256);
      if (t > 0) st.cprev[b] = ld_bf16x4(cp + b * 256);
      else if (a.c0) st.cprev[b] = pack4(*reinterpret_cast<const f32x4*>(a.c0 + sq * U + off));
      else st.cprev[b] = pack4(zero4);
      if (a.dh_last_only) st.dho[b] = (valid && t == T - 1) ? *reinterpret_cast<const f32x4*>(a.dh + sq * U + off) : zero4;
      else st.dho[b] = valid ? *reinterpret_cast<const f32x4*>(a.dh + bu + off) : zero4;
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int64_t r = s0 + 4 * g + j;
      const bool rok = r < a.B;
      const int64_t rr = rok ? r : 0;
#pragma unroll
      for (int kb = 0; kb < UB; ++kb) {
        const int u = 16 * kb + c;
        float hv = 0.f;
        if (rok) {
          if (t > 0) hv = a.hseq[(rr * T + t - 1) * (int64_t)U + u];
          else if (a.h0) hv = a.h0[rr * U + u];
        }
        st.hprev[kb][j] = hv;
      }
#pragma unroll
      for (int kt = 0; kt < KT; ++kt) {
        const int f = 16 * kt + c;
        st.xt[kt][j] = (rok && f < IN) ? a.x[(rr * T + t) * (int64_t)IN + f] : 0.f;
      }
    }
  };

  Step cur, nxt;
  f32x4 ctc[UB];   // c_t
#pragma unroll
  for (int b = 0; b < UB; ++b)
    ctc[b] = active ? unpack4(ld_bf16x4(cw + (int64_t)(T - 1) * (UB * 256) + b * 256)) : zero4;
  if (active) load_step(T - 1, nxt);
  for (int t = T - 1; t >= 0 && active; --t) {
    cur = nxt;
    if (t > 0) load_step(t - 1, nxt);          // in flight during this step
    f32x4 cp[UB];                               // c_{t-1}
#pragma unroll
    for (int b = 0; b < UB; ++b) cp[b] = unpack4(cur.cprev[b]);
    f32x4 dzt[MT];
#pragma unroll
    for (int b = 0; b < UB; ++b) {
      const f32x4 gi = unpack4(cur.gi[b]), gf = unpack4(cur.gf[b]), gc = unpack4(cur.gc[b]),
                  go = unpack4(cur.go[b]);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float dh = cur.dho[b][i] + dhr[b][i];
        const float ct = ctc[b][i];
        const float ac = act_f(a.act, ct);
        const float dc = dcn[b][i] + dh * go[i] * act_d(a.act, ct, ac);
        dzt[b][i] = dc * gc[i] * gi[i] * (1.f - gi[i]);
        dzt[UB + b][i] = dc * cp[b][i] * gf[i] * (1.f - gf[i]);
        const float gcd = a.act == ACT_RELU ? (gc[i] > 0.f ? 1.f : 0.f) : fmaf(-gc[i], gc[i], 1.f);
        dzt[2 * UB + b][i] = dc * gi[i] * gcd;
        dzt[3 * UB + b][i] = dh * ac * go[i] * (1.f - go[i]);
        dcn[b][i] = dc * gf[i];
      }
      ctc[b] = cp[b];   // c_{t-1} is the next (earlier) step's c_t
    }
    if (!valid) {
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) dzt[mt] = zero4;
    }
    bf16x4 dzb[MT];
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) {
      dzb[mt] = pack4(dzt[mt]);
      accb[mt] += dzt[mt];
    }
    // critical path: recurrent gradient for step t-1
#pragma unroll
    for (int b = 0; b < UB; ++b) {
      f32x4 acc = zero4;
#pragma unroll
      for (int kt = 0; kt < MT; ++kt) acc = mfma16(uf[b][kt], dzb[kt], acc);
      dhr[b] = acc;
    }
    // input gradient dX_t^T = W . dz_t^T
    if (want_dx) {
#pragma unroll
      for (int kt = 0; kt < KT; ++kt) {
        f32x4 acc = zero4;
#pragma unroll
        for (int mt = 0; mt < MT; ++mt) acc = mfma16(wf[kt][mt], dzb[mt], acc);
        if (valid) {
          float* p = a.dx + (sq * T + t) * (int64_t)IN;
          const int f0 = 16 * kt + 4 * g;
          if (xvec == 4) {
            if (f0 < IN) *reinterpret_cast<f32x4*>(p + f0) = acc;
          } else if (xvec == 2) {
            if (f0 < IN) *reinterpret_cast<f32x2_t*>(p + f0) = f32x2_t{acc[0], acc[1]};
            if (f0 + 2 < IN) *reinterpret_cast<f32x2_t*>(p + f0 + 2) = f32x2_t{acc[2], acc[3]};
          } else {
#pragma unroll
            for (int i = 0; i < 4; ++i)
              if (f0 + i < IN) p[f0 + i] = acc[i];
          }
        }
      }
    }
    // weight gradients: dz_t^T as A operand (one LDS transpose per gate tile)
    bf16x4 hB[UB], xB[KT];
#pragma unroll
    for (int kb = 0; kb < UB; ++kb) hB[kb] = pack4(cur.hprev[kb]);
#pragma unroll
    for (int kt = 0; kt < KT; ++kt) xB[kt] = pack4(cur.xt[kt]);
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) {
      const bf16x4 adz = lds_transpose(dzb[mt], scr + mt * 512, c, g);
#pragma unroll
      for (int kt = 0; kt < KT; ++kt) accW[mt][kt] = mfma16(adz, xB[kt], accW[mt][kt]);
#pragma unroll
      for (int kb = 0; kb < UB; ++kb) accU[mt][kb] = mfma16(adz, hB[kb], accU[mt][kb]);

    }
  }
  if (valid && active) {
#pragma unroll
    for (int b = 0; b < UB; ++b) {
      const int off = 16 * b + 4 * g;
      if (a.dh0) *reinterpret_cast<f32x4*>(a.dh0 + sq * U + off) = dhr[b];
      if (a.dc0) *reinterpret_cast<f32x4*>(a.dc0 + sq * U + off) = dcn[b];
    }
  }
  // db: sum the 16 sequence lanes c of each row group (butterfly within 16 lanes)
#pragma unroll
  for (int mt = 0; mt < MT; ++mt)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      float v = accb[mt][i];
#pragma unroll
      for (int o = 1; o < 16; o <<= 1) v += __shfl_xor(v, o, 64);
      accb[mt][i] = v;
    }
  // the 4 waves add their accumulators into the workgroup slab in LDS in a fixed
  // order (deterministic), then the workgroup writes ONE slab (4x fewer bytes for
  // the slab reduction than a slab per wave).  C layout: row m = gate 16mt + 4g + i,
  // column = lane c.
  for (int turn = 0; turn < WAVES; ++turn) {
    __syncthreads();
    if (turn == w && active) {
#pragma unroll
      for (int mt = 0; mt < MT; ++mt)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int m = 16 * mt + 4 * g + i;
#pragma unroll
          for (int kt = 0; kt < KT; ++kt) slab[m * LDW + 16 * kt + c] += accW[mt][kt][i];
#pragma unroll
          for (int kb = 0; kb < UB; ++kb) slab[G4 * LDW + m * U + 16 * kb + c] += accU[mt][kb][i];
          if (c == 0) slab[G4 * LDW + G4 * U + m] += accb[mt][i];
        }
    }
  }
  __syncthreads();
  float* out = a.partials + (int64_t)blockIdx.x * S;
  for (int i = threadIdx.x; i < S; i += WAVES * 64) out[i] = slab[i];
}

template <int U, int KT>
hipError_t launch_fwd(const FusedFwdArgs& a, hipStream_t st) {
  const int grid = (int)((a.B + 16 * WAVES - 1) / (16 * WAVES));
  hipLaunchKernelGGL((lstm_fused_fwd_kernel<U, KT>), dim3(grid), dim3(WAVES * 64), 0, st, a);
  return hipGetLastError();
}

template <int U, int KT>
hipError_t launch_bwd(const FusedBwdArgs& a, hipStream_t st) {
  const int grid = (int)((a.B + 16 * WAVES - 1) / (16 * WAVES));
  hipLaunchKernelGGL((lstm_fused_bwd_kernel<U, KT>), dim3(grid), dim3(WAVES * 64), 0, st, a);
  return hipGetLastError();
}

template <typename F>
hipError_t dispatch(int U, int IN, F&& f) {
  const int KT = (IN + 15) / 16;
#define SML_UK(u, k) \
  if (U == u && KT <= k) return f(std::integral_constant<int, u>{}, std::integral_constant<int, k>{});
  SML_UK(16, 1) SML_UK(16, 2) SML_UK(16, 4)
  SML_UK(32, 1) SML_UK(32, 2)
#undef SML_UK
  return hipErrorInvalidValue;
}

int row_vec(const void* p, int IN) {
  const uintptr_t u = (uintptr_t)p;
  if ((IN & 3) == 0 && (u & 15) == 0) return 4;
  if ((IN & 1) == 0 && (u & 7) == 0) return 2;
  return 1;
}

}  // namespace

namespace sml {

bool lstm_fused_supported(int U, int IN) {
  const int KT = (IN + 15) / 16;
  // larger (U, IN) would spill the backward kernel's weight-gradient accumulators
  // (U = 64 layers use the unfused recurrence + K1/K2 path)
  return IN >= 1 && (U == 16 ? KT <= 4 : (U == 32 ? KT <= 2 : false));
}

int lstm_fused_slab(int U, int IN) {
  const int KT = (IN + 15) / 16;
  const int kt = KT <= 1 ? 1 : (KT <= 2 ? 2 : 4);   // the dispatch bucket
  return 4 * U * (16 * kt + U + 1);
}

int lstm_fused_waves(int64_t B) { return (int)(((B + 16 * WAVES - 1) / (16 * WAVES)) * WAVES); }
int lstm_fused_slabs(int64_t B) { return (int)((B + 16 * WAVES - 1) / (16 * WAVES)); }

hipError_t lstm_fused_fwd_launch(const float* x, const float* W, const float* Uw, const float* b, const float* h0,
                                 const float* c0, float* hseq, void* cseq_bf16, void* gates_bf16, int64_t B, int T,
                                 int IN, int U, int act, hipStream_t stream) {
  FusedFwdArgs a{x, W, Uw, b, h0, c0, hseq, (__bf16*)cseq_bf16, (__bf16*)gates_bf16, B, T, IN, act, row_vec(x, IN)};
  return dispatch(U, IN, [&](auto u, auto k) { return launch_fwd<decltype(u)::value, decltype(k)::value>(a, stream); });
}

hipError_t lstm_fused_bwd_launch(const float* dh, const void* gates_bf16, const void* cseq_bf16, const float* hseq,
                                 const float* x, const float* h0, const float* c0, const float* W, const float* Uw,
                                 float* dx, float* dh0, float* dc0, float* partials, int64_t B, int T, int IN, int U,
                                 int act, int dh_last_only, hipStream_t stream) {
  FusedBwdArgs a{dh,       (const __bf16*)gates_bf16, (const __bf16*)cseq_bf16, hseq, x, h0, c0, W, Uw, dx, dh0, dc0,
                 partials, B,  T,  IN, act, dh_last_only, dx ? row_vec(dx, IN) : 1};
  return dispatch(U, IN, [&](auto u, auto k) { return launch_bwd<decltype(u)::value, decltype(k)::value>(a, stream); });
}

}  // namespace sml
