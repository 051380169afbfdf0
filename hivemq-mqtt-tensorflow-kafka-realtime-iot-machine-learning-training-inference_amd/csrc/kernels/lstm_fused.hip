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
// GEMMs).  Fused, the forward writes h (the layer output) and the cell state, both
// bf16; the backward reads x, h, c and dh once and RECOMPUTES the gates:
//
//   forward, per step t (one wave = 16 sequences, h / c in VGPRs):
//     z^T[4u,16] = b + W^T . x_t^T + U^T . h_{t-1}^T     (all on MFMA)
//     c_t -> bf16 store (for BPTT), h_t -> bf16 store
//
// Inter-layer tensors are bf16 (h, and dh / dx between two LSTM layers): every
// consumer of h rounds it to bf16 for an MFMA anyway (the recurrence itself, the next
// layer's x.W, this layer's recompute and dU), so fp32 storage bought no accuracy
// and cost half of the layer's HBM bytes.  The model input x may stay fp32.
//   backward, per step t = T-1 .. 0:
//     z^T recomputed from x_t, h_{t-1} (which the weight gradients read anyway):
//       (KT + U/16) * 4U/16 MFMAs instead of 8U bytes per sequence-step written by
//       the forward and read back here -- the kernels are HBM-bound, MFMA is idle
//     dz_t from (dh_t + U.dz_{t+1}), the gates and the cell state
//     dh_{t-1}^T = U . dz_t^T                (critical path, MFMA)
//     dX_t^T     = W . dz_t^T                (MFMA, optional)
//     dW^T += dz_t^T . x_t,  dU^T += dz_t^T . h_{t-1},  db += colsum(dz_t) (fp32)
//       -> register accumulators (AGPRs) over the wave's 16 sequences x T
//          steps; the contraction over sequences needs dz_t^T as an A operand,
//          obtained with one LDS transpose per gate tile (ds_read_b64_tr_b16).
//     Each wave writes one fp32 slab of [dW^T | dU^T | db]; slab_sum_kernel
//     (dense.hip) reduces the slabs deterministically.
//
// Saved-state layout ("fragment-native"): the cell state is only ever read back by
// the backward kernel, by the same lane of the same wave that wrote it, so it is
// stored in MFMA C-fragment order, not [B, T, U]:
//   cseq[wave][t][tile 0..U/16)[lane 0..64)[4] bf16
// Every store / load of a 16-sequence tile is then ONE contiguous 512-byte access per
// wave instead of 16 scattered 32-byte pieces (rows T*U*2 bytes apart), and the
// buffer is padded to whole waves (16 sequences) so no lane needs a bounds check.
//
// MFMA orientation (v_mfma_f32_16x16x16_bf16, lane c = l & 15, g = l >> 4):
//   C tile mt of z: lane (c, g) holds gate 16mt + 4g + i of sequence s0 + c, so
//   the four gates of unit u sit in tiles q*UB + u/16 of the same lane/register.
// This file (the backward) is compiled without -amdgpu-mfma-vgpr-form so the
// weight-gradient accumulators can live in AGPRs (launch_bounds(256, 1): 512
// registers/lane); the forward is lstm_fused_fwd.hip (VGPR form), shared helpers
// are in include/lstm_fused_impl.h.
#include <cstdlib>

#include "lstm_fused_impl.h"

using namespace sml;
using namespace sml_lstm;

namespace {

struct FusedBwdArgs {
  const __bf16* dh;    // [B, T, U] bf16 gradient w.r.t. the h sequence ([B, U] of h_T when dh_last_only)
  const __bf16* cseq;  // fragment-native, as written by the forward kernel
  const __bf16* hseq;  // [B, T, U] bf16 (the forward's output)
  const void* x;       // [B, T, IN] fp32 or bf16
  const float* h0;     // [B, U] or null
  const float* c0;     // [B, U] or null
  const float* W;      // [IN, 4U]
  const float* Uw;     // [U, 4U]
  const float* bias;   // [4U]
  void* dx;            // [B16, T, 16*KT] in x's dtype (padded rows / columns, the caller narrows) or null
  float* dh0;          // [B, U] or null
  float* dc0;          // [B, U] or null
  float* partials;     // [nblocks, S]: dW^T [4U][16KT] | dU^T [4U][U] | db [4U] (one slab per workgroup)
  int64_t B;
  int T, IN, act;
  int dh_last_only;    // return_sequences=False: only h_T received a gradient (no [B, T, U] zeros read)
  int64_t x_seq;       // elements between consecutive sequences of x (T*IN contiguous, IN sliding windows)
  __bf16* dzs;         // U >= 64 (DZS): dz_t stored fragment-native [B/16, T, 4U/16, 64, 4] bf16 for
                       // lstm_dz_wgrad_kernel (the weight gradients do not fit one wave's registers)
  int frag;            // fragment mode requested (the launch picks the FR instance)
};

// BM: bias mode (lstm_fused_impl.h bias_mode).  BX: the x operand carries constant 1.0
// columns at IN and IN + 1, the recompute's W^T fragments the bias there (bf16 hi + lo), so
// the gate recompute needs no bias read; BX and DB: column IN of the dW^T accumulator is
// sum_t,seq dz = db -- no per-step db adds (with them, the layer-1 kernel spent 13 % more
// wave cycles, mostly in s_waitcnt: profiles/r04), at the price of bf16-rounded dz in db, as
// in dW and dU.
// DX: the input gradient is wanted (compile-time: the first layer of a stack needs none).
// RF: weight A fragments kept in registers for the whole launch instead of re-read from
// LDS every step (bits: 1 the recurrent U fragments of the dh chain, 2 the gate
// recompute's [W^T | U^T], 4 the dX fragments W) -- where the registers exist, see launch_bwd.
// PFD: operand prefetch distance of the one-step loop (steps in flight ahead of the one computing).
// FR: fragment mode -- the h sequence, a bf16 x (a lower layer's h), dh (unless dh_last_only) and dx
// are [B/16, T, U/16 | KT, 64 lanes, 4] bf16 (the layout of c): every per-step access of a wave is one
// contiguous 512-byte piece per tile instead of 16 row pieces (the stacked model's layers, fed by
// lstm_fused_fwd2's HF mode).
template <int U, int KT, int XV, typename XT, int ACT, bool DX = true, int RF = 0, int BM = BM_PLAIN, int PFD = 1,
          bool FR = false>
__global__ __launch_bounds__(WAVES * 64, 1) void lstm_fused_bwd_kernel(FusedBwdArgs a) {
  constexpr bool BX = BM == BM_BX, DB = BM != BM_PLAIN;   // bias in the MFMAs / db from the dW^T column
  using XR = typename RowRaw<XT>::type;
  constexpr int G4 = 4 * U, MT = G4 / 16, UB = U / 16;
  constexpr int LDW = 16 * KT;
  constexpr int S = G4 * (LDW + U + 1);
  // DZS (U >= 64): dW^T | dU^T alone would take 4U x (16 KT + U) / 64 >= 320 accumulator registers per
  // lane, more than a wave has -- this kernel runs the recurrence, dh, dX and (PLAIN) db and stores dz_t
  // (bf16, the precision dW / dU consume anyway); lstm_dz_wgrad_kernel contracts it, split over gate groups
  constexpr bool DZS = U >= 64;
  constexpr int NTR = MT + KT + UB;                 // LDS transposes per step: dz tiles, x tiles, h tiles
  __shared__ __attribute__((aligned(16))) char scratch[WAVES][DZS ? 16 : NTR * 512];
  __shared__ __attribute__((aligned(16))) float slab[DZS ? (BM == BM_PLAIN ? G4 : 1) : S];   // the workgroup's combined weight-gradient slab
  // Weight A fragments, shared by the 4 waves, [tile][lane] bf16x4 (conflict-free
  // ds_read_b64).  RF selects which stay in registers for the launch; the rest are read
  // in the loop through an opaque lane offset so the compiler cannot hoist them (all
  // three sets together, with dX, would not fit next to the accumulators):
  //   wfwd: W^T / U^T (forward orientation, gate recompute), ufl: U (dh), wfl: W (dX)
  __shared__ __attribute__((aligned(16))) bf16x4 wfwd[MT * (KT + UB) * 64];
  __shared__ __attribute__((aligned(16))) bf16x4 ufl[UB * MT * 64];
  __shared__ __attribute__((aligned(16))) bf16x4 wfl[KT * MT * 64];
  __shared__ __attribute__((aligned(16))) float sbias[G4];
  const int lane = threadIdx.x & 63, c = lane & 15, g = lane >> 4;
  // wave-uniform (SGPR) wave index: the per-step operand addresses below are an SGPR base plus a
  // per-lane 32-bit offset fixed for the tile (global_load saddr form) instead of 64-bit VGPR
  // pointers advanced per step (~12 v_lshl_add_u64 per step and their registers, profiles/r06)
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  // Persistent grid (lstm_fused_slabs): workgroup blockIdx.x takes 4-wave groups of 16-sequence
  // tiles blockIdx.x, + gridDim.x, ... -- the weight fragments are staged once per workgroup
  // and the weight gradients of all its tiles land in ONE slab (4x fewer slab bytes written
  // and re-read by slab_sum at one workgroup per CU).  The per-tile values below are set by
  // the tile loop; the lambdas read them by reference.
  const int64_t nblk = (a.B + 16 * WAVES - 1) / (16 * WAVES);
  int64_t wave_id = (int64_t)blockIdx.x * WAVES + w;
  int64_t s0 = wave_id * 16;
  bool active = s0 < a.B;  // waves past B contribute zeros (they still join the block barriers)
  int64_t seq = s0 + c;
  bool valid = seq < a.B;
  int64_t sq = valid ? seq : a.B - 1;
  bool any_active = false;
  const int IN = a.IN, T = a.T;
  char* scr = scratch[w];
  for (int i = threadIdx.x; i < (DZS ? (BM == BM_PLAIN ? G4 : 1) : S); i += WAVES * 64) slab[i] = 0.f;
  for (int i = threadIdx.x; i < G4; i += WAVES * 64) sbias[i] = a.bias[i];
  // tile (mt, k) of [W^T | U^T]: k < KT -> W^T[m = gate 16mt + c][feature 16k + 4g + j],
  //                              k >= KT -> U^T[m = gate][unit 16(k-KT) + 4g + j]
  for (int tile = w; tile < MT * (KT + UB); tile += WAVES) {
    const int mt = tile / (KT + UB), k = tile % (KT + UB);
    f32x4 t4;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      if (k < KT) {
        const int f = 16 * k + 4 * g + j;
        t4[j] = BX ? wt_elem_bx(a.W, a.bias, G4, IN, f, 16 * mt + c) : (f < IN ? a.W[(int64_t)f * G4 + 16 * mt + c] : 0.f);
      } else {
        t4[j] = a.Uw[(16 * (k - KT) + 4 * g + j) * G4 + 16 * mt + c];
      }
    }
    wfwd[tile * 64 + lane] = pack4(t4);
  }

  // A fragments: U[m = unit 16b + c][k = gate 16kt + 4g + j] (for dh), W[m = feature][k = gate] (for dX)
  const bool want_dx = DX && a.dx != nullptr;
  for (int tile = w; tile < UB * MT; tile += WAVES) {
    const int b = tile / MT, kt = tile % MT;
    f32x4 t4;
#pragma unroll
    for (int j = 0; j < 4; ++j) t4[j] = a.Uw[(16 * b + c) * G4 + 16 * kt + 4 * g + j];
    ufl[tile * 64 + lane] = pack4(t4);
  }
  for (int tile = w; tile < KT * MT; tile += WAVES) {
    const int kt = tile / MT, mt = tile % MT;
    const int f = 16 * kt + c;
    f32x4 t4;
#pragma unroll
    for (int j = 0; j < 4; ++j) t4[j] = (want_dx && f < IN) ? a.W[(int64_t)f * G4 + 16 * mt + 4 * g + j] : 0.f;
    wfl[tile * 64 + lane] = pack4(t4);
  }
  __syncthreads();   // weight fragments / sbias visible

  const f32x4 zero4 = {0.f, 0.f, 0.f, 0.f};
  constexpr int NKT = KT + UB;
  constexpr bool RFU = RF & 1, RFW = RF & 2, RFX = DX && (RF & 4);
  bf16x4 rfw[RFW ? MT * NKT : 1], rfu[RFU ? UB * MT : 1], rfx[RFX ? KT * MT : 1];
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
  constexpr int MA = DZS ? 1 : MT;   // weight-gradient accumulator rows (none held under DZS)
  f32x4 accW[MA][KT], accU[MA][UB];
  f32x4 accb[MT];   // db in exact fp32: per lane (sequence c) over time, folded across lanes at the end
#pragma unroll
  for (int mt = 0; mt < MA; ++mt) {
#pragma unroll
    for (int kt = 0; kt < KT; ++kt) accW[mt][kt] = zero4;
#pragma unroll
    for (int kb = 0; kb < UB; ++kb) accU[mt][kb] = zero4;
  }
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) accb[mt] = zero4;
  f32x4 dhr[UB], dcn[UB];
#pragma unroll
  for (int b = 0; b < UB; ++b) dhr[b] = dcn[b] = zero4;
  // BX / DB: the bf16 1.0 bits this lane ORs into its x operand (features IN, IN + 1)
  bf16x4 onex[KT];
  u32x2_t xkeep[KT];   // the x operand's kept columns (row_operand_k)
#pragma unroll
  for (int kt = 0; kt < KT; ++kt) {
    onex[kt] = DB ? ones_at_bias(kt, g, IN) : bf16x4{0, 0, 0, 0};
    xkeep[kt] = row_keep(16 * kt + 4 * g, IN);
  }

  // Per-step operands, all in C orientation (lane c = this lane's sequence): the
  // forward's inputs x_t and h_{t-1} (gates are recomputed from them instead of being
  // stored: 8U bytes per sequence-step less written AND read), c_{t-1}, dh_t.
  // c_t is carried from the previous (later) step's c_{t-1} load: every c is read once.
  struct Step {
    bf16x4 cprev[UB];
    bf16x4 dho[UB];
    bf16x4 hp[UB];     // h_{t-1}[sequence c][unit 16b + 4g + i]
    XR xt[KT];         // x_t[sequence c][feature 16kt + 4g + j]
  };
  __bf16* dzw = DZS ? a.dzs + wave_id * T * (int64_t)(MT * 256) + lane * 4 : nullptr;
  constexpr bool XFR = FR && std::is_same_v<XT, __bf16>;   // x is a fragment-native h sequence
  // Per-lane byte offsets of the tile, fixed over its steps (the uniform parts are added per access):
  // cl = this lane's row of the tile, clamped into B (padding lanes read row B - 1).
  int cl = 0;
  int xo[KT][4];
  constexpr int XS = sizeof(XT);
  const unsigned lo8 = lane * 8;   // fragment-native: lane's 8 bytes of a 512-byte tile
  auto ld8 = [&](const void* base, int64_t uoff, unsigned loff) {   // uniform base + offset, lane offset
    return *reinterpret_cast<const bf16x4*>(static_cast<const char*>(base) + uoff + loff);
  };
  // Loads are unconditional from in-bounds addresses (padding lanes read row B-1),
  // with zeros selected afterwards: no exec-masked branches and no waits in the loop.
  auto load_common = [&](int t, Step& st) {   // raw values; masks are applied in step()
    if (FR && !a.dh_last_only) {
#pragma unroll
      for (int b = 0; b < UB; ++b) st.dho[b] = ld8(a.dh, ((wave_id * T + t) * UB + b) * 512, lo8);
    } else if (a.dh_last_only) {
#pragma unroll
      for (int b = 0; b < UB; ++b) st.dho[b] = ld8(a.dh, s0 * (U * 2), (cl * U + 16 * b + 4 * g) * 2);
    } else {
#pragma unroll
      for (int b = 0; b < UB; ++b) st.dho[b] = ld8(a.dh, (s0 * T + t) * (int64_t)(U * 2), (cl * T * U + 16 * b + 4 * g) * 2);
    }
    if constexpr (XFR) {
#pragma unroll
      for (int kt = 0; kt < KT; ++kt) st.xt[kt] = ld8(a.x, ((wave_id * T + t) * KT + kt) * 512, lo8);
    } else {
      const char* xt0 = static_cast<const char*>(a.x) + (s0 * a.x_seq + (int64_t)t * IN) * XS;   // uniform
#pragma unroll
      for (int kt = 0; kt < KT; ++kt) {
        if constexpr (std::is_same_v<XT, float>) {
          if constexpr (XV == 4) {
            st.xt[kt] = *reinterpret_cast<const f32x4*>(xt0 + xo[kt][0]);
          } else if constexpr (XV == 2) {
            const f32x2_t lo = *reinterpret_cast<const f32x2_t*>(xt0 + xo[kt][0]);
            const f32x2_t hi = *reinterpret_cast<const f32x2_t*>(xt0 + xo[kt][2]);
            st.xt[kt] = XR{lo[0], lo[1], hi[0], hi[1]};
          } else {
#pragma unroll
            for (int j = 0; j < 4; ++j) st.xt[kt][j] = *reinterpret_cast<const float*>(xt0 + xo[kt][j]);
          }
        } else {
          if constexpr (XV == 4) {
            st.xt[kt] = *reinterpret_cast<const bf16x4*>(xt0 + xo[kt][0]);
          } else if constexpr (XV == 2) {
            const s16x2_t lo = *reinterpret_cast<const s16x2_t*>(xt0 + xo[kt][0]);
            const s16x2_t hi = *reinterpret_cast<const s16x2_t*>(xt0 + xo[kt][2]);
            st.xt[kt] = XR{lo[0], lo[1], hi[0], hi[1]};
          } else {
#pragma unroll
            for (int j = 0; j < 4; ++j) st.xt[kt][j] = *reinterpret_cast<const short*>(xt0 + xo[kt][j]);
          }
        }
      }
    }
  };
  auto load_step = [&](int t, Step& st) {   // t >= 1
#pragma unroll
    for (int b = 0; b < UB; ++b) {
      st.cprev[b] = ld8(a.cseq, ((wave_id * T + t - 1) * UB + b) * 512, lo8);
      st.hp[b] = FR ? ld8(a.hseq, ((wave_id * T + t - 1) * UB + b) * 512, lo8)
                    : ld8(a.hseq, (s0 * T + t - 1) * (int64_t)(U * 2), (cl * T * U + 16 * b + 4 * g) * 2);
    }
    load_common(t, st);
  };
  auto load_step0 = [&](Step& st) {         // t = 0: initial state (once per sequence)
#pragma unroll
    for (int b = 0; b < UB; ++b) {
      const int off = 16 * b + 4 * g;
      st.cprev[b] = a.c0 ? pack4(*reinterpret_cast<const f32x4*>(a.c0 + sq * U + off)) : pack4(zero4);
      st.hp[b] = pack4(a.h0 ? *reinterpret_cast<const f32x4*>(a.h0 + sq * U + off) : zero4);
    }
    load_common(0, st);
  };
  auto load_any = [&](int t, Step& st) {
    if (t > 0) load_step(t, st);
    else load_step0(st);
  };

  f32x4 ctc[UB];   // c_t (loaded per tile)

  // Weight gradients, contracted over the wave's 16 sequences: dz_t^T as A operand and
  // x_t / h_{t-1} as B operands [k = sequence][n = feature | unit], each one LDS transpose
  // of the C-orientation tile (padding lanes carry dz = 0, so their rows add nothing).
  // Software-pipelined one step behind the recurrence: step t issues the (independent)
  // weight-gradient MFMAs of step t+1 between its gate-recompute MFMAs and its gate
  // arithmetic, so the MFMA and VALU pipes overlap inside one wave (the kernel runs at
  // one wave per SIMD: there is no other wave to hide either behind).
  bf16x4 pdz[MT], pxb[KT], phb[UB];
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) pdz[mt] = pack4(zero4);
#pragma unroll
  for (int kt = 0; kt < KT; ++kt) pxb[kt] = pack4(zero4);
#pragma unroll
  for (int s = 0; s < UB; ++s) phb[s] = pack4(zero4);
  auto wgrad = [&]() {
    if constexpr (DZS) return;
    else {
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
  };
  // Pair loop (layer 1: register fragments, db column, no dX): each step transposes its own
  // operands right after its dh chain (slot 0: the trip's first step, slot 1: the second)
  // and the second step contracts two steps at once -- K = the 2 x 16 sequence-steps of
  // one 16x16x32 per accumulator tile, so every accumulator is written once per trip (with
  // one 16x16x16 per step the allocator rotated them through spare AGPRs: 96
  // v_accvgpr_mov per step).
  constexpr bool PAIR = RF != 0 && DB && !DX && XV != 1 && !DZS;   // (scalar-row x: the pair loop spilled)
  bf16x4 tdz[2][PAIR ? MT : 1], txb[2][PAIR ? KT : 1], thb[2][PAIR ? UB : 1];
  if constexpr (PAIR) {
#pragma unroll
    for (int q = 0; q < 2; ++q) {
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) tdz[q][mt] = pack4(zero4);
#pragma unroll
      for (int kt = 0; kt < KT; ++kt) txb[q][kt] = pack4(zero4);
#pragma unroll
      for (int s = 0; s < UB; ++s) thb[q][s] = pack4(zero4);
    }
  }
  auto wgrad2 = [&]() {
#pragma unroll
    for (int mt = 0; mt < (PAIR ? MT : 0); ++mt) {
#pragma unroll
      for (int kt = 0; kt < KT; ++kt) accW[mt][kt] = mfma32(tdz[0][mt], tdz[1][mt], txb[0][kt], txb[1][kt], accW[mt][kt]);
#pragma unroll
      for (int kb = 0; kb < UB; ++kb) accU[mt][kb] = mfma32(tdz[0][mt], tdz[1][mt], thb[0][kb], thb[1][kb], accU[mt][kb]);
    }
  };

  // mode 0: one-step loop (weight gradients one step behind through pdz / pxb / phb);
  // 1 / 2: first / second step of a pair-loop trip (tdz / txb / thb slot 0 / 1)
  auto step = [&](int t, const Step& cur, auto mode) {
    constexpr int M = decltype(mode)::value;
    const int ol = opaque_lane(lane);   // re-materialised per step: fragment reads stay in the loop
    auto fw = [&](int i) { if constexpr (RFW) return rfw[i]; else return wfwd[i * 64 + ol]; };
    auto fu = [&](int i) { if constexpr (RFU) return rfu[i]; else return ufl[i * 64 + ol]; };
    auto fx = [&](int i) { if constexpr (RFX) return rfx[i]; else return wfl[i * 64 + ol]; };
    // gate recompute: z^T = b + W^T . x_t^T + U^T . h_{t-1}^T, the forward's exact
    // operands and accumulation order (bit-identical pre-activations)
    bf16x4 xb[KT], hb[UB];
#pragma unroll
    for (int kt = 0; kt < KT; ++kt)   // columns past IN zeroed; DB: IN, IN + 1 -> 1.0 (their weights: bias / 0)
      xb[kt] = row_operand_k(cur.xt[kt], xkeep[kt], onex[kt]);
    // Fragment mode (the stacked model): a padding lane's dh is exactly 0 -- layer 2's dX of a padding
    // sequence, whose dz is 0 -- so only the last-step-only case needs the select (8 VALU per step)
    const bool take_dh = (FR && !a.dh_last_only) ? true : valid && (!a.dh_last_only || t == T - 1);
#pragma unroll
    for (int s = 0; s < UB; ++s) hb[s] = cur.hp[s];
    f32x4 z[MT];
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) {
      z[mt] = BX ? zero4 : *reinterpret_cast<const f32x4*>(sbias + 16 * mt + (ol >> 4) * 4);
      constexpr int NK = KT + UB;   // K-tiles in pairs on 16x16x32, exactly as the forward
#pragma unroll
      for (int k = 0; k + 1 < NK; k += 2)
        z[mt] = mfma32(fw(mt * NK + k), fw(mt * NK + k + 1), k < KT ? xb[k] : hb[k - KT],
                       k + 1 < KT ? xb[k + 1] : hb[k + 1 - KT], z[mt]);
      if constexpr (NK & 1)   // as the forward: never a 16x16x16 on a 16x16x32 result
        z[mt] = mfma32(fw(mt * NK + NK - 1), bf16x4{0, 0, 0, 0}, hb[UB - 1], bf16x4{0, 0, 0, 0}, z[mt]);
    }
    if constexpr (M == 0) wgrad();              // step t+1's weight gradients (zeros on the first step)
    // (pair loop: the weight gradients are contracted at the end of the second step, below --
    // placed after the z recompute of the first step the allocator rotated the accumulators
    // through spare AGPRs: 112 v_accvgpr_mov per trip instead of 32)
            // the previous trip's two steps (zeros on the first trip)
    f32x4 cp[UB], dhi[UB];                      // c_{t-1}, incoming dh_t
#pragma unroll
    for (int b = 0; b < UB; ++b) {
      cp[b] = unpack4(cur.cprev[b]);
      dhi[b] = unpack4(cur.dho[b]);
    }
    f32x4 dzt[MT];
#pragma unroll
    for (int b = 0; b < UB; ++b) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        // fp32 gates, exactly the values the forward used for c_t / h_t
        const float gi = sigmoid_fast(z[b][i]), gf = sigmoid_fast(z[UB + b][i]);
        const float gc = act_f(ACT, z[2 * UB + b][i]), go = sigmoid_fast(z[3 * UB + b][i]);
        const float dh = (take_dh ? dhi[b][i] : 0.f) + dhr[b][i];
        const float ct = ctc[b][i];
        const float ac = act_f(ACT, ct);
        // the gate derivatives with shared factors and s(1-s) = fma(-s, s, s); relu's
        // derivative as selects: 16 VALU per element instead of ~25 (17 v_mul + 3 v_sub + ...)
        const float dhgo = dh * go;
        const float dc = ACT == ACT_RELU ? (ct > 0.f ? dcn[b][i] + dhgo : dcn[b][i])
                                         : fmaf(dhgo, fmaf(-ac, ac, 1.f), dcn[b][i]);
        const float di = dc * gi;
        const float df = dc * gf;
        dzt[b][i] = (dc * gc) * fmaf(-gi, gi, gi);                                   // dc g i(1-i)
        dzt[UB + b][i] = fmaf(-df, gf, df) * cp[b][i];                               // dc f(1-f) c_{t-1}
        dzt[2 * UB + b][i] = ACT == ACT_RELU ? (gc > 0.f ? di : 0.f) : di * fmaf(-gc, gc, 1.f);
        dzt[3 * UB + b][i] = (dh * ac) * fmaf(-go, go, go);                          // dh act(c) o(1-o)
        dcn[b][i] = df;
      }
      ctc[b] = cp[b];   // c_{t-1} is the next (earlier) step's c_t
    }
    // padding lanes (!valid) need no masking here: they never take dh (take_dh) and start
    // from dcn = 0, and every dz term carries a factor dh or dc, so their dz stays exactly 0
    // and they add nothing to the weight gradients
    bf16x4 dzb[MT];
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) {
      dzb[mt] = pack4(dzt[mt]);
      if constexpr (!DB) accb[mt] += dzt[mt];
    }
    if constexpr (DZS) {   // one contiguous 512-byte store per gate tile (padding lanes store dz = 0)
      __bf16* dzp = dzw + (int64_t)t * (MT * 256);
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) *reinterpret_cast<bf16x4*>(dzp + mt * 256) = dzb[mt];
    }
    // critical path: recurrent gradient for step t-1 -- the 4U gate tiles in pairs on
    // 16x16x32 (MT/2 dependent MFMAs, half the issues of two 16x16x16 half-chains)
#pragma unroll
    for (int b = 0; b < UB; ++b) {
      f32x4 acc = zero4;
#pragma unroll
      for (int kt = 0; kt < MT; kt += 2)
        acc = mfma32(fu(b * MT + kt), fu(b * MT + kt + 1), dzb[kt], dzb[kt + 1], acc);
      dhr[b] = acc;
    }
    // input gradient dX_t^T = W . dz_t^T
    if (DX && want_dx) {
#pragma unroll
      for (int kt = 0; kt < KT; ++kt) {
        f32x4 acc = zero4;
#pragma unroll
        for (int mt = 0; mt < MT; mt += 2)
          acc = mfma32(fx(kt * MT + mt), fx(kt * MT + mt + 1), dzb[mt], dzb[mt + 1], acc);
        // dx is [B16, T, 16*KT] (FR: fragment-native): every lane stores its whole piece, unmasked
        const int64_t o = FR ? (wave_id * T + t) * (int64_t)(KT * 256) + kt * 256 + lane * 4
                             : (seq * T + t) * (int64_t)(16 * KT) + 16 * kt + 4 * g;
        if constexpr (std::is_same_v<XT, float>) *reinterpret_cast<f32x4*>(static_cast<float*>(a.dx) + o) = acc;
        else *reinterpret_cast<bf16x4*>(static_cast<__bf16*>(a.dx) + o) = pack4(acc);
      }
    }
    if constexpr (M == 0) {   // operands of this step's weight gradients, consumed one step later
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) pdz[mt] = dzb[mt];
#pragma unroll
      for (int kt = 0; kt < KT; ++kt) pxb[kt] = xb[kt];
#pragma unroll
      for (int s = 0; s < UB; ++s) phb[s] = hb[s];
    } else {                  // transposed now, contracted by the next trip's first step
      constexpr int q = M - 1;
      if constexpr (M == 2) wgrad2();         // slot 0: this trip's first step, slot 1: the previous
                                              // trip's second step (zeros on the first trip)
#pragma unroll
      for (int kb = 0; kb < UB; ++kb) thb[q][kb] = lds_transpose(hb[kb], scr + (MT + KT + kb) * 512, c, g);
#pragma unroll
      for (int kt = 0; kt < KT; ++kt) txb[q][kt] = lds_transpose(xb[kt], scr + (MT + kt) * 512, c, g);
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) tdz[q][mt] = lds_transpose(dzb[mt], scr + mt * 512, c, g);
    }
  };

  // the next step's operands are in flight while the current one computes (a deeper,
  // unrolled three-buffer prefetch measured slower for U = 32: 626 vs 525 us).
  // Register-fragment builds with the db column (PAIR: layer 1 of the stack, one wave per SIMD anyway) take
  // two steps per trip with two fixed operand buffers, and only steps whose predecessor is
  // a stored one (t - 2 >= 1): no buffer copies (the one-step loop moved ~70 registers per
  // step) and no t = 0 branch splitting the loop body -- 418 -> 362 us for the U = 32 layer
  // (profiles/r04).  The two-wave builds keep the one-step loop: the pair loop's registers
  // pushed them past 256 (one wave per SIMD, 247 -> 326 us).
  for (int64_t blk = blockIdx.x; blk < nblk; blk += gridDim.x) {   // block-uniform trip count
  wave_id = blk * WAVES + w;
  s0 = wave_id * 16;
  active = s0 < a.B;
  seq = s0 + c;
  valid = seq < a.B;
  sq = valid ? seq : a.B - 1;
  cl = (int)(sq - s0);
#pragma unroll
  for (int kt = 0; kt < KT; ++kt)
#pragma unroll
    for (int j = 0; j < 4; ++j) {   // clamped in-row columns, as load_row4 (the operand masks the ones past IN)
      const int k0 = 16 * kt + 4 * g + (XV == 2 ? (j & 2) : (XV == 4 ? 0 : j));
      xo[kt][j] = (int)((cl * a.x_seq + (k0 < IN ? k0 : 0)) * XS);
    }
  if constexpr (DZS) dzw = a.dzs + wave_id * T * (int64_t)(MT * 256) + lane * 4;
  any_active |= active;
  // fresh recurrence and weight-gradient pipeline per tile (the accumulators carry on)
#pragma unroll
  for (int b = 0; b < UB; ++b) {
    dhr[b] = dcn[b] = zero4;
    ctc[b] = active ? unpack4(ld8(a.cseq, ((wave_id * T + T - 1) * UB + b) * 512, lo8)) : zero4;
  }
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) pdz[mt] = pack4(zero4);
#pragma unroll
  for (int kt = 0; kt < KT; ++kt) pxb[kt] = pack4(zero4);
#pragma unroll
  for (int s = 0; s < UB; ++s) phb[s] = pack4(zero4);
  if constexpr (PAIR) {
#pragma unroll
    for (int q = 0; q < 2; ++q) {
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) tdz[q][mt] = pack4(zero4);
#pragma unroll
      for (int kt = 0; kt < KT; ++kt) txb[q][kt] = pack4(zero4);
#pragma unroll
      for (int s = 0; s < UB; ++s) thb[q][s] = pack4(zero4);
    }
  }
  if (active) {
    Step nxt;
    load_any(T - 1, nxt);
    int t = T - 1;
    if constexpr (PAIR) {   // (with per-step db adds, BM_PLAIN, the pair loop spills at U = 32)
      Step sb;
      for (; t >= 3; t -= 2) {
        load_step(t - 1, sb);
        step(t, nxt, std::integral_constant<int, 1>{});
        load_step(t - 2, nxt);
        step(t - 1, sb, std::integral_constant<int, 2>{});
      }
      // the second step of a trip contracts (this trip's first step, the previous trip's
      // second step); left over: the last trip's second step (slot 1) alone
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) tdz[0][mt] = pack4(zero4);
      wgrad2();
    } else if constexpr (PFD == 2) {
      // two steps in flight: the U = 16 layer with dX at two waves per SIMD does ~1 us of work per
      // step, less than an HBM round trip under load -- with one step ahead its waves sat in
      // s_waitcnt 53 % of their cycles (profiles/r05/lstm)
      Step n2 = nxt;
      if (T >= 2) load_any(T - 2, n2);
      for (; t >= 3; --t) {
        const Step cur = nxt;
        nxt = n2;
        load_step(t - 2, n2);
        step(t, cur, std::integral_constant<int, 0>{});
      }
      for (; t >= 0; --t) {
        const Step cur = nxt;
        nxt = n2;
        if (t >= 2) load_any(t - 2, n2);
        step(t, cur, std::integral_constant<int, 0>{});
      }
    } else {
      for (; t >= 2; --t) {   // one step per trip, no t = 0 branch in the body
        const Step cur = nxt;
        load_step(t - 1, nxt);
        step(t, cur, std::integral_constant<int, 0>{});
      }
    }
    for (; t >= 0; --t) {
      const Step cur = nxt;
      if (t >= 1) load_any(t - 1, nxt);
      step(t, cur, std::integral_constant<int, 0>{});
    }
    wgrad();                                    // step 0's weight gradients
  }
  if (valid && active) {
#pragma unroll
    for (int b = 0; b < UB; ++b) {
      const int off = 16 * b + 4 * g;
      if (a.dh0) *reinterpret_cast<f32x4*>(a.dh0 + sq * U + off) = dhr[b];
      if (a.dc0) *reinterpret_cast<f32x4*>(a.dc0 + sq * U + off) = dcn[b];
    }
  }
  }   // tile loop
  // db: sum the 16 sequence lanes c of each row group (butterfly within 16 lanes)
  if constexpr (!DB)
#pragma unroll
  for (int mt = 0; mt < MT; ++mt)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      float v = accb[mt][i];
#pragma unroll
      for (int o = 1; o < 16; o <<= 1) v += __shfl_xor(v, o, 64);
      accb[mt][i] = v;
    }
  if constexpr (DZS) {   // only db (PLAIN), into the slab's db row; lstm_dz_wgrad_kernel writes the rest
    if constexpr (!DB) {
      for (int turn = 0; turn < WAVES; ++turn) {
        __syncthreads();
        if (turn == w && any_active && c == 0) {
#pragma unroll
          for (int mt = 0; mt < MT; ++mt)
#pragma unroll
            for (int i = 0; i < 4; ++i) slab[16 * mt + 4 * g + i] += accb[mt][i];
        }
      }
      __syncthreads();
      float* out = a.partials + (int64_t)blockIdx.x * S + G4 * LDW + G4 * U;
      for (int i = threadIdx.x; i < G4; i += WAVES * 64) out[i] = slab[i];
    }
    return;
  } else {
  // the 4 waves add their accumulators into the workgroup slab in LDS in a fixed
  // order (deterministic), then the workgroup writes ONE slab (4x fewer bytes for
  // the slab reduction than a slab per wave).  C layout: row m = gate 16mt + 4g + i,
  // column = lane c.
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
  if constexpr (DB) {   // db = column IN of dW^T (a constant-1 input); columns IN, IN + 1 are padding
    for (int m = threadIdx.x; m < G4; m += WAVES * 64) {
      slab[G4 * LDW + G4 * U + m] = slab[m * LDW + IN];
      slab[m * LDW + IN] = 0.f;
      if (IN + 1 < LDW) slab[m * LDW + IN + 1] = 0.f;
    }
    __syncthreads();
  }
  float* out = a.partials + (int64_t)blockIdx.x * S;
  for (int i = threadIdx.x; i < S; i += WAVES * 64) out[i] = slab[i];
  }
}

// Weight gradients of a DZS layer (U >= 64) from the stored dz: workgroup (x, y) takes the
// 16-sequence tiles of the persistent grid's workgroup x (the same tiles, so slab x gets the
// same rows) and the gate rows of group y (MG gate tiles), and contracts over its sequences and
// the T steps exactly as the fused kernel's wgrad(): dz_t^T as A operand, x_t (with the bias
// columns of BX / DB) and h_{t-1} as B operands, each through one LDS transpose.  MG = 8: 8 x
// (KT + U/16) accumulator tiles = 192 AGPRs at U = 64, KT = 2.  Writes the group's rows of
// dW^T, dU^T and (BX / DB) db of slab x; PLAIN db comes from the recurrence kernel (fp32 dz).
template <int U, int KT, int XV, typename XT, int BM, int MG>
__global__ __launch_bounds__(WAVES * 64, 1) void lstm_dz_wgrad_kernel(FusedBwdArgs a) {
  constexpr bool DB = BM != BM_PLAIN;
  using XR = typename RowRaw<XT>::type;
  constexpr int G4 = 4 * U, MT = G4 / 16, UB = U / 16, LDW = 16 * KT;
  constexpr int S = G4 * (LDW + U + 1);
  constexpr int RW = 16 * MG;                       // gate rows of this group
  __shared__ __attribute__((aligned(16))) char scratch[WAVES][(MG + KT + UB) * 512];
  __shared__ __attribute__((aligned(16))) float slab[RW * (LDW + U)];
  const int lane = threadIdx.x & 63, c = lane & 15, g = lane >> 4;
  const int w = threadIdx.x >> 6;
  const int mt0 = blockIdx.y * MG;
  const int IN = a.IN, T = a.T;
  char* scr = scratch[w];
  for (int i = threadIdx.x; i < RW * (LDW + U); i += WAVES * 64) slab[i] = 0.f;
  const f32x4 zero4 = {0.f, 0.f, 0.f, 0.f};
  f32x4 accW[MG][KT], accU[MG][UB];
#pragma unroll
  for (int m = 0; m < MG; ++m) {
#pragma unroll
    for (int kt = 0; kt < KT; ++kt) accW[m][kt] = zero4;
#pragma unroll
    for (int kb = 0; kb < UB; ++kb) accU[m][kb] = zero4;
  }
  bf16x4 onex[KT];
#pragma unroll
  for (int kt = 0; kt < KT; ++kt) onex[kt] = DB ? ones_at_bias(kt, g, IN) : bf16x4{0, 0, 0, 0};
  const int64_t nblk = (a.B + 16 * WAVES - 1) / (16 * WAVES);
  bool any_active = false;
  for (int64_t blk = blockIdx.x; blk < nblk; blk += gridDim.x) {
    const int64_t wave_id = blk * WAVES + w;
    const int64_t s0 = wave_id * 16;
    if (s0 >= a.B) continue;   // wave-uniform; no block barrier inside the tile loop
    any_active = true;
    const int64_t seq = s0 + c;
    const bool valid = seq < a.B;
    const int64_t sq = valid ? seq : a.B - 1;
    const __bf16* dzw = a.dzs + wave_id * T * (int64_t)(MT * 256) + lane * 4 + mt0 * 256;
    const XT* xrow = static_cast<const XT*>(a.x) + sq * a.x_seq;
    for (int t = 0; t < T; ++t) {
      bf16x4 dz[MG], hb[UB], xb[KT];
#pragma unroll
      for (int m = 0; m < MG; ++m) dz[m] = ld_bf16x4(dzw + (int64_t)t * (MT * 256) + m * 256);
#pragma unroll
      for (int kt = 0; kt < KT; ++kt) {
        const XR raw = load_row4<XV>(xrow + (int64_t)t * IN, 16 * kt + 4 * g, IN);
        xb[kt] = row_operand(raw, 16 * kt + 4 * g, IN);
        if constexpr (DB) xb[kt] |= onex[kt];
      }
#pragma unroll
      for (int b = 0; b < UB; ++b) {
        const int off = 16 * b + 4 * g;
        if (t > 0) hb[b] = ld_bf16x4(a.hseq + (sq * T + t - 1) * (int64_t)U + off);
        else hb[b] = pack4(a.h0 ? *reinterpret_cast<const f32x4*>(a.h0 + sq * U + off) : zero4);
      }
      // padding lanes carry dz = 0 (the recurrence kernel's invariant): their rows add nothing
      bf16x4 hB[UB], xB[KT];
#pragma unroll
      for (int kb = 0; kb < UB; ++kb) hB[kb] = lds_transpose(hb[kb], scr + (MG + KT + kb) * 512, c, g);
#pragma unroll
      for (int kt = 0; kt < KT; ++kt) xB[kt] = lds_transpose(xb[kt], scr + (MG + kt) * 512, c, g);
#pragma unroll
      for (int m = 0; m < MG; ++m) {
        const bf16x4 adz = lds_transpose(dz[m], scr + m * 512, c, g);
#pragma unroll
        for (int kt = 0; kt < KT; ++kt) accW[m][kt] = mfma16(adz, xB[kt], accW[m][kt]);
#pragma unroll
        for (int kb = 0; kb < UB; ++kb) accU[m][kb] = mfma16(adz, hB[kb], accU[m][kb]);
      }
    }
  }
  for (int turn = 0; turn < WAVES; ++turn) {   // fixed-order combine of the 4 waves (deterministic)
    __syncthreads();
    if (turn == w && any_active) {
#pragma unroll
      for (int m = 0; m < MG; ++m)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int r = 16 * m + 4 * g + i;
#pragma unroll
          for (int kt = 0; kt < KT; ++kt) slab[r * LDW + 16 * kt + c] += accW[m][kt][i];
#pragma unroll
          for (int kb = 0; kb < UB; ++kb) slab[RW * LDW + r * U + 16 * kb + c] += accU[m][kb][i];
        }
    }
  }
  __syncthreads();
  float* out = a.partials + (int64_t)blockIdx.x * S;
  const int r0 = 16 * mt0;
  for (int i = threadIdx.x; i < RW * LDW; i += WAVES * 64) {
    const int r = i / LDW, col = i % LDW;
    float v = slab[i];
    if (DB && col == IN) out[G4 * LDW + G4 * U + r0 + r] = v;   // db = column IN (a constant-1 input)
    if (DB && (col == IN || col == IN + 1)) v = 0.f;
    out[(r0 + r) * LDW + col] = v;
  }
  for (int i = threadIdx.x; i < RW * U; i += WAVES * 64) out[G4 * LDW + r0 * U + i] = slab[RW * LDW + i];
}

// the fragment-mode instances: the stacked model's layer 1 (U 32, fp32 x, no dX) and layer 2
// (U 16, bf16 x = layer 1's h, dX)
template <int U, int KT, typename XT, bool DX>
constexpr bool frag_instance() {
  return KT == 2 && ((U == 32 && !DX && std::is_same_v<XT, float>) || (U == 16 && DX && std::is_same_v<XT, __bf16>));
}

// activation as a template parameter: a runtime switch became ~40 scalar branches
// per step, which split the time loop into basic blocks the scheduler cannot overlap
template <int U, int KT, int XV, typename XT>
hipError_t launch_bwd(const FusedBwdArgs& a, hipStream_t st) {
  const int grid = lstm_fused_slabs(a.B, U, a.dx != nullptr);
  // Without dX (the first layer of a stack, U = 32 at one wave per SIMD) every weight
  // fragment fits in registers next to the AGPR accumulators: the per-step LDS fragment
  // reads were exposed latency there (SQ_WAIT_ANY 41 % of wave cycles) and the kernel
  // runs 17 % faster (bench_lstm 62.3 -> 68.1 M windows/s, profiles/r02).  With dX, at
  // two waves per SIMD, register fragments measured the same as LDS reads (67.8 vs 67.9).
  static const int pf_env = [] {   // SML_LSTM_BWD_PF=1|2|3: the U = 16 dX build's prefetch (A/B)
    const char* e = std::getenv("SML_LSTM_BWD_PF");
    return e ? std::atoi(e) : 0;
  }();
  auto go = [&](auto dx, auto rf, auto bmc) {
    constexpr bool DX = decltype(dx)::value;
    constexpr int RF = decltype(rf)::value;
    constexpr int BM = decltype(bmc)::value;
    auto launch = [&](auto kern) { hipLaunchKernelGGL(kern, dim3(grid), dim3(WAVES * 64), 0, st, a); };
    if constexpr (frag_instance<U, KT, XT, DX>()) {
      if (a.frag) {
        constexpr int PFD = (U == 16 && DX) ? 2 : 1;
        if (a.act == ACT_RELU) launch(lstm_fused_bwd_kernel<U, KT, XV, XT, ACT_RELU, DX, RF, BM, PFD, true>);
        else launch(lstm_fused_bwd_kernel<U, KT, XV, XT, ACT_TANH, DX, RF, BM, PFD, true>);
        return;
      }
    }
    if constexpr (U == 16 && DX) {
      if (pf_env == 1) {   // one step ahead, every fragment set in registers
        if (a.act == ACT_RELU) launch(lstm_fused_bwd_kernel<U, KT, XV, XT, ACT_RELU, DX, 7, BM, 1>);
        else launch(lstm_fused_bwd_kernel<U, KT, XV, XT, ACT_TANH, DX, 7, BM, 1>);
        return;
      }
      if (pf_env == 3) {   // two steps ahead, every fragment set in registers
        if (a.act == ACT_RELU) launch(lstm_fused_bwd_kernel<U, KT, XV, XT, ACT_RELU, DX, 7, BM, 2>);
        else launch(lstm_fused_bwd_kernel<U, KT, XV, XT, ACT_TANH, DX, 7, BM, 2>);
        return;
      }
    }
    constexpr int PFD = (U == 16 && DX) ? 2 : 1;
    if (a.act == ACT_RELU) launch(lstm_fused_bwd_kernel<U, KT, XV, XT, ACT_RELU, DX, RF, BM, PFD>);
    else launch(lstm_fused_bwd_kernel<U, KT, XV, XT, ACT_TANH, DX, RF, BM, PFD>);
  };
  auto with_bm = [&](auto dx, auto rf) {   // the same decision as the forward (lstm_fused_fwd.hip)
    switch (bias_mode(a.IN, KT)) {
      case BM_BX: go(dx, rf, std::integral_constant<int, BM_BX>{}); break;
      case BM_DB: go(dx, rf, std::integral_constant<int, BM_DB>{}); break;
      default: go(dx, rf, std::integral_constant<int, BM_PLAIN>{});
    }
  };
  if constexpr (U >= 64) {   // DZS: fragments from LDS, then the gate-group weight-gradient kernel
    if (a.dx) with_bm(std::true_type{}, std::integral_constant<int, 0>{});
    else with_bm(std::false_type{}, std::integral_constant<int, 0>{});
    constexpr int MG = 8;
    const dim3 wg(grid, (4 * U / 16) / MG);
    switch (bias_mode(a.IN, KT)) {
      case BM_BX: hipLaunchKernelGGL((lstm_dz_wgrad_kernel<U, KT, XV, XT, BM_BX, MG>), wg, dim3(WAVES * 64), 0, st, a); break;
      case BM_DB: hipLaunchKernelGGL((lstm_dz_wgrad_kernel<U, KT, XV, XT, BM_DB, MG>), wg, dim3(WAVES * 64), 0, st, a); break;
      default: hipLaunchKernelGGL((lstm_dz_wgrad_kernel<U, KT, XV, XT, BM_PLAIN, MG>), wg, dim3(WAVES * 64), 0, st, a);
    }
    return hipGetLastError();
  } else {
    // U = 16 with dX (layer 2 of the stack): every fragment set fits in registers at two waves
    // per SIMD (174 VGPRs + 64 AGPRs); U = 32 with dX reads them from LDS every step
    if (a.dx) {
      if constexpr (U == 16) with_bm(std::true_type{}, std::integral_constant<int, 3>{});   // two steps ahead
      else with_bm(std::true_type{}, std::integral_constant<int, 0>{});
    } else {
      with_bm(std::false_type{}, std::integral_constant<int, 3>{});
    }
    return hipGetLastError();
  }
}

}  // namespace

namespace sml {

bool lstm_fused_supported(int U, int IN) {
  const int KT = (IN + 15) / 16;
  // U = 64 (DZS): dz stored, weight gradients by lstm_dz_wgrad_kernel; larger U / IN use the
  // unfused recurrence + K1/K2 path
  return IN >= 1 && (U == 16 ? KT <= 4 : (U == 32 || U == 64 ? KT <= 2 : false));
}

int lstm_fused_slab(int U, int IN) {
  const int KT = (IN + 15) / 16;
  const int kt = KT <= 1 ? 1 : (KT <= 2 ? 2 : 4);   // the dispatch bucket
  return 4 * U * (16 * kt + U + 1);
}

int lstm_fused_dx_ld(int IN) {
  const int KT = (IN + 15) / 16;
  return 16 * (KT <= 1 ? 1 : (KT <= 2 ? 2 : 4));
}

bool lstm_fused_frag_supported(int U, int IN, bool x_bf16, bool want_dx) {
  const int KT = (IN + 15) / 16;
  return KT == 2 && ((U == 32 && !x_bf16 && !want_dx) || (U == 16 && x_bf16 && want_dx && IN == 32));
}

int64_t lstm_fused_dz_bytes(int64_t B, int T, int U) {   // DZS layers: [B/16 padded, T, 4U] bf16
  return U >= 64 ? (B + 15) / 16 * 16 * (int64_t)T * 4 * U * 2 : 0;
}

int lstm_fused_waves(int64_t B) { return (int)(((B + 16 * WAVES - 1) / (16 * WAVES)) * WAVES); }
int lstm_fused_slabs(int64_t B, int U, bool dx) {
  const int64_t nblk = (B + 16 * WAVES - 1) / (16 * WAVES);
  static const int cus = [] {
    int d = 0, n = 0;
    if (hipGetDevice(&d) != hipSuccess || hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, d) != hipSuccess)
      n = 0;
    return n > 0 ? n : 256;
  }();
  // resident workgroups per CU: the U = 32 layer without dX runs one wave per SIMD (register
  // fragments next to the AGPR accumulators), the other builds two
  const int64_t per_cu = ((U == 32 && !dx) || U >= 64) ? 1 : 2;
  static const bool persist = [] {   // SML_LSTM_PERSIST=0: one tile group per workgroup (A/B)
    const char* e = std::getenv("SML_LSTM_PERSIST");
    return !(e && e[0] == '0');
  }();
  return (int)(persist ? std::min<int64_t>(nblk, (int64_t)cus * per_cu) : nblk);
}

hipError_t lstm_fused_bwd_launch(const void* dh_bf16, const void* cseq_bf16, const void* hseq_bf16, const void* x,
                                 bool x_bf16, const float* h0, const float* c0, const float* W, const float* Uw,
                                 const float* b, void* dx, float* dh0, float* dc0, float* partials, int64_t B, int T,
                                 int IN, int U, int act, int dh_last_only, int64_t x_seq, void* dz_scratch,
                                 int frag, hipStream_t stream) {
  if (frag && !lstm_fused_frag_supported(U, IN, x_bf16, dx != nullptr)) return hipErrorInvalidValue;
  if (U >= 64 && dz_scratch == nullptr) return hipErrorInvalidValue;   // lstm_fused_dz_bytes
  if (lstm_split_applies(U, IN, dx != nullptr, x_bf16, dh_last_only != 0))   // two waves per tile (lstm_fused_split.hip)
    return lstm_split_bwd_launch(dh_bf16, cseq_bf16, hseq_bf16, x, x_bf16, h0, c0, W, Uw, b, dh0, dc0, partials, B, T,
                                 IN, act, dh_last_only, x_seq > 0 ? x_seq : (int64_t)T * IN, frag, stream);
  FusedBwdArgs a{(const __bf16*)dh_bf16, (const __bf16*)cseq_bf16, (const __bf16*)hseq_bf16, x, h0, c0, W, Uw, b, dx,
                 dh0, dc0, partials, B, T, IN, act, dh_last_only, x_seq > 0 ? x_seq : (int64_t)T * IN,
                 (__bf16*)dz_scratch, frag};
  return dispatch(U, IN, row_vec(x, IN, x_bf16 ? 2 : 4), x_bf16, [&](auto u, auto k, auto v, auto xt) {
    using XT = std::remove_const_t<std::remove_pointer_t<decltype(xt)>>;
    return launch_bwd<decltype(u)::value, decltype(k)::value, decltype(v)::value, XT>(a, stream);
  });
}

}  // namespace sml
