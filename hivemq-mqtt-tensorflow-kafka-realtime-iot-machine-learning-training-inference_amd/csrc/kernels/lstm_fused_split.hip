// sml-build: agpr-accumulators
//
// Unit-block split backward of a U = 32 fused LSTM layer without dX (the first layer of the
// stacked config-3 model, reference LSTM-TensorFlow-IO-Kafka/cardata-v2.py:177-183), for gfx950.
//
// Why: lstm_fused.hip runs this layer with one 16-sequence tile per wave, whose weight-gradient
// accumulators (dW^T | dU^T, 4U x (16 KT + U) fp32 = 128 AGPRs) plus register weight fragments and
// the BPTT state took 500 of the 512 registers: ONE wave per SIMD.  One wave alone issues a VALU
// instruction every ~4 cycles where two or more waves share the SIMD's 2-cycle rate
// (MI355X_MICROARCH.md, 'vector-instruction ISSUE cost'; profiles/r06 valu_rate), and this layer is
// VALU-bound: 368 VALU per step, 63 % of its cycles issuing VALU (profiles/r06/pmc/lstm_swizzled.txt).
//
// Here TWO waves share a tile, one per 16-unit block b (U = 32 = 2 blocks): wave b recomputes the
// 4 gate tiles of its own units (i, f, c~, o of units 16b..16b+15: tiles mt = 2q + b), runs their
// gate derivatives and owns their weight-gradient rows -- 64 registers of accumulators instead of
// 128.  The only cross-block coupling of BPTT is dh_{t-1} = U . dz_t, a contraction over ALL 4U
// gates: each step the two waves exchange their dz tiles through LDS (one barrier per step), and
// each computes its own unit block of dh_{t-1} with a 16x16x32 chain over the 8 gate tiles (own
// tile and partner tile of a gate as the two K halves).  The gate recompute uses the one-wave
// kernel's operands and order, so the gates are bit-identical to the forward's.
//
// Operand streaming: a step of a split wave is ~half the one-wave step, shorter than an HBM round
// trip under this load, and register prefetch buffers no longer fit beside the accumulators (a
// first build with loads two steps ahead in registers spilled and ran 394 us, waiting on memory:
// profiles/r06).  So every per-step operand -- c_{t-1}, dh_t, h_{t-1} and the x rows of the tile --
// is copied global -> LDS by the LDS-DMA engine (global_load_lds_dword[x4], no registers) into a
// ring of RD steps per tile, issued RD - 1 steps ahead by the tile's wave 0 and made visible to
// wave 1 by the step barrier; ordering is an explicit counted s_waitcnt vmcnt per step (the loop
// issues no other vector-memory instruction).
//
// dz exchange: the dz tiles are written once, in the XOR-swizzled transpose layout (sml_common.h
// tr_wr_off): the partner reads them back in C orientation (same lane offsets, the B operand of
// dh's MFMAs), the owner reads them transposed (ds_read_b64_tr_b16, the A operand of its weight
// gradients).  x_t and h_{t-1} tiles (the weight gradients' B operands) are written by one wave
// each (wave 0: x, wave 1: h) and read transposed by both.  Double-buffered by step parity.
//
// Workgroup: 4 waves = 2 tiles x 2 unit blocks, two workgroups per CU (eight waves, two per
// SIMD), persistent over 32-sequence groups; one fp32 slab [dW^T | dU^T | db] per workgroup as
// lstm_fused.hip writes it (slab_sum_kernel reduces them).  Bias modes BX / DB only (db is the
// dW^T column of a constant-1 x column), fp32 x, dh for every step; other layers keep the one-wave
// kernel (lstm_split_applies).
#include <cstdlib>

#include "lstm_fused_impl.h"

using namespace sml;
using namespace sml_lstm;

namespace {

struct SplitArgs {
  const __bf16* dh;    // [B, T, U] bf16 rows, fragment-native under FR
  const __bf16* cseq;  // fragment-native (the forward's)
  const __bf16* hseq;  // [B, T, U] bf16 rows, fragment-native under FR
  const float* x;      // [B, T, IN] fp32 rows (x_seq floats between sequences)
  const float* h0;
  const float* c0;
  const float* W;      // [IN, 4U]
  const float* Uw;     // [U, 4U]
  const float* bias;   // [4U]
  float* dh0;
  float* dc0;
  float* partials;     // [grid, S]
  int64_t B;
  int T, IN;
  int64_t x_seq;
};

constexpr int U = 32, G4 = 128, MT = 8, UB = 2;
constexpr int NTL = 12;                   // 512-byte LDS tiles per step buffer: 8 dz, 2 x, 2 h
constexpr int TILE_BUF = 2 * NTL * 512;   // per 16-sequence tile: two step slots
constexpr int RD = 4;                     // operand ring depth (steps)
constexpr int RSLOT = 5 * 1024;           // ring slot of a tile: c 1 K | dh 1 K | h 1 K | x rows <= 2 K
constexpr int RING = RD * RSLOT;

__device__ __forceinline__ bf16x4 lds_rd(const char* base, int off) { return *(const lds_bf16x4*)(base + off); }
__device__ __forceinline__ void lds_wr(char* base, int off, bf16x4 v) { *(lds_bf16x4*)(base + off) = v; }
__device__ __forceinline__ bf16x4 lds_rd_tr(const char* base, int off) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_bf16x4*)(base + off));
}
typedef __attribute__((address_space(3))) const f32x2_t lds_f2;
typedef __attribute__((address_space(3))) const float lds_f1;

// global -> LDS copies (LDS destination = M0 + 16 / 4 * lane), wave-uniform global base (SGPR pair) +
// per-lane 32-bit offset.  Inline asm, as ae_fused.hip's ring: the compiler cannot see that the
// ring is disjoint from what the loop reads and would drain it with vmcnt(0) before LDS reads.
#pragma clang diagnostic push
#pragma clang diagnostic ignored "-Winline-asm"   // m0 is deliberately clobbered
__device__ __forceinline__ void dma16(const void* g, unsigned voff, unsigned m0) {
  asm volatile("s_mov_b32 m0, %0\n\tglobal_load_lds_dwordx4 %1, %2" ::"s"(m0), "v"(voff), "s"(g) : "memory", "m0");
}
__device__ __forceinline__ void dma4(const void* g, unsigned voff, unsigned m0) {
  asm volatile("s_mov_b32 m0, %0\n\tglobal_load_lds_dword %1, %2" ::"s"(m0), "v"(voff), "s"(g) : "memory", "m0");
}
#pragma clang diagnostic pop
template <int N>
__device__ __forceinline__ void wait_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// KT: x K-tiles (IN <= 16 KT); FR: h and dh fragment-native (the stacked model) instead of [B, T, U]
// rows.  The x rows are copied 4 bytes per lane (global_load_lds_dwordx3 does not place lane i's 12 bytes
// at M0 + 12 i: measured wrong, tools/debug/split_diag.py)
// NTW: 16-sequence tiles per workgroup (2: four waves, two workgroups per CU; 1: two waves, four per CU --
// the step barrier then couples only the tile's pair)
template <int KT, int ACT, int BM, bool FR, int NTW>
__global__ __launch_bounds__(NTW * 128, 2) void lstm_split_bwd_kernel(SplitArgs a) {
  constexpr int SPW = 2 * NTW;   // waves per workgroup
  static_assert(BM != BM_PLAIN, "db comes from the constant-1 x column");
  constexpr bool BX = BM == BM_BX;
  constexpr int LDW = 16 * KT, NK = KT + UB;
  constexpr int S = G4 * (LDW + U + 1);
  constexpr int STEP_BYTES = NTW * TILE_BUF, MAIN = STEP_BYTES + NTW * RING;
  constexpr int LDS_BYTES = (S * 4 > MAIN) ? S * 4 : MAIN;
  // x DMA instructions per step: 16 rows x IN floats, one float per lane, always NXMAX (enough for
  // IN = 16 KT - 1; pieces past 16 IN re-read row 0 into the slot's unused x bytes) -- branch-free
  constexpr int NXMAX = (16 * (16 * KT - 1) + 63) / 64, NXH = NXMAX / 2;
  // DMA instructions per step and wave: wave 0 c + dh + the first NXH x pieces, wave 1 h + the rest
  // (c, dh, h are one 16-byte copy each fragment-native, dh / h four 4-byte gathers as rows)
  constexpr int G0 = (FR ? 2 : 5) + NXH, G1 = (FR ? 1 : 4) + (NXMAX - NXH);
  // the step buffers and operand rings while the tiles run, the workgroup's slab after the last one
  __shared__ __attribute__((aligned(16))) char lds[LDS_BYTES];
  const int lane = threadIdx.x & 63, c = lane & 15, g = lane >> 4;
  // wave-uniform (SGPR) wave index: ring bookkeeping and every DMA base stay scalar
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), p = w >> 1, b = w & 1;   // tile slot, unit block
  const int IN = a.IN, T = a.T;
  const int wro = tr_wr_off(c, g), rdo = tr_rd_off(c, g);
  char* tb = lds + p * TILE_BUF;                   // this tile's two step slots
  const char* rg = lds + STEP_BYTES + p * RING;    // this tile's operand ring
  const unsigned rg_lds = (unsigned)(uintptr_t)((__attribute__((address_space(3))) char*)lds) + STEP_BYTES + p * RING;

  // A fragments (registers for the launch).  rw[q][k]: tile (mt = 2q + b, k) of [W^T | U^T]
  // (forward orientation, the gate recompute); ruo[q] / rup[q]: U[unit 16b + c][gate 16 mt + 4g + j]
  // of gate tile mt = 2q + b (own) / 2q + 1 - b (the partner's), the K halves of dh's MFMAs.
  bf16x4 rw[4][NK], ruo[4], rup[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int mt = 2 * q + b;
#pragma unroll
    for (int k = 0; k < NK; ++k) {
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
      rw[q][k] = pack4(t4);
    }
    f32x4 t4, u4;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      t4[j] = a.Uw[(16 * b + c) * G4 + 16 * (2 * q + b) + 4 * g + j];
      u4[j] = a.Uw[(16 * b + c) * G4 + 16 * (2 * q + 1 - b) + 4 * g + j];
    }
    ruo[q] = pack4(t4);
    rup[q] = pack4(u4);
  }
  f32x4 bz[BX ? 1 : 4];   // DB: the bias rows of the own gate tiles (BX: inside the fragments)
  if constexpr (!BX) {
#pragma unroll
    for (int q = 0; q < 4; ++q) bz[q] = *reinterpret_cast<const f32x4*>(a.bias + 16 * (2 * q + b) + 4 * g);
  }
  bf16x4 onex[KT];
#pragma unroll
  for (int kt = 0; kt < KT; ++kt) onex[kt] = ones_at_bias(kt, g, IN);

  const f32x4 zero4 = {0.f, 0.f, 0.f, 0.f};
  f32x4 accW[4][KT], accU[4][UB];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
#pragma unroll
    for (int kt = 0; kt < KT; ++kt) accW[q][kt] = zero4;
#pragma unroll
    for (int ub = 0; ub < UB; ++ub) accU[q][ub] = zero4;
  }

  const int P = IN, npc = 16 * P;   // x pieces: 16 rows x IN floats
  const int64_t ntile = (a.B + 15) / 16;
  const int64_t ngrp = (ntile + NTW - 1) / NTW;
  bool any_active = false;
  f32x4 dhr, dcn, ctc;
  int64_t lt = 0;     // the tile whose rows this wave reads (uniform)
  bool valid = false;
  unsigned xoff[NXMAX], goff[4];   // per-lane DMA source offsets of the tile

  struct Ops {
    bf16x4 cprev;      // c_{t-1}, own unit block
    bf16x4 dho;        // incoming dh_t, own unit block
    bf16x4 hp[UB];     // h_{t-1}, both blocks (the recompute's and dU's operand)
    f32x4 xt[KT];      // x_t row piece: features 16kt + 4g + j of sequence c (columns past IN: junk, masked)
  };
  // step s's operands -> ring slot s % RD, shared by the tile's two waves (G0 / G1 instructions)
  auto issue = [&](int s) {
    const unsigned dst = rg_lds + (unsigned)(s & (RD - 1)) * RSLOT;
    const int sm1 = s > 0 ? s - 1 : 0;   // c_{s-1}, h_{s-1}; s = 0 takes c0 / h0 instead (a dummy copy)
    const char* xg = reinterpret_cast<const char*>(a.x) + (lt * 16 * a.x_seq + (int64_t)s * IN) * 4;
    if (b == 0) {
      dma16(reinterpret_cast<const char*>(a.cseq) + (lt * T + sm1) * 1024, lane * 16, dst);
      if constexpr (FR) {
        dma16(reinterpret_cast<const char*>(a.dh) + (lt * T + s) * 1024, lane * 16, dst + 1024);
      } else {   // [B, T, U] rows gathered into the fragment-native image, 4 bytes per lane
        const char* dg = reinterpret_cast<const char*>(a.dh) + ((lt * 16) * T + s) * (int64_t)(U * 2);
#pragma unroll
        for (int k = 0; k < 4; ++k) dma4(dg, goff[k], dst + 1024 + k * 256);
      }
#pragma unroll
      for (int i = 0; i < NXH; ++i) dma4(xg, xoff[i], dst + 3072 + i * 256);
    } else {
      if constexpr (FR) {
        dma16(reinterpret_cast<const char*>(a.hseq) + (lt * T + sm1) * 1024, lane * 16, dst + 2048);
      } else {
        const char* hg = reinterpret_cast<const char*>(a.hseq) + ((lt * 16) * T + sm1) * (int64_t)(U * 2);
#pragma unroll
        for (int k = 0; k < 4; ++k) dma4(hg, goff[k], dst + 2048 + k * 256);
      }
#pragma unroll
      for (int i = NXH; i < NXMAX; ++i) dma4(xg, xoff[i], dst + 3072 + i * 256);
    }
  };
  // the ring slot of step s -> registers (both waves; the slot's group has landed and the step
  // barrier since has made it visible)
  auto ring_read = [&](int s, Ops& o) {
    const char* sl = rg + (s & (RD - 1)) * RSLOT;
    o.cprev = lds_rd(sl, b * 512 + lane * 8);
    o.dho = lds_rd(sl, 1024 + b * 512 + lane * 8);
#pragma unroll
    for (int ub = 0; ub < UB; ++ub) o.hp[ub] = lds_rd(sl, 2048 + ub * 512 + lane * 8);
    const char* xr = sl + 3072 + c * IN * 4;
#pragma unroll
    for (int kt = 0; kt < KT; ++kt) {
      const int k0 = 16 * kt + 4 * g;
      if ((IN & 1) == 0) {
        const f32x2_t lo = *(lds_f2*)(xr + 4 * (k0 < IN ? k0 : 0));
        const f32x2_t hi = *(lds_f2*)(xr + 4 * (k0 + 2 < IN ? k0 + 2 : 0));
        o.xt[kt] = f32x4{lo[0], lo[1], hi[0], hi[1]};
      } else {
#pragma unroll
        for (int j = 0; j < 4; ++j) o.xt[kt][j] = *(lds_f1*)(xr + 4 * (k0 + j < IN ? k0 + j : 0));
      }
    }
  };

  // one BPTT step, first half: recompute, gate derivatives, dz tiles out (step buffer slot sl)
  auto step_a = [&](int t, const Ops& cur, int sl, bf16x4 (&dzb)[4]) {
    char* sb = tb + sl * (NTL * 512);
    bf16x4 xb[KT];
#pragma unroll
    for (int kt = 0; kt < KT; ++kt) xb[kt] = row_operand(cur.xt[kt], 16 * kt + 4 * g, IN) | onex[kt];
    f32x4 z[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      if constexpr (BX) z[q] = zero4;
      else z[q] = bz[q];
#pragma unroll
      for (int k = 0; k + 1 < NK; k += 2)
        z[q] = mfma32(rw[q][k], rw[q][k + 1], k < KT ? xb[k] : cur.hp[k - KT], k + 1 < KT ? xb[k + 1] : cur.hp[k + 1 - KT],
                      z[q]);
      if constexpr (NK & 1) z[q] = mfma32(rw[q][NK - 1], bf16x4{0, 0, 0, 0}, cur.hp[UB - 1], bf16x4{0, 0, 0, 0}, z[q]);
    }
    const f32x4 cp = unpack4(cur.cprev), dhi = unpack4(cur.dho);
    f32x4 dzt[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const float gi = sigmoid_fast(z[0][i]), gf = sigmoid_fast(z[1][i]);
      const float gc = act_f(ACT, z[2][i]), go = sigmoid_fast(z[3][i]);
      const float dh = (valid ? dhi[i] : 0.f) + dhr[i];
      const float ct = ctc[i];
      const float ac = act_f(ACT, ct);
      const float dhgo = dh * go;
      const float dc = ACT == ACT_RELU ? (ct > 0.f ? dcn[i] + dhgo : dcn[i]) : fmaf(dhgo, fmaf(-ac, ac, 1.f), dcn[i]);
      const float di = dc * gi;
      const float df = dc * gf;
      dzt[0][i] = (dc * gc) * fmaf(-gi, gi, gi);
      dzt[1][i] = fmaf(-df, gf, df) * cp[i];
      dzt[2][i] = ACT == ACT_RELU ? (gc > 0.f ? di : 0.f) : di * fmaf(-gc, gc, 1.f);
      dzt[3][i] = (dh * ac) * fmaf(-go, go, go);
      dcn[i] = df;
    }
    ctc = cp;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      dzb[q] = pack4(dzt[q]);
      lds_wr(sb, (2 * q + b) * 512 + wro, dzb[q]);
    }
    if constexpr (KT == 2) {   // wave 0 writes the x tiles, wave 1 the h tiles (selects, no branch)
#pragma unroll
      for (int k = 0; k < 2; ++k) lds_wr(sb, (8 + 2 * b + k) * 512 + wro, b ? cur.hp[k] : xb[k]);
    } else {                   // both waves write every x / h tile (identical bytes)
#pragma unroll
      for (int kt = 0; kt < KT; ++kt) lds_wr(sb, (8 + kt) * 512 + wro, xb[kt]);
#pragma unroll
      for (int ub = 0; ub < UB; ++ub) lds_wr(sb, (10 + ub) * 512 + wro, cur.hp[ub]);
    }
  };
  // second half (after the step barrier): dh_{t-1} of the own unit block, weight gradients
  auto step_b = [&](int sl, const bf16x4 (&dzb)[4]) {
    const char* sb = tb + sl * (NTL * 512);
    bf16x4 dzo[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) dzo[q] = lds_rd(sb, (2 * q + 1 - b) * 512 + wro);
    f32x4 acc = zero4;
#pragma unroll
    for (int q = 0; q < 4; ++q) acc = mfma32(ruo[q], rup[q], dzb[q], dzo[q], acc);   // K halves: own, partner
    dhr = acc;
    bf16x4 xB[KT], hB[UB];
#pragma unroll
    for (int kt = 0; kt < KT; ++kt) xB[kt] = lds_rd_tr(sb, (8 + kt) * 512 + rdo);
#pragma unroll
    for (int ub = 0; ub < UB; ++ub) hB[ub] = lds_rd_tr(sb, (10 + ub) * 512 + rdo);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const bf16x4 adz = lds_rd_tr(sb, (2 * q + b) * 512 + rdo);
#pragma unroll
      for (int kt = 0; kt < KT; ++kt) accW[q][kt] = mfma16(adz, xB[kt], accW[q][kt]);
#pragma unroll
      for (int ub = 0; ub < UB; ++ub) accU[q][ub] = mfma16(adz, hB[ub], accU[q][ub]);
    }
  };
  // wave 0: step s - 1's group has landed (n = the groups issued after it, min(RD - 2, s - 1))
  auto wait_group = [&](int s) {
    if (s - 1 >= RD - 2) {
      if (b == 0) wait_vm<G0 * (RD - 2)>();
      else wait_vm<G1 * (RD - 2)>();
    } else {
      wait_vm<0>();
    }
  };

  for (int64_t grp = blockIdx.x; grp < ngrp; grp += gridDim.x) {   // workgroup-uniform trip count
    const int64_t tile = grp * NTW + p;
    const bool active = tile < ntile;
    any_active |= active;
    lt = active ? tile : ntile - 1;   // an idle tile reads the last real one's rows (its dz stays 0)
    const int nvalid = (int)((a.B - lt * 16) < 16 ? (a.B - lt * 16) : 16);   // rows of the tile inside B
    valid = active && c < nvalid;
#pragma unroll
    for (int k = 0; k < 4; ++k) {   // row gathers: fragment-native byte k*256 + 4 lane of a 512-byte block pair
      const int pos = k * 256 + lane * 4, lp = pos >> 3, half = (pos >> 2) & 1;
      const int l2 = lp & 63, cc = l2 & 15, gg = l2 >> 4, ub = lp >> 6;
      const int cr = cc < nvalid ? cc : nvalid - 1;
      goff[k] = (unsigned)((cr * T * U + 16 * ub + 4 * gg + 2 * half) * 2);
    }
#pragma unroll
    for (int i = 0; i < NXMAX; ++i) {   // x pieces: row r, float q
      const int k = 64 * i + lane, r = k / P, q = k % P;
      const int rr = r < nvalid ? r : nvalid - 1;
      xoff[i] = k < npc ? (unsigned)((rr * a.x_seq + q) * 4) : 0u;
    }
    ctc = unpack4(ld_bf16x4(a.cseq + (lt * T + (T - 1)) * (int64_t)(UB * 256) + b * 256 + lane * 4));
    dhr = dcn = zero4;
    // retire every compiler-visible load / store (this tile's c_T, the last tile's dh0 / dc0) before
    // the ring: the per-step waits count only DMA
    __builtin_amdgcn_s_waitcnt(0x0F70);   // vmcnt(0) expcnt(7) lgkmcnt(15)
    for (int s = T - 1; s >= 0 && s >= T - (RD - 1); --s) issue(s);
    wait_group(T);
    __syncthreads();   // group T - 1 visible to wave 1; the previous tile's step buffers are free
    Ops cur;
    ring_read(T - 1, cur);
    for (int t = T - 1; t >= 1; --t) {
      if (t - (RD - 1) >= 0) issue(t - (RD - 1));
      bf16x4 dzb[4];
      step_a(t, cur, t & 1, dzb);
      wait_group(t);
      __syncthreads();
      ring_read(t - 1, cur);   // step t - 1's operands (group t - 1 landed before this barrier)
      step_b(t & 1, dzb);
    }
    // step 0 from the initial state: c_{-1} = c0, h_{-1} = h0 (the ring is drained: group 0 was
    // waited with vmcnt(0) before the last barrier)
    {
      const int64_t sq = lt * 16 + (valid ? c : nvalid - 1);
      cur.cprev = a.c0 ? pack4(*reinterpret_cast<const f32x4*>(a.c0 + sq * U + 16 * b + 4 * g)) : pack4(zero4);
#pragma unroll
      for (int ub = 0; ub < UB; ++ub)
        cur.hp[ub] = pack4(a.h0 ? *reinterpret_cast<const f32x4*>(a.h0 + sq * U + 16 * ub + 4 * g) : zero4);
      bf16x4 dzb[4];
      step_a(0, cur, 0, dzb);
      __syncthreads();
      step_b(0, dzb);
    }
    if (valid) {
      const int64_t off = (lt * 16 + c) * U + 16 * b + 4 * g;
      if (a.dh0) *reinterpret_cast<f32x4*>(a.dh0 + off) = dhr;
      if (a.dc0) *reinterpret_cast<f32x4*>(a.dc0 + off) = dcn;
    }
    __syncthreads();   // step 0's buffer reads done before the next tile's first writes
  }

  // slab: the step buffers and rings are dead; the 4 waves add their rows in a fixed order
  __syncthreads();
  float* slab = reinterpret_cast<float*>(lds);
  for (int i = threadIdx.x; i < S; i += SPW * 64) slab[i] = 0.f;
  for (int turn = 0; turn < SPW; ++turn) {
    __syncthreads();
    if (turn == w && any_active) {
#pragma unroll
      for (int q = 0; q < 4; ++q)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int m = 16 * (2 * q + b) + 4 * g + i;
#pragma unroll
          for (int kt = 0; kt < KT; ++kt) slab[m * LDW + 16 * kt + c] += accW[q][kt][i];
#pragma unroll
          for (int ub = 0; ub < UB; ++ub) slab[G4 * LDW + m * U + 16 * ub + c] += accU[q][ub][i];
        }
    }
  }
  __syncthreads();
  // db = column IN of dW^T (a constant-1 input); columns IN, IN + 1 are padding
  for (int m = threadIdx.x; m < G4; m += SPW * 64) {
    slab[G4 * LDW + G4 * U + m] = slab[m * LDW + IN];
    slab[m * LDW + IN] = 0.f;
    if (IN + 1 < LDW) slab[m * LDW + IN + 1] = 0.f;
  }
  __syncthreads();
  float* out = a.partials + (int64_t)blockIdx.x * S;
  for (int i = threadIdx.x; i < S; i += SPW * 64) out[i] = slab[i];
}

// Off by default: measured SLOWER than the one-wave kernel on the seq-50 layer (config 3 A/B, same box:
// 90.7 M windows/s with NTW 2 and 93.4 M with NTW 1 against 100.1 M one-wave; the layer's kernel 328 vs
// 280 us).  Per wave and step it issues ~200 VALU + ~55 SALU and waits ~1 000 cycles on the dz-exchange
// chain and the step barrier: ~3 000 cycles per half-tile step against the one-wave kernel's ~2 650
// per whole-tile step (profiles/r06/SUMMARY.md section 6).  SML_LSTM_SPLIT=1 selects it (A/B; read per
// call, the tests flip it).
bool split_env() {
  const char* e = std::getenv("SML_LSTM_SPLIT");
  return e && e[0] == '1';
}
int split_ntw() {    // SML_LSTM_SPLIT_NTW=1|2: tiles per workgroup (A/B; read per call: grid and launch agree)
  const char* e = std::getenv("SML_LSTM_SPLIT_NTW");
  return e && e[0] == '1' ? 1 : 2;
}

int cu_count() {
  static const int cus = [] {
    int d = 0, n = 0;
    if (hipGetDevice(&d) != hipSuccess || hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, d) != hipSuccess)
      n = 0;
    return n > 0 ? n : 256;
  }();
  return cus;
}

}  // namespace

namespace sml {

bool lstm_split_applies(int U_, int IN, bool dx, bool x_bf16, bool dh_last_only) {
  const int KT = (IN + 15) / 16;
  return split_env() && U_ == 32 && !dx && !x_bf16 && !dh_last_only && IN >= 3 && KT <= 2 &&
         bias_mode(IN, KT) != BM_PLAIN;
}

int lstm_split_grid(int64_t B) {   // eight waves per CU (two per SIMD), persistent
  const int ntw = split_ntw();
  const int64_t ngrp = ((B + 15) / 16 + ntw - 1) / ntw;
  return (int)std::max<int64_t>(1, std::min<int64_t>(ngrp, (int64_t)cu_count() * (4 / ntw)));
}

hipError_t lstm_split_bwd_launch(const void* dh, const void* cseq, const void* hseq, const void* x, bool x_bf16,
                                 const float* h0, const float* c0, const float* W, const float* Uw, const float* b,
                                 float* dh0, float* dc0, float* partials, int64_t B, int T, int IN, int act,
                                 int dh_last_only, int64_t x_seq, int frag, hipStream_t st) {
  if (!lstm_split_applies(32, IN, false, x_bf16, dh_last_only != 0) || T < 1 || B < 1) return hipErrorInvalidValue;
  if (act != ACT_RELU && act != ACT_TANH) return hipErrorInvalidValue;
  const int KT = (IN + 15) / 16;
  if (frag && KT != 2) return hipErrorInvalidValue;
  SplitArgs a{(const __bf16*)dh, (const __bf16*)cseq, (const __bf16*)hseq, (const float*)x, h0, c0, W, Uw, b, dh0, dc0,
              partials, B, T, IN, x_seq};
  const int bm = bias_mode(IN, KT);
  const int ntw = split_ntw();
  const dim3 grid(lstm_split_grid(B)), block(ntw * 128);
  auto go = [&](auto kt, auto fr) {
    constexpr int K = decltype(kt)::value;
    constexpr bool FRc = decltype(fr)::value;
    auto launch = [&](auto kern) { hipLaunchKernelGGL(kern, grid, block, 0, st, a); };
    auto with_ntw = [&](auto bmc, auto actc) {
      constexpr int BMc = decltype(bmc)::value, ACc = decltype(actc)::value;
      if (ntw == 1) launch(lstm_split_bwd_kernel<K, ACc, BMc, FRc, 1>);
      else launch(lstm_split_bwd_kernel<K, ACc, BMc, FRc, 2>);
    };
    using BXc = std::integral_constant<int, BM_BX>;
    using DBc = std::integral_constant<int, BM_DB>;
    using RE = std::integral_constant<int, ACT_RELU>;
    using TA = std::integral_constant<int, ACT_TANH>;
    if (bm == BM_BX) {
      if (act == ACT_RELU) with_ntw(BXc{}, RE{});
      else with_ntw(BXc{}, TA{});
    } else {
      if (act == ACT_RELU) with_ntw(DBc{}, RE{});
      else with_ntw(DBc{}, TA{});
    }
    return hipGetLastError();
  };
  using K1 = std::integral_constant<int, 1>;
  using K2 = std::integral_constant<int, 2>;
  if (frag) return go(K2{}, std::true_type{});
  return KT <= 1 ? go(K1{}, std::false_type{}) : go(K2{}, std::false_type{});
}

}  // namespace sml
