// sml-build: no-slp
// Persistent small-batch autoencoder trainer for gfx950 (MI355X).
//
// The reference trains its dense autoencoder with Keras `fit`: batch 100 in
// cardata-v3 (AUTOENCODER-TensorFlow-IO-Kafka/cardata-v3.py:176-177, 212-222), batch 32
// in cardata-v1 and the creditcard notebooks -- one Adam update per small batch.  A
// launch-per-step design is launch-bound there (~10 us per step).  This kernel keeps the
// whole optimizer loop on the device: ONE workgroup runs `nsteps` sequential Keras steps
// -- normalise, forward, MSE + L1 activity loss, categorical accuracy, backward, weight
// gradients, Adam -- with parameters, Adam moments and activations on chip.  Only the
// next batch's rows come from HBM, prefetched into registers one step ahead.  All
// arithmetic is fp32 (v_mfma_f32_16x16x4_f32 is an exact fp32 fma chain), so this is
// also the exact-semantics path: it matches an fp32 PyTorch Keras-Adam run to
// summation-order rounding.
//
// Step structure (512 threads = 8 waves, batch B <= 128 = 8 row tiles of 16):
//   phase A  wave w owns rows 16w..16w+15.  The forward and the activation-gradient
//            backward run entirely in registers on fp32 MFMA in FEATURE-MAJOR
//            orientation: a layer computes Z^T = W^T . H^T, whose C/D layout
//            (lane (c, g) holds Z^T[4g+i][row c]) is exactly the B-operand layout of the
//            next layer's K-steps (K-step s takes register s&3 of output tile s>>2, so
//            lane group g contributes feature f(s,g) = 16(s>>2) + 4g + (s&3)); the A
//            operand (weights) is read in that same permuted K order from LDS images
//            stored in fragment order (one contiguous 256-byte block per K-step: no
//            bank conflicts).  Bias = the accumulator's initial value.  Loss and the L1
//            activity term are lane-local.  The wave then stores its activations /
//            gradients / reconstructions [row][feature] to LDS (column-swizzled, see
//            swz()).
//   barrier
//   phase B  waves 0-5 each own one 16x16 tile of the padded parameter image: weight
//            gradient act^T . dz over the B rows (fp32 MFMA, K = 4 rows per
//            instruction, bias rows read a constant 1), then Keras Adam on the 4
//            parameters per lane they hold in registers for the whole launch, and
//            write the new values into the forward / backward weight fragments;
//            waves 6-7 take the argmax accuracy of one row per lane meanwhile (off the
//            critical path: the same argmax in phase A, on the row waves, cost
//            0.4-0.5 us per step, profiles/r03).
//   barrier
// Two barriers per step (the round-1 version had eight, one per layer phase, and did
// every dot product on the VALU: 12 us per batch-100 step).  At batch 32 (two row waves)
// ae_minibatch_pipe_kernel below replaces the barriers with LDS stage counters and runs the
// tile gradients + Adam of W2-W4 under the backward pass.
//
// Fleet mode: a grid of M workgroups trains M independent models at once (per-device
// digital-twin models, ensembles, learning-rate sweeps), one per workgroup, each with
// its own parameters, optimizer state, ring cursor and metrics.
#include "sml_common.h"
#include "sml_ops.h"
#include "sml_p2p.h"

#include <type_traits>

using namespace sml;

namespace {

constexpr int NT = 512;   // 8 waves: one 16-row tile each in phase A
// LDS capacity classes (rows per step): 48 keeps Smem small so two fleet models share a
// CU (Keras default batch 32); 128 covers cardata-v3's batch 100 (one workgroup per CU).
constexpr int MB_SMALL = 48, MB_LARGE = 128, MAXB = MB_LARGE;
// activation row strides in LDS (floats): 16 and 48 are 16 (mod 32), so the phase-B
// reads of rows r and r+1 by the two 16-lane halves of a ds_read_b32 group never share a bank
constexpr int XS = 48;   // x / dz4 rows (<= 32 features)
constexpr int HS = 16;   // hidden rows (<= 16 features)
// Column swizzle of those rows: feature f of row r lives at column f ^ swz(r).  A phase-A
// ds_write_b128 is serviced in 8-lane groups (rows 16w + 0..7 of one column block, bank =
// dword mod 32): unswizzled, rows r and r + 2 hit the same 16-byte bank slot (4-way
// conflict, ~60 % of the kernel's SQ_LDS_BANK_CONFLICT, profiles/r03); swizzled, the 8 rows
// cover 8 distinct slots.  The phase-B ds_read_b32 groups read rows 4 s4 + {0, 1} (or
// {2, 3}) -- one swz value per group -- so they stay conflict-free.
__device__ __forceinline__ int swz(int r) { return 4 * ((r >> 1) & 3); }
// padded parameter image (ae_fused.hip / ops/ae.py LAYOUT): L1 [32][16] @0 (bias row 31),
// L2 [16][16] @512, L3 @768 (bias row 15), L4 [16][32] @1024 (bias row 15)
constexpr int IMG2 = 512, IMG3 = 768, IMG4 = 1024, NPARAM = 1536;
// LDS weight fragments (floats), one 64-float block per K-step, in lane order
constexpr int F1 = 0;                 // fwd L1: [8 K-steps][64]    A = W1[f(s,g)][c]
constexpr int F2 = F1 + 8 * 64;       // fwd L2: [4][64]            A = W2[4g+s][c]
constexpr int F3 = F2 + 4 * 64;       // fwd L3: [4][64]
constexpr int F4 = F3 + 4 * 64;       // fwd L4: [2 tiles][4][64]   A = W4[4g+s][16t+c]
constexpr int G4 = F4 + 8 * 64;       // bwd dz3: [8][64]           A = W4[c][f(s,g)]
constexpr int G3 = G4 + 8 * 64;       // bwd dz2: [4][64]           A = W3[c][4g+s]
constexpr int G2 = G3 + 4 * 64;       // bwd dz1: [4][64]           A = W2[c][4g+s]
constexpr int BB1 = G2 + 4 * 64, BB2 = BB1 + 16, BB3 = BB2 + 16, BB4 = BB3 + 16, W_END = BB4 + 32;

struct MBArgs {
  const float* x;       // ring [ring][ld] of raw rows
  int64_t ld, ring;     // row stride, ring rows (multiple of B)
  int64_t* cursor;      // ring read position (rows), advanced by B per step
  const float* scale;   // [D] fused normalize_fn, may be null
  const float* shift;
  float* params;        // padded image [1536]
  float* m;
  float* v;
  int64_t* iter;
  float* metrics;       // {sum sq err, sum |h1|, correct, rows} (+=)
  int B, nsteps, D, n1, n2, n3, a1, a2, a3, a4;
  float l1, lr, beta1, beta2, eps, gscale;
  int want_acc;
  unsigned long long* prof;   // optional [11]: per-phase cycles summed over steps (wave 0, model 0):
                              // 0 phase A, 1 barrier 1, 2 phase B (gradients + Adam), 3 barrier 2, 8 total
  // fleet mode: workgroup b trains model b.  params / m / v are [M][NPARAM], iter /
  // cursor [M], metrics [M][4]; model b reads x + b * xmodel (0 = one shared ring).
  int64_t xmodel;
  const float* lrs;     // optional [M] per-model learning rates (hyper-parameter sweeps)
  const int64_t* ragged;   // optional [M][3] {first row, ring rows, steps}: models of different
                           // sizes in one flat row array, each taking its own number of steps
  // data parallelism at Keras granularity (runtime/p2p.h): every step's gradient tile is
  // pushed to every peer rank's receive buffer and the world's partials are summed in
  // rank order before Adam.  Rank = dp_rank0 + blockIdx.x (one process per GPU launches
  // one workgroup; in-launch ranks = a fleet of replicas).  dp_ranks <= 1: off.
  uint64_t* const* dp_peers;
  int dp_ranks, dp_rank0;
  int* dp_status;           // set to 1 when a peer's gradient never arrived (timeout)
  long long dp_timeout;     // s_memrealtime ticks (100 MHz)
  // Streaming epoch (runtime/stream_ring.h): rows are still arriving while the kernel runs.
  // The host publishes the rows copied into the ring so far (sr_avail: absolute count,
  // host-mapped, written by the copy stream after each copy) and, once the stream has
  // ended, the total (sr_total, -1 before).  The kernel waits for each next batch, stops
  // when the next full batch would pass the total, and reports the rows it no longer needs
  // (sr_consumed: back-pressure).  Ring memory is uncached (a copy on another engine must
  // never be shadowed by a stale line of the previous lap).  Null: a resident ring.
  const int64_t* sr_avail;
  const int64_t* sr_total;
  int64_t* sr_consumed;
  int* sr_status;           // 1 = no rows arrived within sr_timeout
  long long sr_timeout;
};

template <int MB>
struct Smem {   // MB 48: ~47 KB, MB 128: ~108 KB
  float w[W_END];
  float x[MB * XS];                     // normalised inputs (phase-B activation of L1)
  float h1[MB * HS], h2[MB * HS], h3[MB * HS];
  float dz4[MB * XS];
  float dz3[MB * HS], dz2[MB * HS], dz1[MB * HS];
  float y[MB * XS];                     // reconstructions (phase-B argmax accuracy)
  float one[4];                         // constant 1 (bias-row activation), dummy store slot
  float red[3][16];                     // per-wave partial metrics (<= 16 waves)
  int abort;                            // DP: a gradient exchange timed out (all waves stop)
  int stream_end;                       // streaming: no further full batch (all waves stop)
  alignas(16) unsigned cnt[8];          // pipelined build: stage counters (CE1.., CU1..)
  int stream_last;                      // pipelined build, streaming: index of the last step (INT_MAX: open)
  int first_ok;                         // pipelined build, streaming: the first batch arrived (1)
};

// logical feature of K-step s for lane group g (the C/D register order of the producer)
__host__ __device__ constexpr int feat(int s, int g) { return 16 * (s >> 2) + 4 * g + (s & 3); }

// LDS positions of parameter image slot p in the forward-operand and backward-operand
// fragment images (`none` = not used there: a dummy word, so the stores need no branch).
// Bias rows go to the bias vectors only.
__device__ __forceinline__ void lds_slots(int p, int& fw, int& bw, int none) {
  fw = bw = none;
  if (p < IMG2) {
    const int k = p >> 4, j = p & 15;
    if (k == 31) { fw = BB1 + j; return; }
    fw = F1 + (4 * (k >> 4) + (k & 3)) * 64 + 16 * ((k & 15) >> 2) + j;
  } else if (p < IMG4) {
    const bool l2 = p < IMG3;
    const int base = l2 ? IMG2 : IMG3;
    const int k = (p - base) >> 4, j = (p - base) & 15;
    if (k == 15) { fw = (l2 ? BB2 : BB3) + j; return; }
    fw = (l2 ? F2 : F3) + (k & 3) * 64 + 16 * (k >> 2) + j;
    bw = (l2 ? G2 : G3) + (j & 3) * 64 + 16 * (j >> 2) + k;
  } else {
    const int k = (p - IMG4) >> 5, j = (p - IMG4) & 31;
    if (k == 15) { fw = BB4 + j; return; }
    fw = F4 + (4 * (j >> 4) + (k & 3)) * 64 + 16 * (k >> 2) + (j & 15);
    bw = G4 + (4 * (j >> 4) + (j & 3)) * 64 + 16 * ((j & 15) >> 2) + k;
  }
}

// One 16x16 tile of the padded image whose gradient a phase-B wave computes with fp32
// MFMAs (K = 4 batch rows per instruction).  Tiles: 0/1 = L1 rows 0-15 / 16-31, 2 = L2,
// 3 = L3, 4/5 = L4 cols 0-15 / 16-31; wave w < 6 owns tile w.
struct Tile {
  int act, as, am;  // activation base (float offset into Smem), row stride, this lane's column;
                    // a bias-row lane reads the constant-1 word with stride 0 (branch-free)
  int dz, ds, dc;   // upstream-gradient base, row stride, this lane's column
  int slot0, sst;   // image slots of C[4g+i][c]: slot0 + i * sst (consecutive image rows)
  __device__ __forceinline__ int slot(int i) const { return slot0 + i * sst; }
};

template <class SM>
__device__ __forceinline__ Tile make_tile(int id, int c, int g, const SM& S, const float* sbase) {
  Tile T;
  int row0 = 0, col0 = 0, img = 0, istride = 16, bias_row = 15;
  if (id <= 1) {
    row0 = 16 * id; bias_row = 31;
    T.act = (int)(S.x - sbase); T.as = XS; T.dz = (int)(S.dz1 - sbase); T.ds = HS;
  } else if (id == 2) {
    img = IMG2; T.act = (int)(S.h1 - sbase); T.as = HS; T.dz = (int)(S.dz2 - sbase); T.ds = HS;
  } else if (id == 3) {
    img = IMG3; T.act = (int)(S.h2 - sbase); T.as = HS; T.dz = (int)(S.dz3 - sbase); T.ds = HS;
  } else {
    col0 = 16 * (id - 4); img = IMG4; istride = 32;
    T.act = (int)(S.h3 - sbase); T.as = HS; T.dz = (int)(S.dz4 - sbase); T.ds = XS;
  }
  const int m = row0 + c;
  T.am = m;
  if (m == bias_row) {
    T.act = (int)(S.one - sbase);
    T.as = 0;
  }
  T.dc = col0 + c;
  T.slot0 = img + (row0 + 4 * g) * istride + col0 + c;
  T.sst = istride;
  return T;
}

// BF phase B: a tile's weight gradient act^T . dz over the batch rows, 16 rows per
// v_mfma_f32_16x16x16_bf16 (lane (c, g) takes rows 16 q + 4 g + j of its activation column and
// dz column; swizzled columns as phase A stored them; rows past the batch hold zero dz), two
// accumulator chains.  The fp32 form contracts 4 rows per v_mfma_f32_16x16x4f32.
// NB > 0: the block count is compile-time (TB builds), the loop unrolls and every LDS read
// is issued ahead of the MFMAs; NB = 0: nblk at run time.
template <int NB = 0>
__device__ __forceinline__ f32x4 wgrad_bf16(const float* av, const float* dv, const Tile& T, int nblk, int g) {
  f32x4 part[2] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}};
  constexpr int NBU = NB > 0 ? NB : 1;
#pragma unroll
  for (int q = 0; q < (NB > 0 ? NBU : nblk); ++q) {
    f32x4 x, d;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int r = 16 * q + 4 * g + j;
      const int sw = swz(r);
      x[j] = av[r * T.as + (T.as ? (T.am ^ sw) : 0)];
      d[j] = dv[r * T.ds + (T.dc ^ sw)];
    }
    part[q & 1] = mfma16(pack4(x), pack4(d), part[q & 1]);
  }
  return part[0] + part[1];
}

// Streaming epoch: wait until rows [0, need) are in the ring.  1 = they are, 0 = the stream
// ended before `need`, -1 = nothing arrived within the timeout.  Wave-uniform.
__device__ __forceinline__ int64_t ld_host64(const int64_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ int stream_wait(const MBArgs& a, int64_t need, int64_t& avail) {
  if (avail >= need) return 1;
  const long long t0 = (long long)__builtin_amdgcn_s_memrealtime();
  for (;;) {
    avail = ld_host64(a.sr_avail);   // same address in every lane: a wave-uniform value
    if (avail >= need) return 1;
    const int64_t total = ld_host64(a.sr_total);
    if (total >= 0) {   // the host writes the final avail before the total
      avail = ld_host64(a.sr_avail);
      return avail >= need ? 1 : 0;
    }
    if ((long long)__builtin_amdgcn_s_memrealtime() - t0 > a.sr_timeout) return -1;
    __builtin_amdgcn_s_sleep(2);
  }
}

// LDS-only barrier: the next batch's global prefetch stays in flight across it
// (__syncthreads' release fence would also drain vmcnt).
__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

__device__ __forceinline__ f32x4 mfma4(float a, float b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

// Activation codes: compile-time when PACK >= 0 (a1 | a2<<2 | a3<<4 | a4<<6), else runtime.
constexpr int PACK_REF = ACT_TANH | (ACT_RELU << 2) | (ACT_TANH << 4) | (ACT_RELU << 6);
template <int PACK>
__device__ __forceinline__ int act_code(const MBArgs& a, int l) {
  if constexpr (PACK >= 0) return (PACK >> (2 * l)) & 3;
  else return l == 0 ? a.a1 : l == 1 ? a.a2 : l == 2 ? a.a3 : a.a4;
}

__device__ __forceinline__ void st4(float* p, f32x4 v) { *reinterpret_cast<f32x4*>(p) = v; }
__device__ __forceinline__ f32x4 ld4(const float* p) { return *reinterpret_cast<const f32x4*>(p); }

// Four K-steps of a phase-A contraction: fp32 (four v_mfma_f32_16x16x4f32, K-step s = register s
// of the B tile and fragment row s) or, with BF, ONE v_mfma_f32_16x16x16_bf16 over the same 16
// features: lane (c, g)'s four fragment words W[4g + j][c] (rows j of the fp32 image) and its four
// B registers H^T[4g + j][c] are exactly the bf16 A / B operands of that instruction, so the fp32
// images serve both forms (phase B keeps updating only them).  fp32 accumulation either way.
template <bool BF>
__device__ __forceinline__ f32x4 kstep4(const float* frag, int lane, const f32x4& b, f32x4 acc) {
  if constexpr (BF) {
    const f32x4 a = {frag[lane], frag[64 + lane], frag[128 + lane], frag[192 + lane]};
    return mfma16(pack4(a), pack4(b), acc);
  } else {
#pragma unroll
    for (int s = 0; s < 4; ++s) acc = mfma4(frag[s * 64 + lane], b[s], acc);
    return acc;
  }
}

// one hidden-width layer in registers: Z^T = W^T . H^T + b (4 K-steps over 16 features)
template <bool BF = false>
__device__ __forceinline__ f32x4 layer16(const float* frag, const float* bias, int lane, int g, const f32x4& h) {
  return kstep4<BF>(frag, lane, h, ld4(bias + 4 * g));
}

// Sum over the 4 lanes of a row (l, l^16, l^32, l^48) with the gfx950 row swaps:
// permlane16_swap of two copies leaves {rows 0,0,2,2} in one result and {rows 1,1,3,3} in the
// other, permlane32_swap the same across halves; every lane ends with the same bits.
__device__ __forceinline__ float rowsum4(float v) {
  const unsigned u = __float_as_uint(v);
  const auto r16 = __builtin_amdgcn_permlane16_swap(u, u, false, false);
  const float s = __uint_as_float(r16[0]) + __uint_as_float(r16[1]);
  const unsigned w = __float_as_uint(s);
  const auto r32 = __builtin_amdgcn_permlane32_swap(w, w, false, false);
  return __uint_as_float(r32[0]) + __uint_as_float(r32[1]);
}

// Layer 4's padded tail on the VALU (inputs <= 18: the car-sensor schema).  With NO = KSX - 4
// <= 2 real features past 16, 14 of the 16 outputs of layer 4's second tile are padding, and so
// are three quarters of the backward's K-steps 4 .. 3 + NO.  Outputs 16 + o are a 4-term dot per
// lane over its h3 features (W4[4g + i][16 + o]: one 16-byte read from the backward fragment
// image), then the row's 4 lanes summed; the inputs x[16 + o] are summed over the row's lanes at
// the top of the step (off the chain), so every lane computes the same dz and the backward's two
// K-steps become 8 fmas.  6 of the 36 fp32 MFMAs per row tile go.  Same-box A/B (r04o2/o3,
// profiles/r04 SUMMARY §6): batch 32 (pipelined build) +2 %, batch 100 +0.7 %; doing the same for
// layer 1's inputs 16 + o (2 more MFMAs) measured slower at batch 100 and was dropped.
// SML_MB_TAILV=0 compiles the MFMA forms back in.
#ifndef SML_MB_TAILV
#define SML_MB_TAILV 1
#endif
template <int KSX>
constexpr bool tail_valu() { return SML_MB_TAILV && KSX > 4 && KSX <= 6; }

// Categorical accuracy of row r: argmax of y and x, ties -> lowest feature (1 or 0).  The
// row's 20 first (logical) features come in as five 16-byte reads per array; logical block
// jl sits at physical block jl ^ (swz(r) / 4) of its 16-column half.
template <int KD>
__device__ __forceinline__ float row_correct(const float* y, const float* x, int r, int D) {
  const int sb = swz(r) >> 2;
  const float* yr = y + r * XS;
  const float* xq = x + r * XS;
  f32x4 yb[5], xb[5];
#pragma unroll
  for (int jl = 0; jl < 5; ++jl) {
    const int pj = jl < 4 ? (jl ^ sb) : 4 + sb;
    yb[jl] = ld4(yr + 4 * pj);
    xb[jl] = ld4(xq + 4 * pj);
  }
  float by = yb[0][0], bx = xb[0][0];
  int iy = 0, ix = 0;
#pragma unroll
  for (int f = 1; f < (KD < 20 ? KD : 20); ++f) {   // branch-free selects, increasing f
    const float yv = yb[f >> 2][f & 3], xw = xb[f >> 2][f & 3];
    const bool gy = f < D && yv > by, gx = f < D && xw > bx;
    by = gy ? yv : by;
    iy = gy ? f : iy;
    bx = gx ? xw : bx;
    ix = gx ? f : ix;
  }
  if constexpr (KD > 20) {   // wide inputs: the remaining features one by one
#pragma unroll
    for (int f = 20; f < KD; ++f) {
      const int pf = f ^ swz(r);
      const float yv = yr[pf], xw = xq[pf];
      const bool gy = f < D && yv > by, gx = f < D && xw > bx;
      by = gy ? yv : by;
      iy = gy ? f : iy;
      bx = gx ? xw : bx;
      ix = gx ? f : ix;
    }
  }
  return iy == ix ? 1.f : 0.f;
}

// KD: compiled input width class (<= 18 -> 6 K-steps, 32 -> 8); TB: batch (0 = runtime);
// PACK: activation codes (-1 = runtime); WPE: minimum waves per SIMD the register
// allocation must allow (2 = one workgroup per CU, the latency-optimal single-model
// build; 4 = <= 128 VGPRs, two fleet models per CU); MB: LDS capacity class (rows);
// DPX: compiled with the in-kernel gradient exchange (a runtime-gated exchange in the
// single-replica build cost 0.4-0.5 us per batch-32 step, profiles/r02)
// BF: phase A's forward / activation-gradient contractions on bf16 MFMAs (kstep4), fp32 elsewhere
template <int KD, int TB, int PACK, int WPE = 2, int MB = MB_SMALL, bool DPX = false, bool BF = false>
__global__ __launch_bounds__(NT) __attribute__((amdgpu_waves_per_eu(WPE))) void ae_minibatch_kernel(MBArgs a0) {
  static_assert(TB <= MB, "compiled batch exceeds the LDS capacity class");
  static_assert(KD <= 32, "input width <= 32");
  constexpr int KSX = KD <= 16 ? 4 : 4 + (KD - 16 < 4 ? KD - 16 : 4);   // K-steps over the input features
  using Smem = ::Smem<MB>;
  extern __shared__ __attribute__((aligned(16))) float smem_raw[];
  MBArgs a = a0;   // fleet mode: rebase every per-model pointer on the workgroup's model
  {
    const int mdl = blockIdx.x;
    a.x += mdl * a.xmodel;
    if (a.ragged) {
      const int64_t* rg = a.ragged + 3 * mdl;
      a.x += rg[0] * a.ld;
      a.ring = rg[1];
      a.nsteps = (int)rg[2];
    }
    a.params += mdl * NPARAM;
    a.m += mdl * NPARAM;
    a.v += mdl * NPARAM;
    a.iter += mdl;
    if (a.cursor) a.cursor += mdl;
    if (a.metrics) a.metrics += 4 * mdl;
    if (a.lrs) a.lr = a.lrs[mdl];
    if (mdl) a.prof = nullptr;
  }
  Smem& S = *reinterpret_cast<Smem*>(smem_raw);
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int c = lane & 15, g = lane >> 4;
  const int B = TB ? TB : a.B, D = a.D, n1 = a.n1, n2 = a.n2, n3 = a.n3;
  const int a1 = act_code<PACK>(a, 0), a2 = act_code<PACK>(a, 1), a3 = act_code<PACK>(a, 2), a4 = act_code<PACK>(a, 3);
  const float* sbase = smem_raw;

  // ---- zero the weight fragments (padding entries are never written) ----
  for (int e = t; e < W_END; e += NT) S.w[e] = 0.f;
  __syncthreads();

  // ---- phase-B tiles + their Adam moments (registers for the whole launch) ----
  const bool has_tile = wave < 6;
  const Tile T = make_tile(has_tile ? wave : 0, c, g, S, sbase);
  float mo[4], vo[4], wo[4];   // Adam moments + the parameters themselves (sole writer)
  int fpos[4], bpos[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int p = T.slot(i);
    mo[i] = has_tile ? a.m[p] : 0.f;
    vo[i] = has_tile ? a.v[p] : 0.f;
    wo[i] = has_tile ? a.params[p] : 0.f;
    lds_slots(p, fpos[i], bpos[i], (int)(S.one + 1 - S.w));
    if (has_tile) {
      S.w[fpos[i]] = wo[i];
      S.w[bpos[i]] = wo[i];
    }
  }
  if (t == 0) {
    S.one[0] = 1.f;
    S.abort = 0;
    S.stream_end = 0;
  }
  const bool dp = DPX && a.dp_ranks > 1;
  const int dp_rank = a.dp_rank0 + (int)blockIdx.x;

  // ---- phase-A input operands: lane (c, g) of wave w holds row 16w + c, features f(s, g) ----
  const int row_l = 16 * wave + c;           // this lane's row within the batch
  const bool has_rows = 16 * wave < B;       // wave-uniform
  const bool row_ok = row_l < B;
  float sc[KSX], sh[KSX];
  bool fok[KSX];
#pragma unroll
  for (int s = 0; s < KSX; ++s) {
    const int f = feat(s, g);
    fok[s] = f < D;
    sc[s] = fok[s] ? (a.scale ? a.scale[f] : 1.f) : 0.f;
    sh[s] = (fok[s] && a.scale) ? a.shift[f] : 0.f;
  }
  int64_t cur = a.cursor ? a.cursor[0] : 0;
  auto advance = [&](int64_t c0) { c0 += B; return c0 >= a.ring ? c0 - a.ring : c0; };
  float xr[KSX];
  auto fetch = [&](int64_t c0) {
    // clamped address (always in bounds), masked where the value is used
    const float* rp = a.x + (c0 + (row_ok ? row_l : 0)) * a.ld;
#pragma unroll
    for (int s = 0; s < KSX; ++s) xr[s] = __builtin_nontemporal_load(rp + (fok[s] ? feat(s, g) : 0));
  };
  const bool stream = a.sr_avail != nullptr;
  int64_t avail = 0;   // streaming: rows known to be in the ring (cached; re-polled only when short)
  int first_ok = 1;
  if (stream) {   // ONE decision for the whole workgroup: waves that disagreed near the timeout
                  // would split between the in-loop barrier and the final one and hang
    if (t == 0) {
      int64_t av = 0;
      S.first_ok = stream_wait(a, (int64_t)B, av);
      if (S.first_ok < 0) __hip_atomic_store(a.sr_status, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
    __syncthreads();
    first_ok = S.first_ok;
  }
  if (has_rows && first_ok == 1) fetch(cur);
  int64_t nxt = advance(cur);

  float sq = 0.f, ab = 0.f, corr = 0.f;
  const float two_over_d = 2.0f / (float)D;
  const int64_t it0 = a.iter[0];
  // Adam bias corrections beta^t as running fp64 products (powf per step costs ~350
  // instructions on the critical path; fp64 keeps the product exact to ~1e-16 * t)
  double b1t = pow((double)a.beta1, (double)it0), b2t = pow((double)a.beta2, (double)it0);
  const bool prof = WPE == 2 && a.prof != nullptr && t == 0;   // fleet build: no profiling registers
  unsigned long long pc[11] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
  unsigned long long tp = 0, t_start = 0;
  auto mark = [&](int k) {
    if (prof) {
      const unsigned long long now = __builtin_readcyclecounter();
      pc[k] += now - tp;
      tp = now;
    }
  };
  __syncthreads();
  if (prof) t_start = tp = __builtin_readcyclecounter();

  // Reference activations (tanh / relu / linear: act(0) == 0): padded features stay exactly
  // zero by induction (zero padded weights -> zero activations -> zero padded gradients), so
  // only the batch-row mask is needed; sigmoid (act(0) = 0.5) or runtime codes mask features.
  constexpr bool FMASK = PACK < 0 || ((PACK & 3) == ACT_SIGMOID) || (((PACK >> 2) & 3) == ACT_SIGMOID) ||
                         (((PACK >> 4) & 3) == ACT_SIGMOID) || (((PACK >> 6) & 3) == ACT_SIGMOID);
  const float rowf = row_ok ? 1.f : 0.f;
  const float l1r = row_ok ? a.l1 : 0.f;
  auto fm = [&](bool keep, float v) { return FMASK ? (keep ? v : 0.f) : v; };

  const int64_t cur0 = cur;
  int done = a.nsteps;   // optimizer steps applied (fewer only when a DP exchange gave up)
  // DP: a step whose gradient exchange timed out is rolled back on EVERY wave (some waves'
  // granules may have arrived): these hold the state from before the step's update
  float wp[4] = {0.f, 0.f, 0.f, 0.f}, mp[4] = {0.f, 0.f, 0.f, 0.f}, vp[4] = {0.f, 0.f, 0.f, 0.f};
  float sq0 = 0.f, ab0 = 0.f, corr0 = 0.f;
  if (stream && first_ok != 1) done = 0;
  for (int step = 0; step < a.nsteps && first_ok == 1; ++step) {
    if (DPX) {
      sq0 = sq;
      ab0 = ab;
      corr0 = corr;
    }
    // ================= phase A: forward + activation gradients of this wave's 16 rows =================
    if (has_rows) {
      float xv[8];
#pragma unroll
      for (int s = 0; s < 8; ++s) xv[s] = 0.f;
#pragma unroll
      for (int s = 0; s < KSX; ++s) xv[s] = (row_ok && fok[s]) ? fmaf(xr[s], sc[s], sh[s]) : 0.f;
      float xh[2];   // TV: inputs 16 + o of this lane's row (lane group 0's xv[4 + o]) in all 4 lanes
#pragma unroll
      for (int o = 0; o < 2; ++o) xh[o] = (tail_valu<KSX>() && !BF && 4 + o < KSX) ? rowsum4(xv[4 + o]) : 0.f;
      if (step + 1 < a.nsteps) {   // next step's rows: in flight across phase B
        int more = 1;
        if (stream) {   // the next batch must have landed in the ring (or the stream ends here)
          more = stream_wait(a, (int64_t)(step + 2) * B, avail);
          if (more != 1 && lane == 0) {
            S.stream_end = 1;
            if (more < 0) __hip_atomic_store(a.sr_status, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
          }
        }
        if (more == 1) {
          fetch(nxt);
          cur = nxt;
          nxt = advance(cur);
        }
      }
      // L1: h1^T = act1(W1^T x^T + b1)
      f32x4 z1 = ld4(S.w + BB1 + 4 * g);
#pragma unroll
      for (int s4 = 0; s4 < KSX; s4 += 4) {
        if constexpr (BF) {   // K-steps past KSX: zero inputs against zero padding rows
          z1 = kstep4<BF>(S.w + F1 + s4 * 64, lane, f32x4{xv[s4], xv[s4 + 1], xv[s4 + 2], xv[s4 + 3]}, z1);
        } else {
#pragma unroll
          for (int s = s4; s < (s4 + 4 < KSX ? s4 + 4 : KSX); ++s) z1 = mfma4(S.w[F1 + s * 64 + lane], xv[s], z1);
        }
      }
      f32x4 h1, h2, h3;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float h = fm(4 * g + i < n1, act_fwd(a1, z1[i]));
        h1[i] = h;
        ab = fmaf(fabsf(h), rowf, ab);
      }
      // L2, L3
      const f32x4 z2 = layer16<BF>(S.w + F2, S.w + BB2, lane, g, h1);
#pragma unroll
      for (int i = 0; i < 4; ++i) h2[i] = fm(4 * g + i < n2, act_fwd(a2, z2[i]));
      const f32x4 z3 = layer16<BF>(S.w + F3, S.w + BB3, lane, g, h2);
#pragma unroll
      for (int i = 0; i < 4; ++i) h3[i] = fm(4 * g + i < n3, act_fwd(a3, z3[i]));
      // L4 (two output tiles), MSE, dz4 = act4'(y) * 2 (y - x) / D   (1/B applied in Adam)
      constexpr bool TV = tail_valu<KSX>() && !BF;   // bf16: the tail tile is one more cheap MFMA
      f32x4 y[2], dz4[2], w4h[2];
#pragma unroll
      for (int t4 = 0; t4 < (TV ? 1 : 2); ++t4) {
        f32x4 acc = ld4(S.w + BB4 + 16 * t4 + 4 * g);
        acc = kstep4<BF>(S.w + F4 + 4 * t4 * 64, lane, h3, acc);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int f = 16 * t4 + 4 * g + i;
          const float yy = fm(f < D, act_fwd(a4, acc[i]));
          const float e = row_ok ? yy - xv[4 * t4 + i] : 0.f;   // padded features: 0 - 0
          sq = fmaf(e, e, sq);
          y[t4][i] = yy;
          dz4[t4][i] = act_grad(a4, yy, two_over_d * e);
        }
      }
      float dzh[2];   // TV: dz of outputs 16 + o, the same in all 4 lanes of a row
      if constexpr (TV) {   // outputs 16 .. 15 + NO: lane group 0 holds them, as the MFMA tile did
        y[1] = dz4[1] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int o = 0; o < KSX - 4; ++o) {
          w4h[o] = ld4(S.w + G4 + (4 + o) * 64 + 4 * g);
          float p = h3[0] * w4h[o][0];
#pragma unroll
          for (int i = 1; i < 4; ++i) p = fmaf(h3[i], w4h[o][i], p);
          const float yy = fm(16 + o < D, act_fwd(a4, S.w[BB4 + 16 + o] + rowsum4(p)));
          const float e = row_ok ? yy - xh[o] : 0.f;
          dzh[o] = act_grad(a4, yy, two_over_d * e);
          const bool g0 = g == 0;
          const float em = g0 ? e : 0.f;
          sq = fmaf(em, em, sq);
          y[1][o] = g0 ? yy : 0.f;
          dz4[1][o] = g0 ? dzh[o] : 0.f;
        }
      }
      // backward: dz3 = act3'(h3) * (W4 dz4^T), dz2 = act2'(h2) * (W3 dz3^T),
      //           dz1 = act1'(h1) * (W2 dz2^T + l1 sign(h1))   (Keras L1 activity regulariser)
      f32x4 acc3 = {0.f, 0.f, 0.f, 0.f};
      if constexpr (BF) {
#pragma unroll
        for (int s4 = 0; s4 < (TV ? 4 : KSX); s4 += 4) acc3 = kstep4<BF>(S.w + G4 + s4 * 64, lane, dz4[s4 >> 2], acc3);
      } else {
#pragma unroll
        for (int s = 0; s < (TV ? 4 : KSX); ++s) acc3 = mfma4(S.w[G4 + s * 64 + lane], dz4[s >> 2][s & 3], acc3);
      }
      if constexpr (TV) {
#pragma unroll
        for (int o = 0; o < KSX - 4; ++o)
#pragma unroll
          for (int i = 0; i < 4; ++i) acc3[i] = fmaf(w4h[o][i], dzh[o], acc3[i]);
      }
      f32x4 dz3, dz2, dz1;
#pragma unroll
      for (int i = 0; i < 4; ++i) dz3[i] = fm(4 * g + i < n3, act_grad(a3, h3[i], acc3[i]));
      f32x4 acc2 = {0.f, 0.f, 0.f, 0.f};
      acc2 = kstep4<BF>(S.w + G3, lane, dz3, acc2);
#pragma unroll
      for (int i = 0; i < 4; ++i) dz2[i] = fm(4 * g + i < n2, act_grad(a2, h2[i], acc2[i]));
      f32x4 acc1 = {0.f, 0.f, 0.f, 0.f};
      acc1 = kstep4<BF>(S.w + G2, lane, dz2, acc1);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float h = h1[i];
        const float sgn = h != 0.f ? __builtin_copysignf(1.0f, h) : 0.f;
        dz1[i] = fm(4 * g + i < n1, act_grad(a1, h, fmaf(l1r, sgn, acc1[i])));
      }
      // rows -> LDS [row][feature ^ swz(row)] for the weight-gradient contraction (16-byte stores)
      const int r = row_l;
      const int cw = (4 * g) ^ swz(r);
      st4(S.x + r * XS + cw, f32x4{xv[0], xv[1], xv[2], xv[3]});
      st4(S.x + r * XS + 16 + cw, f32x4{xv[4], xv[5], xv[6], xv[7]});
      st4(S.h1 + r * HS + cw, h1);
      st4(S.h2 + r * HS + cw, h2);
      st4(S.h3 + r * HS + cw, h3);
      st4(S.dz4 + r * XS + cw, dz4[0]);
      st4(S.dz4 + r * XS + 16 + cw, dz4[1]);
      st4(S.dz3 + r * HS + cw, dz3);
      st4(S.dz2 + r * HS + cw, dz2);
      st4(S.dz1 + r * HS + cw, dz1);
      if (a.want_acc) {
        st4(S.y + r * XS + cw, y[0]);
        st4(S.y + r * XS + 16 + cw, y[1]);
      }
    }
    mark(0);
    lds_barrier();
    mark(1);
    // ================= phase B: weight gradients + Adam (waves 0-5) =================
    b1t *= (double)a.beta1;
    b2t *= (double)a.beta2;
    if (has_tile) {
      const float lr_t = a.lr * __builtin_amdgcn_sqrtf((float)(1.0 - b2t)) * __builtin_amdgcn_rcpf((float)(1.0 - b1t));
      const float* av = sbase + T.act;
      const float* dv = sbase + T.dz;
      // row r = 4 s4 + g has swz(r) = 4 ((2 s4 + (g >> 1)) & 3): one column per lane for even
      // s4 (E) and one for odd s4 (O); the bias-row lane reads the constant word unswizzled
      const int X0 = 4 * (g >> 1), X1 = 4 * (2 + (g >> 1));
      const int aE = T.as ? (T.am ^ X0) : 0, aO = T.as ? (T.am ^ X1) : 0;
      const int dE = T.dc ^ X0, dO = T.dc ^ X1;
      f32x4 acc = {0.f, 0.f, 0.f, 0.f};
      if constexpr (BF) {
        acc = wgrad_bf16<(TB + 15) / 16>(av, dv, T, (B + 15) / 16, g);
      } else if constexpr (TB > 0) {
        constexpr int NS = (TB + 3) / 4;
        constexpr int CH = NS >= 4 ? 4 : NS;   // independent MFMA chains, summed at the end
        f32x4 part[CH];
#pragma unroll
        for (int c4 = 0; c4 < CH; ++c4) part[c4] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int s4 = 0; s4 < NS; ++s4) {
          const int r = 4 * s4 + g;   // rows in [B, 4*NS) hold zero gradients
          part[s4 % CH] = mfma4(av[r * T.as + ((s4 & 1) ? aO : aE)], dv[r * T.ds + ((s4 & 1) ? dO : dE)],
                                part[s4 % CH]);
        }
#pragma unroll
        for (int c4 = 0; c4 < CH; ++c4) acc += part[c4];
      } else {
        f32x4 acc2 = {0.f, 0.f, 0.f, 0.f};
        const int ns = (B + 3) / 4;
        int s4 = 0;
        for (; s4 + 1 < ns; s4 += 2) {
          const int r = 4 * s4 + g;   // s4 even, s4 + 1 odd
          acc = mfma4(av[r * T.as + aE], dv[r * T.ds + dE], acc);
          acc2 = mfma4(av[(r + 4) * T.as + aO], dv[(r + 4) * T.ds + dO], acc2);
        }
        if (s4 < ns) {
          const int r = 4 * s4 + g;
          acc = mfma4(av[r * T.as + aE], dv[r * T.ds + dE], acc);
        }
        acc += acc2;
      }
      if (dp) {
        // push this rank's partial tile to every peer, then sum the world's partials in
        // rank order (bit-identical on every rank) -- one xGMI hop, no launch, no RCCL call
        const int64_t itg = it0 + step;
        const uint32_t tag = p2p_tag(itg);
        const int par = (int)(itg & 1);
        for (int r = 0; r < a.dp_ranks; ++r) {
          if (r == dp_rank) continue;
          uint64_t* pb = a.dp_peers[r];
#pragma unroll
          for (int i = 0; i < 4; ++i) p2p_put(pb + p2p_index(par, dp_rank, a.dp_ranks, NPARAM, T.slot(i)), tag, acc[i]);
        }
        const uint64_t* own = a.dp_peers[dp_rank];
        f32x4 sum = {0.f, 0.f, 0.f, 0.f};
        bool failed = false;
        const long long t0 = (long long)__builtin_amdgcn_s_memrealtime();
        for (int r = 0; r < a.dp_ranks; ++r) {
          float v[4] = {acc[0], acc[1], acc[2], acc[3]};
          if (r != dp_rank) {
            bool got[4] = {false, false, false, false};
            for (;;) {
#pragma unroll
              for (int i = 0; i < 4; ++i)
                if (!got[i]) got[i] = p2p_try(own + p2p_index(par, r, a.dp_ranks, NPARAM, T.slot(i)), tag, v[i]);
              if (__all(got[0] && got[1] && got[2] && got[3])) break;   // wave-uniform exit
              __builtin_amdgcn_s_sleep(1);
              if ((long long)__builtin_amdgcn_s_memrealtime() - t0 > a.dp_timeout) {
                failed = true;
                break;
              }
            }
          }
#pragma unroll
          for (int i = 0; i < 4; ++i) sum[i] += v[i];
          if (failed) break;
        }
        acc = sum;
        if (failed && lane == 0) S.abort = 1;
      }
      if (DPX) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          wp[i] = wo[i];
          mp[i] = mo[i];
          vp[i] = vo[i];
        }
      }
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float gr = acc[i] * a.gscale;
        const float mm = a.beta1 * mo[i] + (1.0f - a.beta1) * gr;
        const float vv = a.beta2 * vo[i] + (1.0f - a.beta2) * gr * gr;
        mo[i] = mm;
        vo[i] = vv;
        wo[i] -= lr_t * mm * __builtin_amdgcn_rcpf(__builtin_amdgcn_sqrtf(vv) + a.eps);   // v_sqrt / v_rcp, ~1 ulp
        S.w[fpos[i]] = wo[i];
        S.w[bpos[i]] = wo[i];
      }
    } else if (a.want_acc && t - 6 * 64 < B) {
      // categorical accuracy (waves 6-7, one row per lane)
      corr += row_correct<KD>(S.y, S.x, t - 6 * 64, D);
    }
    mark(2);
    lds_barrier();
    mark(3);
    if (stream) {   // read after the barrier: every wave sees the same decision
      if (t == 0 && (step & 7) == 7)   // rows of steps <= step are no longer needed (back-pressure)
        __hip_atomic_store(a.sr_consumed, (int64_t)(step + 1) * B, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      if (S.stream_end) {
        done = step + 1;
        break;
      }
    }
    if (dp && S.abort) {   // read after the barrier: every wave leaves together
      // roll the failed step back everywhere: its update, metrics and cursor never happened,
      // so the replica stays in the state it had after `step` completed steps (the host
      // raises P2PTimeout and can resync / retry from there)
      if (has_tile) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          wo[i] = wp[i];
          mo[i] = mp[i];
          vo[i] = vp[i];
        }
      }
      sq = sq0;
      ab = ab0;
      corr = corr0;
      done = step;
      break;
    }
  }

  // ---- write back: the whole image (padding slots keep zero gradients), moments, metrics ----
  if (has_tile) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      a.params[T.slot(i)] = wo[i];
      a.m[T.slot(i)] = mo[i];
      a.v[T.slot(i)] = vo[i];
    }
  }
  float vals[3] = {sq, ab, corr};
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    float s = vals[k];
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) s += __shfl_xor(s, off, 64);
    if (lane == 0) S.red[k][wave] = s;
  }
  __syncthreads();
  if (prof) {
    pc[8] = __builtin_readcyclecounter() - t_start;
    for (int k = 0; k < 11; ++k) a.prof[k] += pc[k];
  }
  if (t == 0) {
    if (a.metrics) {
#pragma unroll
      for (int k = 0; k < 3; ++k) {
        float s = 0.f;
#pragma unroll
        for (int w = 0; w < NT / 64; ++w) s += S.red[k][w];
        a.metrics[k] += s;
      }
      a.metrics[3] += (float)B * (float)done;
    }
    a.iter[0] = it0 + done;
    if (a.cursor) a.cursor[0] = done == a.nsteps ? nxt : (cur0 + (int64_t)done * B) % a.ring;
    if (stream) __hip_atomic_store(a.sr_consumed, (int64_t)done * B, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    if (dp && S.abort) __hip_atomic_store(a.dp_status, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

// ------------------------------------------------------------------------------------------
// Pipelined Keras batch-32 build (reference activations, <= 18 inputs (KD = 18: cardata) or
// <= 31 (KD = 32: the creditcard model D = 30 of the BASELINE row), one replica per
// workgroup; resident ring or streaming epoch).  At batch 32 only waves 0-1 own rows, so the other six waves
// own the six parameter tiles and the two barriers per step become LDS stage counters:
//   row waves   forward, then the backward, bumping E_l as soon as layer l's activation and
//               upstream gradient are stored and its backward fragment has been read (E4
//               after dz3, E3 after dz2, E2 after dz1 is computed, E1 once dz1 is stored);
//               the next step starts once every U_l has counted this step's updates.
//   tile waves  wait for E_l, contract act^T . dz over the 32 rows, Adam, write the forward /
//               backward fragments, bump U_l.
// W4's, W3's and W2's gradients and updates run under the rest of the backward pass; only
// W1's (its gradient is produced last and the next forward needs it first) stays between two
// steps.  Every LDS buffer a row wave writes in step s+1 is written after its U wait, i.e.
// after the tile waves of step s have read it.  Placement under round-robin wave -> SIMD
// assignment: rows on waves 0-1 (SIMDs 0-1); W1's tiles on waves 4-5 (the same SIMDs: they
// run while the row waves wait for them); the tiles that overlap the backward pass on waves
// 2, 3, 6, 7 (SIMDs 2-3).  Wave 6 also takes the accuracy of the 32 rows before it bumps U4.
// LDS operations of one wave complete in order, so a counter bump after a wave's stores (or
// after the reads whose values it has consumed) needs no fence; only the compiler is fenced.
enum { CE1 = 0, CE2, CE3, CE4, CU1, CU2, CU3, CU4 };
// SLEEP: s_sleep argument of the poll loop -- 0 for the row waves (their waits are on the
// critical path), 1 for the tile waves, whose polls would otherwise take issue slots and LDS
// cycles from the row waves sharing their SIMDs
template <int SLEEP = 0>
__device__ __forceinline__ void pcnt_wait(const unsigned* p, unsigned target) {
  while (__hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) < target) __builtin_amdgcn_s_sleep(SLEEP);
  asm volatile("" ::: "memory");
}
__device__ __forceinline__ void pcnt_bump(unsigned* p, int lane) {
  asm volatile("" ::: "memory");
  if (lane == 0) __hip_atomic_fetch_add(p, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
// The row waves' wait at the start of step st (>= 1) for ALL of the previous step's updates
// (U1 >= 2 st, U2, U3 >= st, U4 >= 2 st) in one 16-byte LDS read per poll: W1's update comes
// last, so one round trip replaces four (one before each forward layer).
__device__ __forceinline__ void pcnt_wait_updates(const unsigned* cnt, unsigned st) {
  for (;;) {
    const uint4 u = *reinterpret_cast<const uint4*>(cnt + CU1);   // ds_read_b128 (counters only grow)
    if (u.x >= 2u * st && u.y >= st && u.z >= st && u.w >= 2u * st) break;
    __builtin_amdgcn_s_sleep(0);
    asm volatile("" ::: "memory");   // read again
  }
  asm volatile("" ::: "memory");
}

// wave -> parameter tile (-1: row wave): rows on waves 0-1, W1 on 4-5, W2 2, W3 3, W4 6-7;
// tile -> layer (1-based)
__device__ __forceinline__ int pipe_tile(int wave) { return wave < 2 ? -1 : wave < 4 ? wave : wave < 6 ? wave - 4 : wave - 2; }
__device__ __forceinline__ int tile_layer(int tile) { return tile <= 1 ? 1 : tile <= 3 ? tile : 4; }

// Batch 32 only.  The same scheme at cardata-v3's batch 100 (7 row waves + 6 tile waves in a
// 13-wave workgroup) measured 23.3 vs 27.3 M rows/s for the two-barrier kernel (profiles/r03/s3):
// there every SIMD already carries row waves, and the tile waves' work and polls slow the chain.
template <int PACK, int TB, int KD = 18, bool BF = false>
__global__ __launch_bounds__(NT) __attribute__((amdgpu_waves_per_eu(2))) void ae_minibatch_pipe_kernel(MBArgs a0) {
  static_assert(TB == 32, "pipelined build: two row waves + six tile waves");
  static_assert(KD == 18 || KD == 32, "input width classes of the barrier kernel");
  constexpr int KSX = KD <= 16 ? 4 : 4 + (KD - 16 < 4 ? KD - 16 : 4), NS = TB / 4;   // as ae_minibatch_kernel
  constexpr int NRW = 2, NWV = 8;
  constexpr int MB = MB_SMALL;
  static_assert(((PACK & 3) != ACT_SIGMOID) && (((PACK >> 2) & 3) != ACT_SIGMOID) &&
                (((PACK >> 4) & 3) != ACT_SIGMOID) && (((PACK >> 6) & 3) != ACT_SIGMOID),
                "act(0) == 0 keeps padded features zero (no masks in this build)");
  using Smem = ::Smem<MB>;
  extern __shared__ __attribute__((aligned(16))) float smem_raw[];
  MBArgs a = a0;
  {
    const int mdl = blockIdx.x;
    a.x += mdl * a.xmodel;
    if (a.ragged) {
      const int64_t* rg = a.ragged + 3 * mdl;
      a.x += rg[0] * a.ld;
      a.ring = rg[1];
      a.nsteps = (int)rg[2];
    }
    a.params += mdl * NPARAM;
    a.m += mdl * NPARAM;
    a.v += mdl * NPARAM;
    a.iter += mdl;
    if (a.cursor) a.cursor += mdl;
    if (a.metrics) a.metrics += 4 * mdl;
    if (a.lrs) a.lr = a.lrs[mdl];
  }
  Smem& S = *reinterpret_cast<Smem*>(smem_raw);
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int c = lane & 15, g = lane >> 4;
  constexpr int B = TB;
  const int D = a.D;
  constexpr int a1 = PACK & 3, a2 = (PACK >> 2) & 3, a3 = (PACK >> 4) & 3, a4 = (PACK >> 6) & 3;
  const float* sbase = smem_raw;

  for (int e = t; e < W_END; e += 64 * NWV) S.w[e] = 0.f;
  if (t < 8) S.cnt[t] = 0u;
  __syncthreads();

  const int tile = pipe_tile(wave);
  const bool has_tile = tile >= 0;
  const Tile T = make_tile(has_tile ? tile : 0, c, g, S, sbase);
  float mo[4], vo[4], wo[4];
  int fpos[4], bpos[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int p = T.slot(i);
    mo[i] = has_tile ? a.m[p] : 0.f;
    vo[i] = has_tile ? a.v[p] : 0.f;
    wo[i] = has_tile ? a.params[p] : 0.f;
    lds_slots(p, fpos[i], bpos[i], (int)(S.one + 1 - S.w));
    if (has_tile) {
      S.w[fpos[i]] = wo[i];
      S.w[bpos[i]] = wo[i];
    }
  }
  if (t == 0) S.one[0] = 1.f;

  const bool has_rows = wave < NRW;
  const int row_l = 16 * wave + c;
  const bool row_ok = row_l < B;   // (always, at batch 32)
  const float rowf = row_ok ? 1.f : 0.f, l1r = row_ok ? a.l1 : 0.f;
  float sc[KSX], sh[KSX];
  bool fok[KSX];
#pragma unroll
  for (int s = 0; s < KSX; ++s) {
    const int f = feat(s, g);
    fok[s] = f < D;
    sc[s] = fok[s] ? (a.scale ? a.scale[f] : 1.f) : 0.f;
    sh[s] = (fok[s] && a.scale) ? a.shift[f] : 0.f;
  }
  int64_t cur = a.cursor ? a.cursor[0] : 0;
  auto advance = [&](int64_t c0) { c0 += B; return c0 >= a.ring ? c0 - a.ring : c0; };
  float xr[KSX];
  auto fetch = [&](int64_t c0) {
    const float* rp = a.x + (c0 + (row_ok ? row_l : 0)) * a.ld;
#pragma unroll
    for (int s = 0; s < KSX; ++s) xr[s] = __builtin_nontemporal_load(rp + (fok[s] ? feat(s, g) : 0));
  };
  // Streaming epoch (see MBArgs): thread 0 decides whether the first batch arrived; each row
  // wave then polls for the batch after next at the start of a step, and a wave that finds the
  // stream over writes this step's index to stream_last before its E bumps of the step, so
  // every wave reads it after the counter waits that follow those bumps (LDS operations are
  // performed in one order per CU, each wave's in program order).
  const bool stream = a.sr_avail != nullptr;
  int64_t avail = 0;
  if (t == 0) {
    S.stream_last = 0x7fffffff;
    S.first_ok = stream ? stream_wait(a, (int64_t)B, avail) : 1;
    if (S.first_ok < 0) __hip_atomic_store(a.sr_status, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
  __syncthreads();
  const int nsteps = S.first_ok == 1 ? a.nsteps : 0;
  if (has_rows && nsteps) fetch(cur);
  int64_t nxt = advance(cur);
  const int64_t cur0 = cur;
  int done = nsteps;

  float sq = 0.f, ab = 0.f, corr = 0.f;
  const float two_over_d = 2.0f / (float)D;
  const int64_t it0 = a.iter[0];
  __syncthreads();

  if (has_rows) {
    for (int step = 0; step < nsteps; ++step) {
      const unsigned st = (unsigned)step;
      // Every tile of the previous step is updated (and its LDS reads, incl. the accuracy wave's,
      // are done), so all of this step's stores are safe too.  A resident ring waits after
      // issuing the next rows' loads; a stream must first learn whether this step exists.
      if (stream && step) pcnt_wait_updates(S.cnt, st);
      if (stream) {
        if (S.stream_last < step) {   // another row wave found the stream over last step
          done = step;
          break;
        }
        if (wave == 0 && lane == 0 && step && (step & 7) == 0)   // rows of steps < step are in registers
          __hip_atomic_store(a.sr_consumed, (int64_t)step * B, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      }
      float xv[8];
#pragma unroll
      for (int s = 0; s < 8; ++s) xv[s] = 0.f;
#pragma unroll
      for (int s = 0; s < KSX; ++s) xv[s] = (row_ok && fok[s]) ? fmaf(xr[s], sc[s], sh[s]) : 0.f;
      float xh[2];
#pragma unroll
      for (int o = 0; o < 2; ++o) xh[o] = (tail_valu<KSX>() && !BF && 4 + o < KSX) ? rowsum4(xv[4 + o]) : 0.f;
      if (step + 1 < nsteps) {   // next step's rows: in flight across this step
        int more = 1;
        if (stream) {
          more = stream_wait(a, (int64_t)(step + 2) * B, avail);
          if (more != 1 && lane == 0) {
            S.stream_last = step;
            if (more < 0) __hip_atomic_store(a.sr_status, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
          }
        }
        if (more == 1) {
          fetch(nxt);
          cur = nxt;
          nxt = advance(cur);
        } else {
          done = step + 1;   // this step is the last
        }
      }
      if (!stream && step) pcnt_wait_updates(S.cnt, st);
      // BF: the backward's fragments read here, off the chain (the E-counter bumps between the
      // backward layers are compiler barriers, so those reads could not move up by themselves;
      // every update of the previous step has landed, and this step's come after the bumps)
      f32x4 pg4[2], pg3, pg2;
      if constexpr (BF) {
        auto frag4 = [&](int base) {
          return f32x4{S.w[base + lane], S.w[base + 64 + lane], S.w[base + 128 + lane], S.w[base + 192 + lane]};
        };
        pg4[0] = frag4(G4);
        pg4[1] = frag4(G4 + 256);
        pg3 = frag4(G3);
        pg2 = frag4(G2);
      }
      f32x4 z1 = ld4(S.w + BB1 + 4 * g);
#pragma unroll
      for (int s4 = 0; s4 < KSX; s4 += 4) {
        if constexpr (BF) {   // K-steps past KSX: zero inputs against zero padding rows
          z1 = kstep4<BF>(S.w + F1 + s4 * 64, lane, f32x4{xv[s4], xv[s4 + 1], xv[s4 + 2], xv[s4 + 3]}, z1);
        } else {
#pragma unroll
          for (int s = s4; s < (s4 + 4 < KSX ? s4 + 4 : KSX); ++s) z1 = mfma4(S.w[F1 + s * 64 + lane], xv[s], z1);
        }
      }
      f32x4 h1, h2, h3;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        h1[i] = act_fwd(a1, z1[i]);
        ab = fmaf(fabsf(h1[i]), rowf, ab);
      }
      const f32x4 z2 = layer16<BF>(S.w + F2, S.w + BB2, lane, g, h1);
#pragma unroll
      for (int i = 0; i < 4; ++i) h2[i] = act_fwd(a2, z2[i]);
      const f32x4 z3 = layer16<BF>(S.w + F3, S.w + BB3, lane, g, h2);
#pragma unroll
      for (int i = 0; i < 4; ++i) h3[i] = act_fwd(a3, z3[i]);
      constexpr bool TV = tail_valu<KSX>() && !BF;   // as ae_minibatch_kernel (bit-identical results)
      f32x4 y[2], dz4[2], w4h[2];
#pragma unroll
      for (int t4 = 0; t4 < (TV ? 1 : 2); ++t4) {
        f32x4 acc = ld4(S.w + BB4 + 16 * t4 + 4 * g);
        acc = kstep4<BF>(S.w + F4 + 4 * t4 * 64, lane, h3, acc);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int f = 16 * t4 + 4 * g + i;
          const float yy = act_fwd(a4, acc[i]);   // padded features: act(0) = 0
          const float e = row_ok ? yy - xv[4 * t4 + i] : 0.f;
          sq = fmaf(e, e, sq);
          y[t4][i] = yy;
          dz4[t4][i] = act_grad(a4, yy, two_over_d * e);
        }
      }
      float dzh[2];
      if constexpr (TV) {
        y[1] = dz4[1] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int o = 0; o < KSX - 4; ++o) {
          w4h[o] = ld4(S.w + G4 + (4 + o) * 64 + 4 * g);
          float p = h3[0] * w4h[o][0];
#pragma unroll
          for (int i = 1; i < 4; ++i) p = fmaf(h3[i], w4h[o][i], p);
          const float yy = act_fwd(a4, S.w[BB4 + 16 + o] + rowsum4(p));
          const float e = row_ok ? yy - xh[o] : 0.f;
          dzh[o] = act_grad(a4, yy, two_over_d * e);
          const bool g0 = g == 0;
          const float em = g0 ? e : 0.f;
          sq = fmaf(em, em, sq);
          y[1][o] = g0 ? yy : 0.f;
          dz4[1][o] = g0 ? dzh[o] : 0.f;
        }
      }
      const int r = row_l;
      const int cw = (4 * g) ^ swz(r);
      st4(S.x + r * XS + cw, f32x4{xv[0], xv[1], xv[2], xv[3]});
      st4(S.x + r * XS + 16 + cw, f32x4{xv[4], xv[5], xv[6], xv[7]});
      st4(S.h3 + r * HS + cw, h3);
      st4(S.dz4 + r * XS + cw, dz4[0]);
      st4(S.dz4 + r * XS + 16 + cw, dz4[1]);
      if (a.want_acc) {
        st4(S.y + r * XS + cw, y[0]);
        st4(S.y + r * XS + 16 + cw, y[1]);
      }
      f32x4 acc3 = {0.f, 0.f, 0.f, 0.f};
      if constexpr (BF) {
#pragma unroll
        for (int s4 = 0; s4 < (TV ? 4 : KSX); s4 += 4) acc3 = mfma16(pack4(pg4[s4 >> 2]), pack4(dz4[s4 >> 2]), acc3);
      } else {
#pragma unroll
        for (int s = 0; s < (TV ? 4 : KSX); ++s) acc3 = mfma4(S.w[G4 + s * 64 + lane], dz4[s >> 2][s & 3], acc3);
      }
      if constexpr (TV) {
#pragma unroll
        for (int o = 0; o < KSX - 4; ++o)
#pragma unroll
          for (int i = 0; i < 4; ++i) acc3[i] = fmaf(w4h[o][i], dzh[o], acc3[i]);
      }
      f32x4 dz3, dz2, dz1;
#pragma unroll
      for (int i = 0; i < 4; ++i) dz3[i] = act_grad(a3, h3[i], acc3[i]);
      pcnt_bump(S.cnt + CE4, lane);   // h3, dz4 (and x, y) stored; G4 read
      st4(S.h2 + r * HS + cw, h2);
      st4(S.dz3 + r * HS + cw, dz3);
      f32x4 acc2 = {0.f, 0.f, 0.f, 0.f};
      if constexpr (BF) acc2 = mfma16(pack4(pg3), pack4(dz3), acc2);
      else acc2 = kstep4<BF>(S.w + G3, lane, dz3, acc2);
#pragma unroll
      for (int i = 0; i < 4; ++i) dz2[i] = act_grad(a2, h2[i], acc2[i]);
      pcnt_bump(S.cnt + CE3, lane);   // h2, dz3 stored; G3 read
      st4(S.h1 + r * HS + cw, h1);
      st4(S.dz2 + r * HS + cw, dz2);
      f32x4 acc1 = {0.f, 0.f, 0.f, 0.f};
      if constexpr (BF) acc1 = mfma16(pack4(pg2), pack4(dz2), acc1);
      else acc1 = kstep4<BF>(S.w + G2, lane, dz2, acc1);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float h = h1[i];
        const float sgn = h != 0.f ? __builtin_copysignf(1.0f, h) : 0.f;
        dz1[i] = act_grad(a1, h, fmaf(l1r, sgn, acc1[i]));
      }
      pcnt_bump(S.cnt + CE2, lane);   // h1, dz2 stored; G2 read
      st4(S.dz1 + r * HS + cw, dz1);
      pcnt_bump(S.cnt + CE1, lane);   // dz1 stored (x was stored with h3)
      if (done == step + 1) break;
    }
  } else {
    const int layer = tile_layer(tile);
    const int ce = CE1 + layer - 1, cu = CU1 + layer - 1;
    double b1t = pow((double)a.beta1, (double)it0), b2t = pow((double)a.beta2, (double)it0);
    const float* av = sbase + T.act;
    const float* dv = sbase + T.dz;
    const int X0 = 4 * (g >> 1), X1 = 4 * (2 + (g >> 1));
    const int aE = T.as ? (T.am ^ X0) : 0, aO = T.as ? (T.am ^ X1) : 0;
    const int dE = T.dc ^ X0, dO = T.dc ^ X1;
    const int acc_row = tile == 4 ? lane : MB_LARGE;   // wave 6: one row per lane
    const bool acc_lane = a.want_acc && acc_row < B;
    for (int step = 0; step < nsteps; ++step) {
      b1t *= (double)a.beta1;
      b2t *= (double)a.beta2;
      const float lr_t = a.lr * __builtin_amdgcn_sqrtf((float)(1.0 - b2t)) * __builtin_amdgcn_rcpf((float)(1.0 - b1t));
      pcnt_wait<1>(S.cnt + ce, (unsigned)NRW * (unsigned)(step + 1));   // every row wave reached layer `layer`
      f32x4 acc = {0.f, 0.f, 0.f, 0.f};   // the barrier kernel's summation order (bit-identical A/B)
      if constexpr (BF) {
        acc = wgrad_bf16<(TB + 15) / 16>(av, dv, T, (B + 15) / 16, g);
      } else {
        f32x4 part[4];
#pragma unroll
        for (int c4 = 0; c4 < 4; ++c4) part[c4] = f32x4{0.f, 0.f, 0.f, 0.f};
        // groups of 4 K-steps, one per accumulator chain
#pragma unroll
        for (int q = 0; q < NS / 4; ++q) {
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const int r = 16 * q + 4 * j + g;
            part[j] = mfma4(av[r * T.as + ((j & 1) ? aO : aE)], dv[r * T.ds + ((j & 1) ? dO : dE)], part[j]);
          }
        }
#pragma unroll
        for (int j = 0; j < NS % 4; ++j) {
          const int r = 16 * (NS / 4) + 4 * j + g;
          part[j] = mfma4(av[r * T.as + ((j & 1) ? aO : aE)], dv[r * T.ds + ((j & 1) ? dO : dE)], part[j]);
        }
#pragma unroll
        for (int c4 = 0; c4 < 4; ++c4) acc += part[c4];
      }
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float gr = acc[i] * a.gscale;
        const float mm = a.beta1 * mo[i] + (1.0f - a.beta1) * gr;
        const float vv = a.beta2 * vo[i] + (1.0f - a.beta2) * gr * gr;
        mo[i] = mm;
        vo[i] = vv;
        wo[i] -= lr_t * mm * __builtin_amdgcn_rcpf(__builtin_amdgcn_sqrtf(vv) + a.eps);
        S.w[fpos[i]] = wo[i];
        S.w[bpos[i]] = wo[i];
      }
      if (acc_lane) corr += row_correct<KD>(S.y, S.x, acc_row, D);
      pcnt_bump(S.cnt + cu, lane);
      if (stream && S.stream_last <= step) break;   // read after this step's E wait: final
    }
  }

  __syncthreads();
  if (has_tile) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      a.params[T.slot(i)] = wo[i];
      a.m[T.slot(i)] = mo[i];
      a.v[T.slot(i)] = vo[i];
    }
  }
  float vals[3] = {sq, ab, corr};
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    float s = vals[k];
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) s += __shfl_xor(s, off, 64);
    if (lane == 0) S.red[k][wave] = s;
  }
  __syncthreads();
  if (t == 0) {
    if (a.metrics) {
#pragma unroll
      for (int k = 0; k < 3; ++k) {
        float s = 0.f;
#pragma unroll
        for (int w = 0; w < NWV; ++w) s += S.red[k][w];
        a.metrics[k] += s;
      }
      a.metrics[3] += (float)B * (float)done;
    }
    a.iter[0] = it0 + done;
    if (a.cursor) a.cursor[0] = done == a.nsteps ? nxt : (cur0 + (int64_t)done * B) % a.ring;
    if (stream) __hip_atomic_store(a.sr_consumed, (int64_t)done * B, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

}  // namespace

namespace sml {

int ae_minibatch_max_batch() { return MAXB; }

hipError_t ae_minibatch_launch(const float* x, int64_t ld, int64_t ring, int64_t* cursor, const float* scale,
                               const float* shift, float* params, float* m, float* v, int64_t* iter, float* metrics,
                               int B, int nsteps, const int* dims, const int* acts, float l1, float lr, float beta1,
                               float beta2, float eps, float gscale, int want_acc, unsigned long long* prof,
                               int nmodels, int64_t xmodel, const float* lrs, const int64_t* ragged,
                               uint64_t* const* dp_peers, int dp_ranks, int dp_rank0, int* dp_status,
                               long long dp_timeout, hipStream_t stream, const MBStream* sr, int precision) {
  // ragged: per-model ring / steps were validated on the host (torch_bind.cpp)
  if (sr && (nmodels != 1 || ragged || dp_ranks > 1 || !sr->avail || !sr->total || !sr->consumed || !sr->status))
    return hipErrorInvalidValue;   // streaming: one model, one replica
  if (B < 1 || B > MAXB || nsteps < 1 || (!ragged && (ring < B || ring % B))) return hipErrorInvalidValue;
  if (dims[0] > 31 || nmodels < 1 || nmodels > (1 << 20) || xmodel < 0) return hipErrorInvalidValue;
  if (dp_ranks > 1 && (!dp_peers || !dp_status || dp_rank0 < 0 || dp_rank0 + nmodels > dp_ranks))
    return hipErrorInvalidValue;
  MBArgs a{x, ld, ring, cursor, scale, shift, params, m, v, iter, metrics, B, nsteps, dims[0], dims[1], dims[2],
           dims[3], acts[0], acts[1], acts[2], acts[3], l1, lr, beta1, beta2, eps, gscale, want_acc, prof,
           xmodel, lrs, ragged, dp_peers, dp_ranks, dp_rank0, dp_status, dp_timeout,
           sr ? sr->avail : nullptr, sr ? sr->total : nullptr, sr ? sr->consumed : nullptr,
           sr ? sr->status : nullptr, sr ? sr->timeout_ticks : 0};
  const bool ref = acts[0] == ACT_TANH && acts[1] == ACT_RELU && acts[2] == ACT_TANH && acts[3] == ACT_RELU;
  // precision 1 (the model's compile(minibatch_precision="bf16")), or -1 with SML_MB_BF16=1 (read per
  // launch, a process-wide default): phase A's contractions on bf16 MFMAs (kstep4) for the
  // reference-activation single-replica builds; fp32 (the Keras-exact path) otherwise
  const char* bfe = precision < 0 ? getenv("SML_MB_BF16") : nullptr;
  const bool bf = (precision == 1 || (bfe && bfe[0] == '1')) && ref && dp_ranks <= 1;
  void (*k)(MBArgs) = nullptr;
  size_t lds = 0;
  auto pick = [&](auto dpx) {
    constexpr bool X = decltype(dpx)::value;
    if (B <= MB_SMALL) {
      lds = sizeof(Smem<MB_SMALL>);
      k = ae_minibatch_kernel<32, 0, -1, 2, MB_SMALL, X>;   // any shape / activations
      if (ref && dims[0] <= 18)
        k = B == 32 ? ae_minibatch_kernel<18, 32, PACK_REF, 2, MB_SMALL, X> : ae_minibatch_kernel<18, 0, PACK_REF, 2, MB_SMALL, X>;
      else if (ref)
        k = B == 32 ? ae_minibatch_kernel<32, 32, PACK_REF, 2, MB_SMALL, X> : ae_minibatch_kernel<32, 0, PACK_REF, 2, MB_SMALL, X>;
      if constexpr (!X) {
        if (bf) k = dims[0] <= 18 ? (B == 32 ? ae_minibatch_kernel<18, 32, PACK_REF, 2, MB_SMALL, false, true>
                                             : ae_minibatch_kernel<18, 0, PACK_REF, 2, MB_SMALL, false, true>)
                                  : (B == 32 ? ae_minibatch_kernel<32, 32, PACK_REF, 2, MB_SMALL, false, true>
                                             : ae_minibatch_kernel<32, 0, PACK_REF, 2, MB_SMALL, false, true>);
      }
      // (a 128-VGPR two-models-per-CU build measured no faster for fleets beyond the CU count:
      // 3.92 vs 3.96 G rows/s at 1024 / 256 models, profiles/r02)
    } else {
      // cardata-v3's fit(batch_size=100) and anything up to 128 rows: one workgroup per CU
      lds = sizeof(Smem<MB_LARGE>);
      k = ae_minibatch_kernel<32, 0, -1, 2, MB_LARGE, X>;
      if (ref && dims[0] <= 18)
        k = B == 100 ? ae_minibatch_kernel<18, 100, PACK_REF, 2, MB_LARGE, X>
                     : ae_minibatch_kernel<18, 0, PACK_REF, 2, MB_LARGE, X>;
      else if (ref) k = ae_minibatch_kernel<32, 0, PACK_REF, 2, MB_LARGE, X>;
      if constexpr (!X) {
        if (bf) k = dims[0] <= 18 ? (B == 100 ? ae_minibatch_kernel<18, 100, PACK_REF, 2, MB_LARGE, false, true>
                                              : ae_minibatch_kernel<18, 0, PACK_REF, 2, MB_LARGE, false, true>)
                                  : ae_minibatch_kernel<32, 0, PACK_REF, 2, MB_LARGE, false, true>;
      }
    }
  };
  if (dp_ranks > 1) pick(std::true_type{});
  else pick(std::false_type{});
  // Keras batch 32, reference stack, one replica per workgroup (alone, fleet or streaming):
  // the pipelined build (SML_MB_PIPE=0 selects the two-barrier kernel, for A/B runs; read per
  // launch).  Same box: 15.5 -> 16.3 M rows/s alone, 3.93 -> 5.73 G rows/s for 1024 models.
  const char* pe = getenv("SML_MB_PIPE");
  if (B == 32 && ref && dp_ranks <= 1 && !prof && !(pe && pe[0] == '0')) {
    if (bf) k = dims[0] <= 18 ? ae_minibatch_pipe_kernel<PACK_REF, 32, 18, true> : ae_minibatch_pipe_kernel<PACK_REF, 32, 32, true>;
    else k = dims[0] <= 18 ? ae_minibatch_pipe_kernel<PACK_REF, 32, 18> : ae_minibatch_pipe_kernel<PACK_REF, 32, 32>;
    lds = sizeof(Smem<MB_SMALL>);
  }
  if (lds > 65536) {   // > 64 KB of dynamic LDS must be opted into per kernel
    const hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(k),
                                             hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return e;
  }
  hipLaunchKernelGGL(k, dim3(nmodels), dim3(NT), lds, stream, a);
  return hipGetLastError();
}

}  // namespace sml
