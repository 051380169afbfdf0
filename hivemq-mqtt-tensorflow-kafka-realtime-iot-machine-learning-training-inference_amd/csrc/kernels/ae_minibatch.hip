// Persistent small-batch autoencoder trainer for gfx950 (MI355X).
//
// The reference trains its dense autoencoder with Keras `fit(batch_size=32)`
// (AUTOENCODER-TensorFlow-IO-Kafka/cardata-v3.py:187-203, the creditcard notebook's
// batch 32): one Adam update per 32 rows.  At that batch size a launch-per-step
// design (ae_fused.hip: train kernel + slab-reduce/Adam kernel) is launch-bound at
// ~10 us per step.  This kernel keeps the whole optimizer loop on the device: ONE
// workgroup runs `nsteps` sequential Keras steps -- normalise, forward, MSE + L1
// activity loss, backward, weight gradients, Adam -- with the parameters, the Adam
// moments and every activation resident on chip (LDS / VGPRs).  Nothing returns to
// HBM between steps except the next batch's rows, which are prefetched into
// registers one step ahead.  All arithmetic is fp32 (bit-for-bit Keras semantics
// are limited only by summation order), so this is also the exact-semantics path.
//
// Layout (per workgroup, 512 threads = 8 waves):
//   weights in LDS, re-strided so every phase reads conflict-free:
//     W1 [32][16] (bias row 31), W2/W3 [16][17] (bias row 15), W4 [16][33] (bias row 15)
//   activations [B][stride] with a constant-1 column at the end (bias gradient =
//   the same dot product as a weight gradient), double-buffered input tiles.
//   Each real parameter (571 for 18-14-7-7-18) is owned by one thread, which keeps
//   its Adam m / v in registers for the whole launch.
// Per step: 8 phases separated by 8 barriers (fwd L1..L4 + loss, bwd L4..L2 with
// argmax accuracy, then gradients + Adam + the next input tile).
// Fleet mode: a grid of M workgroups trains M independent models at once (per-device
// digital-twin models, ensembles, learning-rate sweeps), one per workgroup, each with
// its own parameters, optimizer state, ring cursor and metrics.  A single model
// occupies one CU; M >= 256 fills the chip (~47 KB LDS -> 3 workgroups per CU).
#include "sml_common.h"

using namespace sml;

namespace {

constexpr int NT = 512;   // 8 waves: two per SIMD, so one wave's LDS / VALU latency hides behind the other's
constexpr int MAXB = 48;   // Keras default batch 32 fits; Smem stays under the 64 KB dynamic-LDS default
constexpr int XS = 33;   // input / output row stride (col 32 = 1.0)
constexpr int HS = 17;   // hidden row stride         (col 16 = 1.0)
// image offsets (ae_fused.hip): L1 [32][16] @0, L2 [16][16] @512, L3 @768, L4 [16][32] @1024
constexpr int IMG2 = 512, IMG3 = 768, IMG4 = 1024, NPARAM = 1536;
// LDS weight offsets (floats)
constexpr int LW1 = 0, LW2 = 512, LW3 = LW2 + 16 * HS, LW4 = LW3 + 16 * HS, LW_END = LW4 + 16 * XS;

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
  unsigned long long* prof;   // optional [11]: per-phase cycles summed over steps (wave 0): 8 phases, total,
                              // P8's input stash, P8's gradient MFMAs + Adam (model 0 only)
  // fleet mode: workgroup b trains model b.  params / m / v are [M][NPARAM], iter /
  // cursor [M], metrics [M][4]; model b reads x + b * xmodel (0 = one shared ring).
  int64_t xmodel;
  const float* lrs;     // optional [M] per-model learning rates (hyper-parameter sweeps)
};

struct Smem {   // ~47 KB
  float w[LW_END];
  float x[2][MAXB * XS];
  float h1[MAXB * HS], h2[MAXB * HS], h3[MAXB * HS];
  float y[MAXB * XS];
  float dz4[MAXB * XS], dz3[MAXB * HS], dz2[MAXB * HS], dz1[MAXB * HS];
  float red[3][NT / 64];
};

// image slot -> LDS weight index
__device__ __forceinline__ int lds_of_slot(int s) {
  if (s < IMG2) return LW1 + s;
  if (s < IMG3) { const int k = s - IMG2; return LW2 + (k >> 4) * HS + (k & 15); }
  if (s < IMG4) { const int k = s - IMG3; return LW3 + (k >> 4) * HS + (k & 15); }
  const int k = s - IMG4;
  return LW4 + (k >> 5) * XS + (k & 31);
}

// A 16x16 tile of the padded image whose gradient one wave computes with fp32 MFMAs
// (v_mfma_f32_16x16x4f32: K = 4 batch rows per instruction).  Tiles: 0/1 = L1 rows
// 0-15 / 16-31, 2 = L2, 3 = L3, 4/5 = L4 cols 0-15 / 16-31; wave w < 6 owns tile w.
struct Tile {
  int act, as;      // activation base (float offset into Smem; L1: buffer 0) and row stride
  int acol;         // this lane's activation column (image row m = row0 + c; bias row -> ones column)
  int dz, ds;       // upstream-gradient base + this lane's column, row stride
  int xb;           // L1: activation lives in the current input buffer
  int slot0, sst;   // image slots of C[4g+i][c]: slot0 + i * sst (consecutive image rows)
  int w0, wst;      // their LDS weight indices: w0 + i * wst
  __device__ __forceinline__ int slot(int i) const { return slot0 + i * sst; }
  __device__ __forceinline__ int w(int i) const { return w0 + i * wst; }
};

__device__ __forceinline__ Tile make_tile(int id, int c, int g, const Smem& S, const float* sbase) {
  Tile T;
  int row0 = 0, col0 = 0, img = 0, istride = 16, bias_row = 15;
  if (id <= 1) {
    row0 = 16 * id; img = 0; bias_row = 31;
    T.act = (int)(S.x[0] - sbase); T.as = XS; T.dz = (int)(S.dz1 - sbase); T.ds = HS; T.xb = 1;
  } else if (id == 2) {
    img = IMG2; T.act = (int)(S.h1 - sbase); T.as = HS; T.dz = (int)(S.dz2 - sbase); T.ds = HS; T.xb = 0;
  } else if (id == 3) {
    img = IMG3; T.act = (int)(S.h2 - sbase); T.as = HS; T.dz = (int)(S.dz3 - sbase); T.ds = HS; T.xb = 0;
  } else {
    col0 = 16 * (id - 4); img = IMG4; istride = 32;
    T.act = (int)(S.h3 - sbase); T.as = HS; T.dz = (int)(S.dz4 - sbase); T.ds = XS; T.xb = 0;
  }
  const int m = row0 + c;
  T.acol = m == bias_row ? (id <= 1 ? 32 : 16) : m;
  T.dz += col0 + c;
  T.slot0 = img + (row0 + 4 * g) * istride + col0 + c;
  T.sst = istride;
  T.w0 = lds_of_slot(T.slot0);
  T.wst = id <= 1 ? 16 : id <= 3 ? HS : XS;   // LDS row strides of W1 / W2,W3 / W4
  return T;
}

// LDS-only barrier: the next batch's global prefetch stays in flight across it
// (__syncthreads' release fence would also drain vmcnt).
__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// Fixed-trip dot product (padding columns of activations are zero, so a padded
// trip count is exact and lets every LDS read issue up front).
template <int N>
__device__ __forceinline__ float dotn(const float* act, const float* w, int wstride) {
  float acc0 = 0.f, acc1 = 0.f;   // two chains: half the dependent-FMA latency
#pragma unroll
  for (int i = 0; i < N; i += 2) {
    acc0 = fmaf(act[i], w[i * wstride], acc0);
    if (i + 1 < N) acc1 = fmaf(act[i + 1], w[(i + 1) * wstride], acc1);
  }
  return acc0 + acc1;
}

// Activation codes: compile-time when PACK >= 0 (a1 | a2<<2 | a3<<4 | a4<<6), else runtime.
constexpr int PACK_REF = ACT_TANH | (ACT_RELU << 2) | (ACT_TANH << 4) | (ACT_RELU << 6);
template <int PACK>
__device__ __forceinline__ int act_code(const MBArgs& a, int l) {
  if constexpr (PACK >= 0) return (PACK >> (2 * l)) & 3;
  else return l == 0 ? a.a1 : l == 1 ? a.a2 : l == 2 ? a.a3 : a.a4;
}

// Work items o = t + NT*u, u < N, fully unrolled so every item's LDS reads issue together.
template <int N, class F>
__device__ __forceinline__ void for_items(int t, int limit, F&& f) {
#pragma unroll
  for (int u = 0; u < N; ++u) {
    const int o = t + NT * u;
    if (o < limit) f(o);
  }
}
constexpr int I16 = (MAXB * 16 + NT - 1) / NT;

// KD: trip count over input features (D rounded to a compiled width); TB: batch (0 = runtime);
// PACK: activation codes (-1 = runtime); WPE: minimum waves per SIMD the register
// allocation must allow (2 = one workgroup per CU, the latency-optimal single-model
// build; 4 = <= 128 VGPRs, two fleet models per CU)
template <int KD, int TB, int PACK, int WPE = 2>
__global__ __launch_bounds__(NT) __attribute__((amdgpu_waves_per_eu(WPE))) void ae_minibatch_kernel(MBArgs a0) {
  extern __shared__ float smem_raw[];
  MBArgs a = a0;   // fleet mode: rebase every per-model pointer on the workgroup's model
  {
    const int mdl = blockIdx.x;
    a.x += mdl * a.xmodel;
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
  const int B = TB ? TB : a.B, D = a.D, n1 = a.n1, n2 = a.n2, n3 = a.n3;
  const int a1 = act_code<PACK>(a, 0), a2 = act_code<PACK>(a, 1), a3 = act_code<PACK>(a, 2), a4 = act_code<PACK>(a, 3);
  const float* sbase = smem_raw;
  constexpr int IKD = (MAXB * KD + NT - 1) / NT;
  static_assert(KD == 32 || KD < 32, "KD <= 32");

  // ---- gradient tiles + their Adam moments (registers for the whole launch) ----
  const int c = lane & 15, g = lane >> 4;
  const bool has_tile = wave < 6;
  const Tile T = make_tile(has_tile ? wave : 0, c, g, S, sbase);
  float mo[4], vo[4], wo[4];   // Adam moments + the parameters themselves (sole writer)
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    mo[i] = has_tile ? a.m[T.slot(i)] : 0.f;
    vo[i] = has_tile ? a.v[T.slot(i)] : 0.f;
    wo[i] = has_tile ? a.params[T.slot(i)] : 0.f;
  }

  // ---- weights -> LDS (padding zero), zeroed activations, constant-1 bias columns ----
  for (int s = t; s < NPARAM; s += NT) S.w[lds_of_slot(s)] = a.params[s];
  for (int e = t; e < MAXB * XS; e += NT) {
    const float one = (e % XS) == 32 ? 1.f : 0.f;
    S.x[0][e] = one;
    S.x[1][e] = one;
    S.dz4[e] = 0.f;
  }
  for (int e = t; e < MAXB * HS; e += NT) {
    const float one = (e % HS) == 16 ? 1.f : 0.f;
    S.h1[e] = one; S.h2[e] = one; S.h3[e] = one;
    S.dz1[e] = 0.f; S.dz2[e] = 0.f; S.dz3[e] = 0.f;
  }

  // ---- input tiles: element e = t + NT*u of the MAXB x 32 tile (cols >= D -> 0) ----
  constexpr int XU = MAXB * 32 / NT;   // 3 elements per thread
  static_assert(MAXB * 32 % NT == 0, "input tile must split evenly over the threads");
  float sc[XU], sh[XU];
#pragma unroll
  for (int u = 0; u < XU; ++u) {
    const int f = (t + NT * u) & 31;
    sc[u] = f < D ? (a.scale ? a.scale[f] : 1.f) : 0.f;
    sh[u] = (f < D && a.scale) ? a.shift[f] : 0.f;
  }
  int64_t cur = a.cursor ? a.cursor[0] : 0;
  float xr[XU];
  auto fetch = [&](int64_t c0) {
#pragma unroll
    for (int u = 0; u < XU; ++u) {
      const int e = t + NT * u, r = e >> 5, f = e & 31;
      // clamped address (always in bounds), masked where the value is used
      const int64_t row = c0 + (r < B ? r : 0);
      xr[u] = __builtin_nontemporal_load(a.x + row * a.ld + (f < D ? f : 0));
    }
  };
  auto stash = [&](float* xt) {
#pragma unroll
    for (int u = 0; u < XU; ++u) {
      const int e = t + NT * u, r = e >> 5, f = e & 31;
      if (r < B) xt[r * XS + f] = f < D ? fmaf(xr[u], sc[u], sh[u]) : 0.f;
    }
  };
  auto advance = [&](int64_t c0) { c0 += B; return c0 >= a.ring ? c0 - a.ring : c0; };

  __syncthreads();
  fetch(cur);
  stash(S.x[0]);
  int64_t nxt = advance(cur);
  if (a.nsteps > 1) fetch(nxt);

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

  for (int step = 0; step < a.nsteps; ++step) {
    const float* X = S.x[step & 1];
    // P1: h1 = act1(x W1 + b1)
    for_items<I16>(t, B * 16, [&](int o) {
      const int r = o >> 4, j = o & 15;
      const float z = dotn<KD>(X + r * XS, S.w + LW1 + j, 16) + S.w[LW1 + 31 * 16 + j];
      const float h = j < n1 ? act_fwd(a1, z) : 0.f;
      ab += fabsf(h);
      S.h1[r * HS + j] = h;
    });
    lds_barrier();
    mark(0);
    // P2, P3
    for_items<I16>(t, B * 16, [&](int o) {
      const int r = o >> 4, j = o & 15;
      const float z = dotn<16>(S.h1 + r * HS, S.w + LW2 + j, HS) + S.w[LW2 + 15 * HS + j];
      S.h2[r * HS + j] = j < n2 ? act_fwd(a2, z) : 0.f;
    });
    lds_barrier();
    mark(1);
    for_items<I16>(t, B * 16, [&](int o) {
      const int r = o >> 4, j = o & 15;
      const float z = dotn<16>(S.h2 + r * HS, S.w + LW3 + j, HS) + S.w[LW3 + 15 * HS + j];
      S.h3[r * HS + j] = j < n3 ? act_fwd(a3, z) : 0.f;
    });
    lds_barrier();
    mark(2);
    // P4: y = act4(h3 W4 + b4); MSE; dz4 (sum-scaled, 1/B in gscale).  Items cover the
    // KD real-or-padding columns only; columns >= KD stay at their zero initialisation.
    for_items<IKD>(t, B * KD, [&](int o) {
      const int r = o / KD, j = o - r * KD;
      const float z = dotn<16>(S.h3 + r * HS, S.w + LW4 + j, XS) + S.w[LW4 + 15 * XS + j];
      const float y = j < D ? act_fwd(a4, z) : 0.f;
      const float e = y - X[r * XS + j];
      sq = fmaf(e, e, sq);
      S.y[r * XS + j] = y;
      S.dz4[r * XS + j] = j < D ? act_grad(a4, y, two_over_d * e) : 0.f;
    });
    lds_barrier();
    mark(3);
    // P5: dz3 = act3'(dz4 W4^T)
    for_items<I16>(t, B * 16, [&](int o) {
      const int r = o >> 4, i = o & 15;
      const float d = act_grad(a3, S.h3[r * HS + i], dotn<KD>(S.dz4 + r * XS, S.w + LW4 + i * XS, 1));
      S.dz3[r * HS + i] = i < n3 ? d : 0.f;
    });
    lds_barrier();
    mark(4);
    // P6: dz2 = act2'(dz3 W3^T)
    for_items<I16>(t, B * 16, [&](int o) {
      const int r = o >> 4, i = o & 15;
      const float d = act_grad(a2, S.h2[r * HS + i], dotn<16>(S.dz3 + r * HS, S.w + LW3 + i * HS, 1));
      S.dz2[r * HS + i] = i < n2 ? d : 0.f;
    });
    lds_barrier();
    mark(5);
    // P7: dz1 = act1'(dz2 W2^T + l1 * sign(h1))   (Keras L1 activity regulariser)
    for_items<I16>(t, B * 16, [&](int o) {
      const int r = o >> 4, i = o & 15;
      const float h = S.h1[r * HS + i];
      const float sgn = h != 0.f ? __builtin_copysignf(1.0f, h) : 0.f;
      const float d = act_grad(a1, h, fmaf(a.l1, sgn, dotn<16>(S.dz2 + r * HS, S.w + LW2 + i * HS, 1)));
      S.dz1[r * HS + i] = i < n1 ? d : 0.f;
    });
    lds_barrier();
    mark(6);
    // P8: weight gradients = act^T . dz over the B rows (fp32 MFMA, K = 4 rows per
    // instruction), Keras Adam on the tile in registers (waves 0-5); argmax accuracy
    // (waves 6-7, which own no tile); next input tile to the other buffer; prefetch.
    if (step + 1 < a.nsteps) {   // next tile -> the other buffer (not read this phase)
      stash(S.x[(step + 1) & 1]);
      cur = nxt;
      nxt = advance(cur);
    }
    mark(9);
    b1t *= (double)a.beta1;
    b2t *= (double)a.beta2;
    const float lr_t = a.lr * __builtin_amdgcn_sqrtf((float)(1.0 - b2t)) * __builtin_amdgcn_rcpf((float)(1.0 - b1t));
    if (has_tile) {
      const float* av = sbase + T.act + ((step & 1) && T.xb ? MAXB * XS : 0) + T.acol;
      const float* dv = sbase + T.dz;
      f32x4 acc = {0.f, 0.f, 0.f, 0.f};
      if constexpr (TB > 0) {
        constexpr int CH = TB / 4 >= 4 ? 4 : TB / 4;   // independent MFMA chains, summed at the end
        f32x4 part[CH];
#pragma unroll
        for (int c4 = 0; c4 < CH; ++c4) part[c4] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int s4 = 0; s4 < TB / 4; ++s4) {
          const int r = 4 * s4 + g;
          part[s4 % CH] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[r * T.as], dv[r * T.ds], part[s4 % CH], 0, 0, 0);
        }
#pragma unroll
        for (int c4 = 0; c4 < CH; ++c4) acc += part[c4];
      } else {
        for (int s4 = 0; s4 < (B + 3) / 4; ++s4) {
          const int r = 4 * s4 + g;
          const float x0 = r < B ? av[r * T.as] : 0.f, d0 = r < B ? dv[r * T.ds] : 0.f;
          acc = __builtin_amdgcn_mfma_f32_16x16x4f32(x0, d0, acc, 0, 0, 0);
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
        S.w[T.w(i)] = wo[i];
      }
      mark(10);
    } else if (a.want_acc && t - 6 * 64 < B) {
      const int r = t - 6 * 64;
      int iy = 0, ix = 0;
      float by = S.y[r * XS], bx = X[r * XS];
#pragma unroll
      for (int f = 1; f < KD; ++f) {   // ties -> lowest index (tf.argmax); branch-free selects
        const float yv = S.y[r * XS + f], xv = X[r * XS + f];
        const bool gy = f < D && yv > by, gx = f < D && xv > bx;
        by = gy ? yv : by;
        iy = gy ? f : iy;
        bx = gx ? xv : bx;
        ix = gx ? f : ix;
      }
      corr += iy == ix ? 1.f : 0.f;
    }
    if (step + 2 < a.nsteps) fetch(nxt);
    lds_barrier();
    mark(7);
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
      a.metrics[3] += (float)B * (float)a.nsteps;
    }
    a.iter[0] = it0 + a.nsteps;
    if (a.cursor) a.cursor[0] = nxt;
  }
}

}  // namespace

namespace sml {

int ae_minibatch_max_batch() { return MAXB; }

hipError_t ae_minibatch_launch(const float* x, int64_t ld, int64_t ring, int64_t* cursor, const float* scale,
                               const float* shift, float* params, float* m, float* v, int64_t* iter, float* metrics,
                               int B, int nsteps, const int* dims, const int* acts, float l1, float lr, float beta1,
                               float beta2, float eps, float gscale, int want_acc, unsigned long long* prof,
                               int nmodels, int64_t xmodel, const float* lrs, hipStream_t stream) {
  if (B < 1 || B > MAXB || nsteps < 1 || ring < B || ring % B) return hipErrorInvalidValue;
  if (dims[0] > 31 || nmodels < 1 || nmodels > (1 << 20) || xmodel < 0) return hipErrorInvalidValue;
  MBArgs a{x, ld, ring, cursor, scale, shift, params, m, v, iter, metrics, B, nsteps, dims[0], dims[1], dims[2],
           dims[3], acts[0], acts[1], acts[2], acts[3], l1, lr, beta1, beta2, eps, gscale, want_acc, prof,
           xmodel, lrs};
  const bool ref = acts[0] == ACT_TANH && acts[1] == ACT_RELU && acts[2] == ACT_TANH && acts[3] == ACT_RELU;
  auto k = ae_minibatch_kernel<32, 0, -1>;   // any shape / activations
  if (ref && dims[0] == 18) k = B == 32 ? ae_minibatch_kernel<18, 32, PACK_REF> : ae_minibatch_kernel<18, 0, PACK_REF>;
  else if (ref) k = B == 32 ? ae_minibatch_kernel<32, 32, PACK_REF> : ae_minibatch_kernel<32, 0, PACK_REF>;
  // a fleet larger than one model per CU: the 128-VGPR build puts two models on each CU
  int dev = 0, cus = 256;
  if (hipGetDevice(&dev) == hipSuccess) hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  if (ref && dims[0] == 18 && B == 32 && nmodels > cus) k = ae_minibatch_kernel<18, 32, PACK_REF, 4>;
  hipLaunchKernelGGL(k, dim3(nmodels), dim3(NT), sizeof(Smem), stream, a);
  return hipGetLastError();
}

}  // namespace sml
