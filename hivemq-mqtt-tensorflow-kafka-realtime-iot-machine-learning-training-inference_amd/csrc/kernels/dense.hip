// K1 / K2: tall-skinny dense layers on MFMA (SURVEY.md §2.2 K1 dense_fwd, K2 dense_bwd).
//
// Every dense layer in the reference is "millions of rows x a few dozen
// features": the LSTM input projection [B*T, 18] . [18, 128], the recurrent
// weight gradient h^T . dz over B*T rows, TimeDistributed(Dense(18)) heads, the
// MNIST heads.  Library GEMMs run these shapes at ~140 GB/s (measured,
// profiles/r01_v2) because their tiling wants large N and K.  Here the whole
// weight matrix lives in VGPRs as MFMA A-fragments and each wave64 streams
// 16-row tiles through it, so the kernels are HBM-bound by construction:
//
//   rowgemm (K1 / the dX half of K2):  Y[M, N] = act(X[M, K] . W[K, N] + b)
//       feature-major:  Y^T tile (16 out-features x 16 rows) = W^T . X^T,
//       X^T tile = B operand  (lane c = row, 4 consecutive features per lane:
//       one 16-byte load), result in C layout (lane c = row, 4 consecutive
//       output features: one 16-byte store).
//
//   wgrad (dW half of K2):  dW[K, N] = X[M, K]^T . dY[M, N],  db = colsum(dY)
//       contraction over rows: operands are loaded straight into MFMA layout,
//       accumulated in registers over the block's rows (the block's waves split
//       the output tiles), and written as one fp32 slab per block;
//       slab_sum_kernel reduces the slabs deterministically.
//       db is summed in exact fp32 from the same loaded values.
//       ``shift_T`` > 0 reads X[r - 1] (zero when r % T == 0): the h_{t-1}
//       operand of the LSTM recurrent-weight gradient without materialising it.
//
// Inputs may be fp32 or bf16; math is bf16 MFMA with fp32 accumulation.
// Shapes: K <= 16*KT, N <= 16*NT with KT*NT <= 32 (weights <= 64 VGPRs); larger
// layers (e.g. MNIST 784 x 128) stay on hipBLASLt where it is efficient.
#include <cstdlib>

#include "sml_common.h"
#include "sml_adam.h"
#include "sml_ops.h"

namespace sml {
namespace {

constexpr int kWaves = 4;
constexpr int kThreads = 64 * kWaves;

template <typename T>
__device__ __forceinline__ float ld1(const T* p);
template <>
__device__ __forceinline__ float ld1<float>(const float* p) { return *p; }
template <>
__device__ __forceinline__ float ld1<__bf16>(const __bf16* p) { return (float)*p; }

// 4 consecutive elements [k0, k0+4) of one row, zero beyond K (row already clamped valid)
template <typename T>
__device__ __forceinline__ f32x4 load4(const T* row, int k0, int K, bool vec_ok) {
  f32x4 r;
  if (vec_ok && k0 + 3 < K) {
    if constexpr (sizeof(T) == 4) {
      r = *reinterpret_cast<const f32x4*>(row + k0);
    } else {
      typedef unsigned short u16x4 __attribute__((ext_vector_type(4)));
      const u16x4 h = *reinterpret_cast<const u16x4*>(row + k0);
#pragma unroll
      for (int j = 0; j < 4; ++j) r[j] = bf16_to_f32(h[j]);
    }
  } else {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int k = k0 + j;
      r[j] = k < K ? ld1<T>(row + (k < K ? k : 0)) : 0.0f;
    }
  }
  return r;
}

template <typename T>
__device__ __forceinline__ void store4(T* row, int n0, int N, f32x4 v, bool vec_ok);
template <>
__device__ __forceinline__ void store4<float>(float* row, int n0, int N, f32x4 v, bool vec_ok) {
  if (vec_ok && n0 + 3 < N) {
    *reinterpret_cast<f32x4*>(row + n0) = v;
  } else {
#pragma unroll
    for (int j = 0; j < 4; ++j)
      if (n0 + j < N) row[n0 + j] = v[j];
  }
}
template <>
__device__ __forceinline__ void store4<__bf16>(__bf16* row, int n0, int N, f32x4 v, bool vec_ok) {
  if (vec_ok && n0 + 3 < N) {
    *reinterpret_cast<bf16x4*>(row + n0) = pack4(v);
  } else {
#pragma unroll
    for (int j = 0; j < 4; ++j)
      if (n0 + j < N) row[n0 + j] = (__bf16)v[j];
  }
}

// ---------------------------------------------------------------------------
// rowgemm: Y = act(X . W + b)
// ---------------------------------------------------------------------------
// W is staged once per block through LDS (coalesced global reads, then each lane
// gathers its A fragments from LDS), and the next row tile's X is prefetched
// into registers while the current tile's MFMAs and stores run.
template <int KT, int NT, typename TX, typename TY>
__global__ __launch_bounds__(kThreads) void rowgemm_kernel(const TX* __restrict__ X, int64_t M, int K, int64_t ldx,
                                                            const float* __restrict__ W, int wsk, int wsn,
                                                            const float* __restrict__ bias, int N, int act,
                                                            TY* __restrict__ Y, int64_t ldy) {
  __shared__ float ws[16 * KT][16 * NT];
  const int lane = threadIdx.x & 63, c = lane & 15, g = lane >> 4;
  // W element (k, n) at W[k * wsk + n * wsn]: a row-major [K, N] weight, or (wsk = 1,
  // wsn = K) the transpose of a row-major [N, K] one -- dX = dY . W^T without a copy of W^T
  for (int i = threadIdx.x; i < 16 * KT * 16 * NT; i += kThreads) {
    const int k = i / (16 * NT), n = i % (16 * NT);
    ws[k][n] = (k < K && n < N) ? W[(int64_t)k * wsk + (int64_t)n * wsn] : 0.0f;
  }
  __syncthreads();
  // W^T fragments: A[m = out feature 16nt + c][k = in feature 16kt + 4g + j] = W[k][m]
  bf16x4 wf[NT][KT];
#pragma unroll
  for (int nt = 0; nt < NT; ++nt)
#pragma unroll
    for (int kt = 0; kt < KT; ++kt) {
      f32x4 t;
#pragma unroll
      for (int j = 0; j < 4; ++j) t[j] = ws[16 * kt + 4 * g + j][16 * nt + c];
      wf[nt][kt] = pack4(t);
    }
  f32x4 bv[NT];
#pragma unroll
  for (int nt = 0; nt < NT; ++nt)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int n = 16 * nt + 4 * g + i;
      bv[nt][i] = (bias != nullptr && n < N) ? bias[n] : 0.0f;
    }
  const bool xvec = (ldx % 4 == 0) && ((reinterpret_cast<uintptr_t>(X) & (4 * sizeof(TX) - 1)) == 0);
  const bool yvec = (ldy % 4 == 0) && ((reinterpret_cast<uintptr_t>(Y) & (4 * sizeof(TY) - 1)) == 0);
  const int64_t ntiles = (M + 15) / 16;
  const int64_t wave = (int64_t)blockIdx.x * kWaves + (threadIdx.x >> 6);
  const int64_t nwaves = (int64_t)gridDim.x * kWaves;

  auto fetch = [&](int64_t tile, f32x4* v) {
    const int64_t row = tile * 16 + c;
    const bool rok = row < M;
    const TX* xr = X + (rok ? row : 0) * ldx;
#pragma unroll
    for (int kt = 0; kt < KT; ++kt) {
      v[kt] = load4<TX>(xr, 16 * kt + 4 * g, K, xvec);
      if (!rok) v[kt] = f32x4{0.f, 0.f, 0.f, 0.f};
    }
  };
  f32x4 nxt[KT];
  if (wave < ntiles) fetch(wave, nxt);
  for (int64_t tile = wave; tile < ntiles; tile += nwaves) {
    bf16x4 xf[KT];
#pragma unroll
    for (int kt = 0; kt < KT; ++kt) xf[kt] = pack4(nxt[kt]);
    if (tile + nwaves < ntiles) fetch(tile + nwaves, nxt);     // overlaps the MFMAs / stores below
    const int64_t row = tile * 16 + c;
    const bool rok = row < M;
    TY* yr = Y + (rok ? row : 0) * ldy;
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) {
      f32x4 acc = bv[nt];
#pragma unroll
      for (int kt = 0; kt < KT; ++kt) acc = mfma16(wf[nt][kt], xf[kt], acc);
      if (act != ACT_LINEAR) {
#pragma unroll
        for (int i = 0; i < 4; ++i) acc[i] = act_fwd(act, acc[i]);
      }
      if (rok) store4<TY>(yr, 16 * nt + 4 * g, N, acc, yvec);
    }
  }
}

// ---------------------------------------------------------------------------
// wgrad: slab[block] = [ X^T . dY  (16KT x 16NT, row-major) | colsum(dY) (16NT) ]
// ---------------------------------------------------------------------------
// Operands are loaded directly in MFMA layout -- lane (c, g) reads element
// column c of rows 4g..4g+3 (the 16 lanes of a row group read 64 contiguous
// bytes of each row) -- so no LDS transpose sits between the global loads and
// the MFMAs, and the next tile's loads are issued before the current tile's
// MFMAs (register double buffer).
template <int KT, int NT, typename TX, typename TY>
__global__ __launch_bounds__(kThreads) void wgrad_kernel(const TX* __restrict__ X, int64_t M, int K, int64_t ldx,
                                                          int shift_T, const TY* __restrict__ DY, int N,
                                                          int64_t ldy, int want_db, float* __restrict__ partials) {
  constexpr int WN = NT < kWaves ? NT : kWaves;   // waves splitting the N tiles
  constexpr int WR = kWaves / WN;                  // waves splitting the rows
  constexpr int NTW = NT / WN;                     // N tiles per wave
  constexpr int LDN = 16 * NT;
  constexpr int S = 16 * KT * LDN + LDN;
  const int lane = threadIdx.x & 63, c = lane & 15, g = lane >> 4;
  const int w = threadIdx.x >> 6;
  const int nw = w % WN, rw = w / WN;

  f32x4 acc[KT][NTW];
  float accb[NTW];   // db in exact fp32: lane (c, g) sums column c over its rows 4g..4g+3
#pragma unroll
  for (int kt = 0; kt < KT; ++kt)
#pragma unroll
    for (int q = 0; q < NTW; ++q) acc[kt][q] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int q = 0; q < NTW; ++q) accb[q] = 0.f;

  const int64_t ntiles = (M + 15) / 16;
  const int64_t first = (int64_t)blockIdx.x * WR + rw;
  const int64_t stride = (int64_t)gridDim.x * WR;
  // lane (c, g): A[m = x feature 16kt + c][k = row 4g + j],  B[k = row 4g + j][n = dy feature 16nt + c]
  auto fetch = [&](int64_t tile, f32x4* vx, f32x4* vy) {
    const int64_t r0 = tile * 16 + 4 * g;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int64_t r = r0 + j;
      bool xok = r < M;
      int64_t xr = r;
      if (shift_T > 0) {
        xok = xok && (r % shift_T) != 0;
        xr = r - 1;
      }
      const TX* xp = X + (xok ? xr : 0) * ldx;
      const TY* yp = DY + (r < M ? r : 0) * ldy;
#pragma unroll
      for (int kt = 0; kt < KT; ++kt) {
        const int col = 16 * kt + c;
        vx[kt][j] = (xok && col < K) ? ld1<TX>(xp + col) : 0.0f;
      }
#pragma unroll
      for (int q = 0; q < NTW; ++q) {
        const int col = 16 * (nw * NTW + q) + c;
        vy[q][j] = (r < M && col < N) ? ld1<TY>(yp + col) : 0.0f;
      }
    }
  };
  f32x4 nx[KT], ny[NTW];
  if (first < ntiles) fetch(first, nx, ny);
  for (int64_t tile = first; tile < ntiles; tile += stride) {
    bf16x4 af[KT], bf[NTW];
    f32x4 cy[NTW];
#pragma unroll
    for (int kt = 0; kt < KT; ++kt) af[kt] = pack4(nx[kt]);
#pragma unroll
    for (int q = 0; q < NTW; ++q) {
      cy[q] = ny[q];
      bf[q] = pack4(ny[q]);
    }
    if (tile + stride < ntiles) fetch(tile + stride, nx, ny);   // in flight during the MFMAs
#pragma unroll
    for (int q = 0; q < NTW; ++q) accb[q] += (cy[q][0] + cy[q][1]) + (cy[q][2] + cy[q][3]);
#pragma unroll
    for (int kt = 0; kt < KT; ++kt)
#pragma unroll
      for (int q = 0; q < NTW; ++q) acc[kt][q] = mfma16(af[kt], bf[q], acc[kt][q]);
  }
  // fold the four row groups g of each column: lanes c, c+16, c+32, c+48
#pragma unroll
  for (int q = 0; q < NTW; ++q) {
    accb[q] += xor16(accb[q], lane);
    accb[q] += xor32(accb[q], lane);
  }

  float* out = partials + (int64_t)blockIdx.x * S;
  if constexpr (WR == 1) {
    // every (kt, nt) fragment has exactly one owner wave: write straight to the slab
#pragma unroll
    for (int kt = 0; kt < KT; ++kt)
#pragma unroll
      for (int q = 0; q < NTW; ++q)
#pragma unroll
        for (int i = 0; i < 4; ++i) out[(16 * kt + 4 * g + i) * LDN + 16 * (nw * NTW + q) + c] = acc[kt][q][i];
    if (g == 0) {
#pragma unroll
      for (int q = 0; q < NTW; ++q) out[16 * KT * LDN + 16 * (nw * NTW + q) + c] = want_db ? accb[q] : 0.0f;
    }
  } else {
    // WR row phases share fragments: add them in fixed wave order through LDS
    __shared__ float slab[S];
    for (int p = 0; p < WR; ++p) {
      if (rw == p) {
#pragma unroll
        for (int kt = 0; kt < KT; ++kt)
#pragma unroll
          for (int q = 0; q < NTW; ++q)
#pragma unroll
            for (int i = 0; i < 4; ++i) {
              float& d = slab[(16 * kt + 4 * g + i) * LDN + 16 * (nw * NTW + q) + c];
              d = (p == 0 ? 0.0f : d) + acc[kt][q][i];
            }
        if (g == 0) {
#pragma unroll
          for (int q = 0; q < NTW; ++q) {
            float& d = slab[16 * KT * LDN + 16 * (nw * NTW + q) + c];
            d = (p == 0 ? 0.0f : d) + (want_db ? accb[q] : 0.0f);
          }
        }
      }
      __syncthreads();
    }
    for (int i = threadIdx.x; i < S; i += kThreads) out[i] = slab[i];
  }
}

// ---------------------------------------------------------------------------
// deterministic parallel slab reduction: out[y][s] = sum_{g in chunk y} in[g][s]
// ---------------------------------------------------------------------------
// 256 threads = 4 slab groups x 64 float4 column quads; each thread sums up to
// kSlabChunk / 4 slabs with independent 16-byte loads, the 4 groups combine in
// LDS in fixed order.  Applied level by level until one slab remains.
constexpr int kSlabChunk = 32;

// MAP (final level only): element s goes to out[map[s]] (map[s] < 0: dropped) -- the
// slab layout scattered straight into a flat gradient buffer (transposes included)
template <bool MAP = false>
__global__ __launch_bounds__(256) void slab_sum_kernel(const float* __restrict__ in, int G, int S,
                                                       float* __restrict__ out, const int* __restrict__ map = nullptr) {
  __shared__ f32x4 red[4][64];
  const int q = threadIdx.x & 63, grp = threadIdx.x >> 6;
  const int quad = blockIdx.x * 64 + q;
  const int g0 = blockIdx.y * kSlabChunk;
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  if (quad * 4 < S) {
    f32x4 v[kSlabChunk / 4];
#pragma unroll
    for (int u = 0; u < kSlabChunk / 4; ++u) {
      const int gi = g0 + grp + 4 * u;
      v[u] = gi < G ? *reinterpret_cast<const f32x4*>(in + (int64_t)gi * S + quad * 4) : f32x4{0.f, 0.f, 0.f, 0.f};
    }
#pragma unroll
    for (int u = 0; u < kSlabChunk / 4; ++u) acc += v[u];
  }
  red[grp][q] = acc;
  __syncthreads();
  if (grp == 0 && quad * 4 < S) {
    const f32x4 t = red[0][q] + red[1][q] + red[2][q] + red[3][q];
    if constexpr (MAP) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int d = map[quad * 4 + j];
        if (d >= 0) out[d] = t[j];
      }
    } else {
      *reinterpret_cast<f32x4*>(out + (int64_t)blockIdx.y * S + quad * 4) = t;
    }
  }
}

// ---------------------------------------------------------------------------
// dispatch over (KT, NT) and dtypes
// ---------------------------------------------------------------------------
template <typename F>
bool dispatch_kn(int KT, int NT, F&& f) {
#define SML_KN(a, b)                                   \
  if (KT == a && NT == b) {                            \
    f(std::integral_constant<int, a>{}, std::integral_constant<int, b>{}); \
    return true;                                       \
  }
  SML_KN(1, 1) SML_KN(1, 2) SML_KN(1, 4) SML_KN(1, 8) SML_KN(1, 16)
  SML_KN(2, 1) SML_KN(2, 2) SML_KN(2, 4) SML_KN(2, 8) SML_KN(2, 16)
  SML_KN(4, 1) SML_KN(4, 2) SML_KN(4, 4) SML_KN(4, 8)
  SML_KN(8, 1) SML_KN(8, 2) SML_KN(8, 4)
#undef SML_KN
  return false;
}

int round_tiles(int d) {
  const int t = (d + 15) / 16;
  if (t <= 1) return 1;
  if (t <= 2) return 2;
  if (t <= 4) return 4;
  if (t <= 8) return 8;
  return 16;
}

int grid_for(int64_t M, int max_blocks) {
  const int64_t tiles = (M + 15) / 16;
  int64_t b = (tiles + kWaves - 1) / kWaves;
  if (b > max_blocks) b = max_blocks;
  return (int)(b < 1 ? 1 : b);
}

}  // namespace

int dense_tiles(int d) { return round_tiles(d); }

int dense_wgrad_slab(int K, int N) {
  const int KT = round_tiles(K), NT = round_tiles(N);
  return 16 * KT * 16 * NT + 16 * NT;
}

int dense_wgrad_grid(int64_t M, int max_blocks) { return grid_for(M, max_blocks); }

int slab_sum_scratch(int G, int S) {
  int total = 0;
  for (int g = G; g > 1;) {
    const int gy = (g + kSlabChunk - 1) / kSlabChunk;
    if (gy > 1) total += gy * S;
    g = gy;
  }
  return total;
}

// sum G slabs of S floats (S % 4 == 0) into out[S]; intermediate levels go to
// consecutive regions of scratch (slab_sum_scratch(G, S) floats)
// One-pass variant for up to a few thousand slabs: 256 threads = 16 column quads x 16 slab
// groups; group j sums slabs j, j + 16, ... with four independent accumulators, the 16 groups
// combine in LDS in fixed order (deterministic).  ONE launch instead of two or three levels:
// each level of the multi-pass reduction cost ~5 us of launch and ramp at the LSTM's slab
// counts (3 x 2 levels per seq-50 training step, profiles/r04).
// Device body of one column chunk (blk) of one slab set: slab_sum1_kernel, and slab_sum2_kernel (two
// independent slab sets in ONE launch -- the seq-50 step's two LSTM layers, whose sums both wait for
// nothing but Adam: one ~5 us launch floor less per step)
// ADAM (slab_sum2 only): each mapped slot's Adam update right where its gradient is final
// (sml_adam.h; the gradient is still written to out), so the step needs no separate Adam launch
__device__ __forceinline__ void slot_adam(const SlabAdam& ad, int d, float g, float lr_t) {
  float mm, vv, pn;
  adam_update(g, ad.m[d], ad.v[d], ad.params[d], lr_t, ad.b1, ad.b2, ad.eps, ad.gscale, mm, vv, pn);
  ad.m[d] = mm;
  ad.v[d] = vv;
  ad.params[d] = pn;
}

template <bool MAP, bool ADAM = false>
__device__ __forceinline__ void slab_sum1_body(const float* __restrict__ in, int G, int S, float* __restrict__ out,
                                               const int* __restrict__ map, int blk, const SlabAdam& ad = SlabAdam{});

template <bool MAP>
__global__ __launch_bounds__(256) void slab_sum1_kernel(const float* __restrict__ in, int G, int S,
                                                        float* __restrict__ out, const int* __restrict__ map) {
  slab_sum1_body<MAP>(in, G, S, out, map, blockIdx.x);
}

// ADAM: blocks [nb0 + nb1, ...) update the slots no slab map covers (ad.rest: the head's, written
// to out by an earlier launch) -- every parameter gets exactly one update
template <bool ADAM>
__global__ __launch_bounds__(256) void slab_sum2_kernel(const float* __restrict__ in0, int G0, int S0,
                                                        const int* __restrict__ map0, const float* __restrict__ in1,
                                                        int G1, int S1, const int* __restrict__ map1, int nb0, int nb1,
                                                        float* __restrict__ out, SlabAdam ad) {
  const int bx = blockIdx.x;   // block-uniform branches
  if (bx < nb0) {
    slab_sum1_body<true, ADAM>(in0, G0, S0, out, map0, bx, ad);
  } else if (bx < nb0 + nb1) {
    slab_sum1_body<true, ADAM>(in1, G1, S1, out, map1, bx - nb0, ad);
  } else if constexpr (ADAM) {
    const int i = (bx - nb0 - nb1) * 256 + threadIdx.x;
    if (i < ad.nrest) {
      const int d = ad.rest[i];
      slot_adam(ad, d, out[d], adam_lr_t(ad.lr, ad.b1, ad.b2, (float)ad.iter[0]));
    }
  }
}

template <bool MAP, bool ADAM>
__device__ __forceinline__ void slab_sum1_body(const float* __restrict__ in, int G, int S, float* __restrict__ out,
                                               const int* __restrict__ map, int blk, const SlabAdam& ad) {
  __shared__ f32x4 red[16][16];
  float tstep = 0.f;
  if constexpr (ADAM) tstep = (float)ad.iter[0];   // issued before the slab loads
  // the slab map's 4 entries of this thread's quad, loaded before the slab loads too (after the sum
  // they were one more dependent round trip: map, then the scatter / the Adam operand gathers)
  int dm[4] = {-1, -1, -1, -1};
  if constexpr (MAP) {
    if ((threadIdx.x >> 4) == 0 && (blk * 16 + (threadIdx.x & 15)) * 4 < S) {
      const int4 mv = *reinterpret_cast<const int4*>(map + (blk * 16 + (threadIdx.x & 15)) * 4);
      dm[0] = mv.x; dm[1] = mv.y; dm[2] = mv.z; dm[3] = mv.w;
    }
  }
  const int qi = threadIdx.x & 15, grp = threadIdx.x >> 4;
  const int quad = blk * 16 + qi;
  f32x4 acc[4] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}};
  if (quad * 4 < S) {
    int g = grp, k = 0;
    for (; g + 48 < G; g += 64, k = 0) {
#pragma unroll
      for (int u = 0; u < 4; ++u) acc[u] += *reinterpret_cast<const f32x4*>(in + (int64_t)(g + 16 * u) * S + quad * 4);
    }
    for (; g < G; g += 16, k = (k + 1) & 3) acc[k] += *reinterpret_cast<const f32x4*>(in + (int64_t)g * S + quad * 4);
  }
  // ADAM: the 12 operand gathers of the quad's slots, all issued at once (clamped index, no branches)
  // before the barrier, so they overlap the other groups' tails and the LDS fold
  float pm[4] = {0.f, 0.f, 0.f, 0.f}, pv[4] = {0.f, 0.f, 0.f, 0.f}, pp[4] = {0.f, 0.f, 0.f, 0.f};
  if constexpr (ADAM) {
    if (grp == 0 && quad * 4 < S) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int dd = dm[j] >= 0 ? dm[j] : 0;
        pm[j] = ad.m[dd];
        pv[j] = ad.v[dd];
        pp[j] = ad.params[dd];
      }
    }
  }
  red[grp][qi] = (acc[0] + acc[1]) + (acc[2] + acc[3]);
  __syncthreads();
  if (grp == 0 && quad * 4 < S) {
    f32x4 t = red[0][qi];
#pragma unroll
    for (int j = 1; j < 16; ++j) t += red[j][qi];
    if constexpr (MAP) {
      const float lr_t = ADAM ? adam_lr_t(ad.lr, ad.b1, ad.b2, tstep) : 0.f;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int d = dm[j];
        if (d >= 0) {
          out[d] = t[j];
          if constexpr (ADAM) {
            float mm, vv, pn;
            adam_update(t[j], pm[j], pv[j], pp[j], lr_t, ad.b1, ad.b2, ad.eps, ad.gscale, mm, vv, pn);
            ad.m[d] = mm;
            ad.v[d] = vv;
            ad.params[d] = pn;
          }
        }
      }
    } else {
      *reinterpret_cast<f32x4*>(out + quad * 4) = t;
    }
  }
}

hipError_t slab_sum2_launch(const float* p0, int G0, int S0, const int* map0, const float* p1, int G1, int S1,
                            const int* map1, float* out, hipStream_t stream, const SlabAdam* adam) {
  if (S0 % 4 != 0 || S1 % 4 != 0 || G0 < 1 || G1 < 1 || !map0 || !map1) return hipErrorInvalidValue;
  const int nb0 = (S0 / 4 + 15) / 16, nb1 = (S1 / 4 + 15) / 16;
  if (adam) {
    if (!adam->params || !adam->m || !adam->v || !adam->iter || adam->nrest < 0 || (adam->nrest && !adam->rest))
      return hipErrorInvalidValue;
    const int nbr = (adam->nrest + 255) / 256;
    hipLaunchKernelGGL(slab_sum2_kernel<true>, dim3(nb0 + nb1 + nbr), dim3(256), 0, stream, p0, G0, S0, map0, p1, G1,
                       S1, map1, nb0, nb1, out, *adam);
  } else {
    hipLaunchKernelGGL(slab_sum2_kernel<false>, dim3(nb0 + nb1), dim3(256), 0, stream, p0, G0, S0, map0, p1, G1, S1,
                       map1, nb0, nb1, out, SlabAdam{});
  }
  return hipGetLastError();
}

hipError_t slab_sum_launch(const float* partials, int G, int S, float* scratch, float* out, hipStream_t stream,
                           const int* map) {
  if (S % 4 != 0 || G < 1) return hipErrorInvalidValue;
  static const bool one_pass = [] {   // SML_SLAB_1P=0: the multi-level reduction (A/B)
    const char* e = std::getenv("SML_SLAB_1P");
    return !(e && e[0] == '0');
  }();
  if (one_pass && G <= 4096) {
    const dim3 grid((S / 4 + 15) / 16);
    if (map) hipLaunchKernelGGL(slab_sum1_kernel<true>, grid, dim3(256), 0, stream, partials, G, S, out, map);
    else hipLaunchKernelGGL(slab_sum1_kernel<false>, grid, dim3(256), 0, stream, partials, G, S, out, nullptr);
    return hipGetLastError();
  }
  const float* src = partials;
  float* buf = scratch;
  int g = G;
  while (true) {
    const int gy = (g + kSlabChunk - 1) / kSlabChunk;
    float* dst = gy == 1 ? out : buf;
    if (gy == 1 && map)
      hipLaunchKernelGGL(slab_sum_kernel<true>, dim3((S / 4 + 63) / 64, 1), dim3(256), 0, stream, src, g, S, dst, map);
    else
      hipLaunchKernelGGL(slab_sum_kernel<false>, dim3((S / 4 + 63) / 64, gy), dim3(256), 0, stream, src, g, S, dst,
                         nullptr);
    if (gy == 1) break;
    src = dst;
    buf = dst + (int64_t)gy * S;
    g = gy;
  }
  return hipGetLastError();
}

// one level: out[gy][S] = sums of chunks of kSlabChunk slabs; returns gy (-1 on bad args)
int slab_sum_level_launch(const float* in, int G, int S, float* out, hipStream_t stream) {
  if (S % 4 != 0 || G < 1) return -1;
  const int gy = (G + kSlabChunk - 1) / kSlabChunk;
  hipLaunchKernelGGL(slab_sum_kernel<false>, dim3((S / 4 + 63) / 64, gy), dim3(256), 0, stream, in, G, S, out, nullptr);
  return gy;
}

bool dense_supported(int K, int N) {
  const int KT = round_tiles(K), NT = round_tiles(N);
  return K <= 16 * KT && N <= 16 * NT && KT * NT <= 32 && KT <= 8 && NT <= 16 && !(KT >= 4 && NT == 16);
}

hipError_t rowgemm_launch(const void* X, int x_bf16, int64_t M, int K, int64_t ldx, const float* W, const float* bias,
                          int N, int act, void* Y, int y_bf16, int64_t ldy, int max_blocks, hipStream_t stream,
                          int w_t) {
  if (M <= 0) return hipSuccess;
  if (!dense_supported(K, N)) return hipErrorInvalidValue;
  const int KT = round_tiles(K), NT = round_tiles(N);
  const int grid = grid_for(M, max_blocks);
  const int wsk = w_t ? 1 : N, wsn = w_t ? K : 1;
  bool ok = dispatch_kn(KT, NT, [&](auto kt, auto nt) {
    constexpr int A = decltype(kt)::value, B = decltype(nt)::value;
    if (x_bf16 && y_bf16)
      hipLaunchKernelGGL((rowgemm_kernel<A, B, __bf16, __bf16>), dim3(grid), dim3(kThreads), 0, stream,
                         (const __bf16*)X, M, K, ldx, W, wsk, wsn, bias, N, act, (__bf16*)Y, ldy);
    else if (x_bf16)
      hipLaunchKernelGGL((rowgemm_kernel<A, B, __bf16, float>), dim3(grid), dim3(kThreads), 0, stream,
                         (const __bf16*)X, M, K, ldx, W, wsk, wsn, bias, N, act, (float*)Y, ldy);
    else if (y_bf16)
      hipLaunchKernelGGL((rowgemm_kernel<A, B, float, __bf16>), dim3(grid), dim3(kThreads), 0, stream,
                         (const float*)X, M, K, ldx, W, wsk, wsn, bias, N, act, (__bf16*)Y, ldy);
    else
      hipLaunchKernelGGL((rowgemm_kernel<A, B, float, float>), dim3(grid), dim3(kThreads), 0, stream,
                         (const float*)X, M, K, ldx, W, wsk, wsn, bias, N, act, (float*)Y, ldy);
  });
  if (!ok) return hipErrorInvalidValue;
  return hipGetLastError();
}

hipError_t wgrad_launch(const void* X, int x_bf16, int64_t M, int K, int64_t ldx, int shift_T, const void* DY,
                        int dy_bf16, int N, int64_t ldy, int want_db, float* partials, int grid, hipStream_t stream) {
  if (!dense_supported(K, N)) return hipErrorInvalidValue;
  const int KT = round_tiles(K), NT = round_tiles(N);
  bool ok = dispatch_kn(KT, NT, [&](auto kt, auto nt) {
    constexpr int A = decltype(kt)::value, B = decltype(nt)::value;
    if (x_bf16 && dy_bf16)
      hipLaunchKernelGGL((wgrad_kernel<A, B, __bf16, __bf16>), dim3(grid), dim3(kThreads), 0, stream,
                         (const __bf16*)X, M, K, ldx, shift_T, (const __bf16*)DY, N, ldy, want_db, partials);
    else if (x_bf16)
      hipLaunchKernelGGL((wgrad_kernel<A, B, __bf16, float>), dim3(grid), dim3(kThreads), 0, stream,
                         (const __bf16*)X, M, K, ldx, shift_T, (const float*)DY, N, ldy, want_db, partials);
    else if (dy_bf16)
      hipLaunchKernelGGL((wgrad_kernel<A, B, float, __bf16>), dim3(grid), dim3(kThreads), 0, stream,
                         (const float*)X, M, K, ldx, shift_T, (const __bf16*)DY, N, ldy, want_db, partials);
    else
      hipLaunchKernelGGL((wgrad_kernel<A, B, float, float>), dim3(grid), dim3(kThreads), 0, stream,
                         (const float*)X, M, K, ldx, shift_T, (const float*)DY, N, ldy, want_db, partials);
  });
  if (!ok) return hipErrorInvalidValue;
  return hipGetLastError();
}

}  // namespace sml
