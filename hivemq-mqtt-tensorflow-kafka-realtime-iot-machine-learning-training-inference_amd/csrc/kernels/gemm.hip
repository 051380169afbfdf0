// General LDS-tiled MFMA GEMM for the shapes the register-resident K1/K2 tiles do not
// cover (dense.hip: K, N <= 128..256): C = act(op(A) . op(B) + bias), any M, N, K.
//
// Who calls it: Dense layers wider than the register tile (MNIST-size 784 x 128 heads,
// user models of other widths; ops/dense.py) and the LSTM projection / weight-gradient
// GEMMs of layers without a fused instance (ops/lstm.py) -- the shapes that used to
// leave the hand-written path for hipBLASLt (VERDICT r04 "vendor fallbacks").
//
// Layout (gfx950, wave64, v_mfma_f32_16x16x32_bf16):
//   * 128 x 128 output tile per 256-thread workgroup, 2 x 2 waves of 64 x 64,
//     BK = 64 per K-step (two 32-deep MFMA chunks), fp32 accumulators (64 per lane).
//   * Each operand is staged through LDS in its GLOBAL orientation, so the global
//     reads are 16-byte vectors along whichever dimension is contiguous and the
//     transposes every backward GEMM needs (X^T . dY, dY . W^T) cost nothing extra:
//       K-contiguous operand  -> image [mn][BK + 8] bf16, fragment = one ds_read_b128;
//       MN-contiguous operand -> image [BK][128 + 16] bf16, fragment = two
//                                ds_read_b64_tr_b16 (the gfx950 transposing LDS read).
//     fp32 operands are converted to bf16 on the way into LDS.
//   * k permutation: inside every 32-deep chunk, hardware k slot 8g + e is logical
//     k 4g + e and slot 8g + 4 + e is logical k 16 + 4g + e (g = lane >> 4).  Both
//     operands use it, so the contraction is unchanged; it makes the transposing
//     reads of lanes 0..31 cover 8 consecutive k rows (bank octets disjoint with the
//     288-byte image row) and the K-contiguous fragment one contiguous 16-byte read.
//   * Operands are swapped in the MFMA (B fragment as the A operand) so each lane's
//     accumulator holds 4 CONSECUTIVE output columns of one row: the epilogue
//     (bias + activation, fp32 or bf16) stores 16 / 8-byte vectors.
//   * Register-staged double-buffered LDS: tile t+1's global loads are issued before
//     tile t's fragment reads and MFMAs and written to the other buffer after them,
//     one barrier per K-step (72 KB LDS -> 2 workgroups per CU).
//   * Split-K for small outputs with a long contraction (weight gradients over
//     millions of rows): grid = tiles x splits, each split writes an fp32 slab and
//     slab_sum_launch (dense.hip) reduces them in fixed order (deterministic).
//   * XCD-aware block order: the bijective remap gives each XCD a contiguous run of
//     tiles (splits of one tile adjacent), so an XCD's L2 holds its A / B panels.
#include "sml_common.h"
#include "sml_ops.h"

namespace sml {
namespace {

constexpr int BM = 128, BN = 128, BK = 64;
constexpr int kT = 256;
constexpr int KC_LD = BK + 8;       // K-contiguous image row: 144 B
constexpr int MN_LD = 128 + 16;     // MN-contiguous image row: 288 B
constexpr int IMG = 128 * KC_LD;    // bf16 elements per operand image (== BK * MN_LD)
static_assert(128 * KC_LD == BK * MN_LD, "both image kinds occupy the same LDS");

typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

// storage column of logical k (a multiple of 4, within the 64-deep step)
__device__ __forceinline__ int kperm(int k) {
  const int r = k & 31;
  return (k & ~31) + 8 * ((r & 15) >> 2) + 4 * (r >> 4);
}

// One operand of the product, element (mn, k) at p[mn * s_mn + k * s_k] where the
// contiguous dimension has stride 1: KC (k contiguous, s_mn = ld) or MN (s_k = ld).
template <bool KC, typename T>
struct Operand {
  static constexpr int V = 16 / sizeof(T);                 // elements per 16-byte vector
  static constexpr int NV = 128 * BK / V / kT;             // vectors per thread per tile
  static constexpr int VPR = KC ? BK / V : 128 / V;        // vectors per image row (along the contiguous dim)

  const T* p;
  int64_t ld;
  int64_t nmn;       // extent of the mn dimension (M or N)
  bool vec;          // ld and base allow 16-byte vector loads

  // (row, col) of vector i of thread `tid` in the tile's global orientation
  __device__ __forceinline__ void coords(int tid, int i, int& row, int& col) const {
    const int idx = tid + kT * i;
    row = idx / VPR;
    col = (idx % VPR) * V;
  }

  __device__ __forceinline__ void load(u32x4* r, int tid, int64_t mn0, int64_t k0, int64_t kend) const {
    const bool full = vec && mn0 + 128 <= nmn && k0 + BK <= kend;
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      int row, col;
      coords(tid, i, row, col);
      // KC: row = mn, col = k.  MN: row = k, col = mn.
      const int64_t mn = KC ? mn0 + row : mn0 + col;
      const int64_t k = KC ? k0 + col : k0 + row;
      const T* src = KC ? p + mn * ld + k : p + k * ld + mn;
      if (full) {
        r[i] = *reinterpret_cast<const u32x4*>(src);
      } else {
        // edge tile: element-wise, zero outside [0, nmn) x [k0, kend)
        unsigned short h[8];
        float f[4];
#pragma unroll
        for (int e = 0; e < V; ++e) {
          const int64_t me = KC ? mn : mn + e, ke = KC ? k + e : k;
          const bool ok = me < nmn && ke < kend;
          const T* q = KC ? p + (ok ? me * ld + ke : 0) : p + (ok ? ke * ld + me : 0);
          if constexpr (sizeof(T) == 4) f[e] = ok ? (float)*q : 0.0f;
          else h[e] = ok ? __builtin_bit_cast(unsigned short, *q) : (unsigned short)0;
        }
        if constexpr (sizeof(T) == 4) {
          r[i] = u32x4{__float_as_uint(f[0]), __float_as_uint(f[1]), __float_as_uint(f[2]), __float_as_uint(f[3])};
        } else {
#pragma unroll
          for (int j = 0; j < 4; ++j) r[i][j] = (unsigned)h[2 * j] | ((unsigned)h[2 * j + 1] << 16);
        }
      }
    }
  }

  // registers -> bf16 image (global orientation; K-contiguous columns in kperm order)
  __device__ __forceinline__ void store(__bf16* img, const u32x4* r, int tid) const {
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      int row, col;
      coords(tid, i, row, col);
      if constexpr (sizeof(T) == 4) {
        const f32x4 v = {__uint_as_float(r[i][0]), __uint_as_float(r[i][1]), __uint_as_float(r[i][2]),
                         __uint_as_float(r[i][3])};
        const bf16x4 b = pack4(v);
        const int off = KC ? row * KC_LD + kperm(col) : row * MN_LD + col;
        *reinterpret_cast<bf16x4*>(img + off) = b;
      } else {
        if constexpr (KC) {
          *reinterpret_cast<u32x2*>(img + row * KC_LD + kperm(col)) = u32x2{r[i][0], r[i][1]};
          *reinterpret_cast<u32x2*>(img + row * KC_LD + kperm(col + 4)) = u32x2{r[i][2], r[i][3]};
        } else {
          *reinterpret_cast<u32x4*>(img + row * MN_LD + col) = r[i];
        }
      }
    }
  }

  // MFMA fragment of the 16-wide mn sub-tile at image column/row `mn`, 32-deep chunk ch:
  // lane (c, g) gets [mn + c][hardware k 8g .. 8g + 7]
  __device__ __forceinline__ s16x8 frag(const __bf16* img, int mn, int ch, int c, int g) const {
    if constexpr (KC) {
      return *reinterpret_cast<const s16x8*>(img + (mn + c) * KC_LD + 32 * ch + 8 * g);
    } else {
      // lane 4q + p of each 16-lane group addresses k row (4g + q), columns 4p .. 4p + 3
      const __bf16* base = img + (32 * ch + 4 * g + (c >> 2)) * MN_LD + mn + 4 * (c & 3);
      const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)base);
      const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(base + 16 * MN_LD));
      return __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
    }
  }
};

__device__ __forceinline__ f32x4 mfma_k32(s16x8 a, s16x8 b, f32x4 c) {
  typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, a), __builtin_bit_cast(bf16x8, b), c, 0,
                                                 0, 0);
}

template <typename TC>
__device__ __forceinline__ void store_c4(TC* dst, f32x4 v, int valid, bool vec) {
  if (vec && valid >= 4) {
    if constexpr (sizeof(TC) == 4) *reinterpret_cast<f32x4*>(dst) = v;
    else *reinterpret_cast<bf16x4*>(dst) = pack4(v);
  } else {
#pragma unroll
    for (int i = 0; i < 4; ++i)
      if (i < valid) dst[i] = (TC)v[i];
  }
}

template <bool AKC, bool BKC, typename TA, typename TB, typename TC>
__global__ __launch_bounds__(kT) void gemm_kernel(const TA* __restrict__ A, int64_t lda, int a_vec,
                                                     const TB* __restrict__ B, int64_t ldb, int b_vec, int64_t M,
                                                     int64_t N, int64_t K, int64_t kchunk, int splits,
                                                     const float* __restrict__ bias, int act, TC* __restrict__ C,
                                                     int64_t ldc, int c_vec, float* __restrict__ partials,
                                                     int64_t Np) {
  __shared__ __attribute__((aligned(16))) __bf16 lds[2][2][IMG];   // [buffer][A | B]
  const int tid = threadIdx.x, lane = tid & 63, c = lane & 15, g = lane >> 4, w = tid >> 6;
  const int wm = (w >> 1) * 64, wn = (w & 1) * 64;

  // bijective XCD remap: blocks that share an XCD (same blockIdx % 8) take a contiguous id run
  const int nwg = gridDim.x, orig = blockIdx.x, xcd = orig & 7, q = nwg >> 3, rr = nwg & 7;
  const int id = (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + (orig >> 3);
  const int split = id % splits, tile = id / splits;
  const int64_t tiles_n = (N + BN - 1) / BN;
  const int64_t m0 = (tile / tiles_n) * BM, n0 = (tile % tiles_n) * BN;
  const int64_t kb = split * kchunk, ke = (kb + kchunk < K) ? kb + kchunk : K;
  const int nk = ke > kb ? (int)((ke - kb + BK - 1) / BK) : 0;

  const Operand<AKC, TA> opa{A, lda, M, a_vec != 0};
  const Operand<BKC, TB> opb{B, ldb, N, b_vec != 0};
  u32x4 ra[Operand<AKC, TA>::NV], rb[Operand<BKC, TB>::NV];

  f32x4 acc[4][4];   // [n sub-tile][m sub-tile]: lane (c, g) holds C[m + c][n + 4g .. 4g + 3]
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  if (nk > 0) {
    opa.load(ra, tid, m0, kb, ke);
    opb.load(rb, tid, n0, kb, ke);
    opa.store(lds[0][0], ra, tid);
    opb.store(lds[0][1], rb, tid);
    __syncthreads();
  }
  for (int t = 0; t < nk; ++t) {
    const int cur = t & 1;
    const bool more = t + 1 < nk;
    if (more) {   // next tile's global loads in flight during this tile's MFMAs
      opa.load(ra, tid, m0, kb + (int64_t)(t + 1) * BK, ke);
      opb.load(rb, tid, n0, kb + (int64_t)(t + 1) * BK, ke);
    }
    const __bf16* ia = lds[cur][0];
    const __bf16* ib = lds[cur][1];
#pragma unroll
    for (int ch = 0; ch < 2; ++ch) {
      s16x8 fa[4], fb[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) fa[i] = opa.frag(ia, wm + 16 * i, ch, c, g);
#pragma unroll
      for (int j = 0; j < 4; ++j) fb[j] = opb.frag(ib, wn + 16 * j, ch, c, g);
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int i = 0; i < 4; ++i) acc[j][i] = mfma_k32(fb[j], fa[i], acc[j][i]);
    }
    if (more) {   // the other buffer was last read in step t - 1, before this step's barrier
      opa.store(lds[cur ^ 1][0], ra, tid);
      opb.store(lds[cur ^ 1][1], rb, tid);
    }
    __syncthreads();
  }

  // epilogue
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int64_t m = m0 + wm + 16 * i + c;
    if (m >= M) continue;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int64_t n = n0 + wn + 16 * j + 4 * g;
      if (partials != nullptr) {
        // split-K slab [M][Np] (Np = N rounded up to 4: columns n .. n+3 all exist)
        if (n < Np) *reinterpret_cast<f32x4*>(partials + (int64_t)split * M * Np + m * Np + n) = acc[j][i];
        continue;
      }
      if (n >= N) continue;
      f32x4 v = acc[j][i];
      const int valid = (int)((N - n) < 4 ? (N - n) : 4);
      if (bias != nullptr) {
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] += e < valid ? bias[n + e] : 0.0f;
      }
      if (act != ACT_LINEAR) {
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = act_fwd(act, v[e]);
      }
      store_c4<TC>(C + m * ldc + n, v, valid, c_vec != 0);
    }
  }
}

template <bool AKC, bool BKC, typename TA, typename TB>
hipError_t launch_c(int c_bf16, dim3 grid, hipStream_t st, const void* A, int64_t lda, int av, const void* B,
                    int64_t ldb, int bv, int64_t M, int64_t N, int64_t K, int64_t kchunk, int splits,
                    const float* bias, int act, void* C, int64_t ldc, int cv, float* partials, int64_t Np) {
  if (c_bf16)
    hipLaunchKernelGGL((gemm_kernel<AKC, BKC, TA, TB, __bf16>), grid, dim3(kT), 0, st, (const TA*)A, lda, av,
                       (const TB*)B, ldb, bv, M, N, K, kchunk, splits, bias, act, (__bf16*)C, ldc, cv, partials, Np);
  else
    hipLaunchKernelGGL((gemm_kernel<AKC, BKC, TA, TB, float>), grid, dim3(kT), 0, st, (const TA*)A, lda, av,
                       (const TB*)B, ldb, bv, M, N, K, kchunk, splits, bias, act, (float*)C, ldc, cv, partials, Np);
  return hipGetLastError();
}

template <bool AKC, bool BKC>
hipError_t launch_ab(int a_bf16, int b_bf16, int c_bf16, dim3 grid, hipStream_t st, const void* A, int64_t lda,
                     int av, const void* B, int64_t ldb, int bv, int64_t M, int64_t N, int64_t K, int64_t kchunk,
                     int splits, const float* bias, int act, void* C, int64_t ldc, int cv, float* partials,
                     int64_t Np) {
#define SML_GEMM_ARGS c_bf16, grid, st, A, lda, av, B, ldb, bv, M, N, K, kchunk, splits, bias, act, C, ldc, cv, partials, Np
  if (a_bf16 && b_bf16) return launch_c<AKC, BKC, __bf16, __bf16>(SML_GEMM_ARGS);
  if (a_bf16) return launch_c<AKC, BKC, __bf16, float>(SML_GEMM_ARGS);
  if (b_bf16) return launch_c<AKC, BKC, float, __bf16>(SML_GEMM_ARGS);
  return launch_c<AKC, BKC, float, float>(SML_GEMM_ARGS);
#undef SML_GEMM_ARGS
}

bool aligned16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; }

}  // namespace

int gemm_auto_splits(int64_t M, int64_t N, int64_t K, int cus) {
  const int64_t tiles = ((M + BM - 1) / BM) * ((N + BN - 1) / BN);
  const int64_t ksteps = (K + BK - 1) / BK;
  const int64_t want = 2LL * cus;   // two resident workgroups per CU
  if (tiles >= want / 2 || ksteps < 8) return 1;
  int64_t s = (want + tiles - 1) / tiles;
  if (s > ksteps / 4) s = ksteps / 4;   // at least 4 K-steps per split
  if (s > 64) s = 64;
  return s < 1 ? 1 : (int)s;
}

int64_t gemm_kchunk(int64_t K, int splits) {
  const int64_t ksteps = (K + BK - 1) / BK;
  return ((ksteps + splits - 1) / splits) * BK;
}

hipError_t gemm_launch(const void* A, int a_bf16, int64_t lda, int a_kc, const void* B, int b_bf16, int64_t ldb,
                       int b_kc, int64_t M, int64_t N, int64_t K, const float* bias, int act, void* C, int c_bf16,
                       int64_t ldc, float* partials, int splits, hipStream_t stream) {
  if (M <= 0 || N <= 0) return hipSuccess;
  if (splits < 1 || (splits > 1 && partials == nullptr) || K < 0) return hipErrorInvalidValue;
  const int64_t kchunk = gemm_kchunk(K, splits);
  const int64_t tiles = ((M + BM - 1) / BM) * ((N + BN - 1) / BN);
  const int64_t nwg = tiles * splits;
  if (nwg > 0x7fffffff) return hipErrorInvalidValue;
  const dim3 grid((unsigned)nwg);
  const int av = (lda % (a_bf16 ? 8 : 4) == 0) && aligned16(A);
  const int bv = (ldb % (b_bf16 ? 8 : 4) == 0) && aligned16(B);
  const int cv = (ldc % 4 == 0) && ((reinterpret_cast<uintptr_t>(C) & (c_bf16 ? 7 : 15)) == 0);
  const int64_t Np = (N + 3) & ~(int64_t)3;
  float* part = splits > 1 ? partials : nullptr;
#define SML_GEMM_ARGS a_bf16, b_bf16, c_bf16, grid, stream, A, lda, av, B, ldb, bv, M, N, K, kchunk, splits, bias, act, C, ldc, cv, part, Np
  if (a_kc && b_kc) return launch_ab<true, true>(SML_GEMM_ARGS);
  if (a_kc) return launch_ab<true, false>(SML_GEMM_ARGS);
  if (b_kc) return launch_ab<false, true>(SML_GEMM_ARGS);
  return launch_ab<false, false>(SML_GEMM_ARGS);
#undef SML_GEMM_ARGS
}

}  // namespace sml
