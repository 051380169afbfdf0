// K8 ingest transforms: the reference's per-event tf.data graph
//   normalize_fn(...)                      cardata-v3.py:78-168  (per-column affine, 4 zeroed columns)
//   .filter(lambda x, y: y == "false")     cardata-v3.py:212     (train on normal events only)
//   metrics=['accuracy'] -> argmax(x)      cardata-v3.py:203-205 (the data half of the metric)
// on the device, for raw [n, D] fp32 rows that land through the pinned H2D ring.
//
// Every kernel here is a pure HBM stream (a few FLOPs per 4-byte element), so the design
// rule is bytes: each byte of x is read once with 16-byte coalesced loads and every output
// byte written once with 16-byte coalesced stores.  The row granularity (18 floats = 72 B)
// does not match the 16-byte lane granularity, so one wave moves a whole group of rows as a
// flat float4 stream and stages it through LDS; the per-row work (argmax, compaction rank)
// then reads rows out of LDS.
//
//   pack_tiles:  wave = 8 tiles of 16 rows.  float4 stream in, x * scale + shift with a
//                per-position scale table (column = flat index mod D), float4 stream out into
//                the tile-packed layout [16 rows | 16 argmax bytes] (tile = 16 * (4D + 1) B,
//                so every output float4 is aligned), argmax of each row from LDS.
//   row_argmax:  the same wave structure without the float stores: one byte per row.
//   normalize_filter (order-preserving stream compaction, 3 launches):
//      count   -- 16 labels per lane (one 16-byte load), per-block kept count;
//      scan    -- one workgroup turns the counts into exclusive block offsets + the total;
//      scatter -- per 64-row wave group: float4-staged rows in LDS, ballot rank, then the
//                 kept rows written as ONE contiguous coalesced run of floats.
// The previous one-thread-per-row kernels read 72-byte rows with lane strides of 72 B and
// ran at ~0.8 TB/s (profiles/r02/ilp/kernel_stats_final.csv:5); see profiles/r03/.
#include <algorithm>

#include "sml_common.h"

namespace {

constexpr int kThreads = 256;
constexpr int kWaves = kThreads / 64;
constexpr int kTilesPerWave = 8;                 // pack / argmax: 8 x 16 = 128 rows per wave group
constexpr int kRowsPerGroup = 16 * kTilesPerWave;

// LDS-visible ordering of one wave's own LDS traffic: make the compiler keep program order
// across the point (the "memory" clobber) and drain outstanding LDS ops.
__device__ __forceinline__ void wave_lds_sync() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_wave_barrier();
}

__device__ __forceinline__ int64_t imin64(int64_t a, int64_t b) { return a < b ? a : b; }
__device__ __forceinline__ int64_t imax64(int64_t a, int64_t b) { return a > b ? a : b; }

__device__ __forceinline__ float4 ld4(const float* p) { return *reinterpret_cast<const float4*>(p); }

}  // namespace

namespace sml {
// Keyed pseudo-random bijection of [0, n) (a balanced 4-round Feistel network over the
// smallest even-bit domain >= n, cycle-walked back into range): an epoch's shuffle as a
// function of the row number, so a packed epoch needs no permutation array, no sort and no
// index reads.  The same function serves the host (FusedAE.perm_indices) and the kernels.
__host__ __device__ __forceinline__ uint64_t perm_mix(uint64_t z) {   // splitmix64 finaliser
  z ^= z >> 30;
  z *= 0xBF58476D1CE4E5B9ull;
  z ^= z >> 27;
  z *= 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
__host__ __device__ __forceinline__ uint64_t perm_apply(uint64_t v, uint64_t key, int half) {
  const uint64_t mask = (1ull << half) - 1ull;
  uint64_t L = v >> half, R = v & mask;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const uint64_t F = perm_mix(R ^ (key + 0x9E3779B97F4A7C15ull * (uint64_t)(i + 1))) & mask;
    const uint64_t t = L ^ F;
    L = R;
    R = t;
  }
  return (L << half) | R;
}
__host__ __device__ __forceinline__ int64_t perm_row(int64_t r, int64_t n, uint64_t key, int half) {
  uint64_t v = perm_apply((uint64_t)r, key, half);
  while (v >= (uint64_t)n) v = perm_apply(v, key, half);   // cycle walk: a bijection on [0, n)
  return (int64_t)v;
}
int perm_half_bits(int64_t n) {
  int b = 2;
  while (b < 62 && (1ll << b) < n) b += 2;
  return b / 2;
}
}  // namespace sml

namespace {

// Where packed row r comes from: r itself, index[r], or the keyed bijection perm_row(r).
struct RowSource {
  const int64_t* index;
  uint64_t key;
  int64_t pn;
  int half;   // > 0: permutation
  __device__ __forceinline__ bool gather() const { return index != nullptr || half > 0; }
  __device__ __forceinline__ int64_t operator()(int64_t r) const {
    if (index) return index[r];
    if (half > 0) return sml::perm_row(r, pn, key, half);
    return r;
  }
};

// argmax over D normalised values of one LDS-resident row: ties to the lowest index, NaN
// never wins (the same comparison order as the training kernels' metric)
template <int DT>
__device__ __forceinline__ int argmax_row(const float* row, int Drt) {
  const int D = DT > 0 ? DT : Drt;
  float best = row[0];
  int bi = 0;
#pragma unroll 6
  for (int j = 1; j < D; ++j) {
    const float v = row[j];
    if (v > best) {
      best = v;
      bi = j;
    }
  }
  return bi;
}

// Stage rows [r0, r0 + nrows) of x (row stride ld) into LDS as normalised fp32, flat [row][D].
// CONTIG (ld == D, x 16-byte aligned, r0 * D a multiple of 4): float4 loads; the per-position
// scale table has 4 * ceil(...) entries indexed by the flat position modulo the table period.
// Generic path (strided rows, or rows gathered through `index`: row r of the group is
// x[index[r0 + r]], e.g. an epoch's shuffle permutation fused into the pack): one element per
// lane, consecutive lanes on consecutive columns of a row.
template <int DT, bool CONTIG>
__device__ __forceinline__ void stage_rows(const float* __restrict__ x, int64_t r0, int nrows, int64_t ld, int Drt,
                                           const float* s_sc, const float* s_sh, int period, float* stage, int lane,
                                           float* __restrict__ out_stream, int64_t out_chunk0, int tile_chunks,
                                           const RowSource& src = RowSource{nullptr, 0, 0, 0},
                                           int64_t* s_src = nullptr, bool vec2 = false) {
  const int D = DT > 0 ? DT : Drt;
  const int nflt = nrows * D;
  if (CONTIG) {
    const float* src = x + r0 * (int64_t)D;
    const int nvec = nflt >> 2;
    for (int c = lane; c < nvec; c += 64) {
      float4 v = ld4(src + 4 * c);
      const int p = (4 * c) % period;
      const float4 a = *reinterpret_cast<const float4*>(s_sc + p);
      const float4 b = *reinterpret_cast<const float4*>(s_sh + p);
      v.x = fmaf(v.x, a.x, b.x);
      v.y = fmaf(v.y, a.y, b.y);
      v.z = fmaf(v.z, a.z, b.z);
      v.w = fmaf(v.w, a.w, b.w);
      *reinterpret_cast<float4*>(stage + 4 * c) = v;
      if (out_stream) {   // tile-packed output: tile t's 4D float4s, then its argmax float4
        const int t = c / tile_chunks, w = c - t * tile_chunks;
        *reinterpret_cast<float4*>(out_stream + 4 * (out_chunk0 + (int64_t)t * (tile_chunks + 1) + w)) = v;
      }
    }
    for (int e = 4 * nvec + lane; e < nflt; e += 64) {   // ragged tail of a partial group
      const int col = e % D;
      stage[e] = fmaf(src[e], s_sc[col], s_sh[col]);
    }
  } else {
    if (src.gather()) {
      // source rows first (index reads / bijection once per row, into LDS), then the row
      // loads all independent: many in flight per lane
      for (int r = lane; r < nrows; r += 64) s_src[r] = src(r0 + r);
      wave_lds_sync();
      if (DT > 0 && (DT & 1) == 0 && vec2) {   // 8-byte aligned rows: D / 2 float2 loads each
        constexpr int H = DT / 2;
        const int nv = nrows * H;
#pragma unroll 4
        for (int c = lane; c < nv; c += 64) {
          const int r = c / H, seg = c - r * H;
          const float2 v = *reinterpret_cast<const float2*>(x + s_src[r] * ld + 2 * seg);
          const int col = 2 * seg;
          *reinterpret_cast<float2*>(stage + r * D + col) =
              make_float2(fmaf(v.x, s_sc[col], s_sh[col]), fmaf(v.y, s_sc[col + 1], s_sh[col + 1]));
        }
      } else {
#pragma unroll 4
        for (int e = lane; e < nflt; e += 64) {
          const int r = e / D, col = e - r * D;
          stage[e] = fmaf(x[s_src[r] * ld + col], s_sc[col], s_sh[col]);
        }
      }
    } else {
      for (int e = lane; e < nflt; e += 64) {
        const int r = e / D, col = e - r * D;
        stage[e] = fmaf(x[(r0 + r) * ld + col], s_sc[col], s_sh[col]);
      }
    }
    if (out_stream) {
      wave_lds_sync();
      const int nvec = nflt >> 2;   // pack: nrows is a multiple of 16, so nflt % 4 == 0
      for (int c = lane; c < nvec; c += 64) {
        const int t = c / tile_chunks, w = c - t * tile_chunks;
        *reinterpret_cast<float4*>(out_stream + 4 * (out_chunk0 + (int64_t)t * (tile_chunks + 1) + w)) =
            *reinterpret_cast<const float4*>(stage + 4 * c);
      }
    }
  }
}

// Scale / shift tables in LDS, indexed by flat position p in [0, period): column p % D.
// period = lcm-friendly 4 * D (a multiple of both 4 and D), so a float4 never wraps.
__device__ __forceinline__ void load_tables(float* s_sc, float* s_sh, int period, int D, const float* scale,
                                            const float* shift) {
  for (int p = threadIdx.x; p < period; p += kThreads) {
    const int col = p % D;
    s_sc[p] = scale ? scale[col] : 1.0f;
    s_sh[p] = scale ? shift[col] : 0.0f;
  }
}

// MODE 0: tile-pack (rows + argmax bytes per 16-row tile); MODE 1: argmax bytes only.
template <int DT, bool CONTIG, int MODE>
__global__ __launch_bounds__(kThreads) void rows_group_kernel(const float* __restrict__ x, int64_t n, int64_t ld,
                                                              int Drt, const float* __restrict__ scale,
                                                              const float* __restrict__ shift,
                                                              uint8_t* __restrict__ out, RowSource src,
                                                              int vec2) {
  const int D = DT > 0 ? DT : Drt;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int period = 4 * D;
  float* s_sc = reinterpret_cast<float*>(smem);
  float* s_sh = s_sc + period;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  // per wave: the staged rows | 128 argmax bytes | 128 source-row indices
  const int srcw = src.gather() ? 2 * kRowsPerGroup : 0;   // contiguous packs keep 4 blocks per CU
  float* stage = s_sh + period + wid * (kRowsPerGroup * D + 32 + srcw);
  uint8_t* s_arg = reinterpret_cast<uint8_t*>(stage + kRowsPerGroup * D);
  int64_t* s_src = reinterpret_cast<int64_t*>(stage + kRowsPerGroup * D + 32);
  load_tables(s_sc, s_sh, period, D, scale, shift);
  __syncthreads();
  const int tile_chunks = 4 * D;   // float4s of one 16-row tile
  const int64_t groups = (n + kRowsPerGroup - 1) / kRowsPerGroup;
  for (int64_t g = (int64_t)blockIdx.x * kWaves + wid; g < groups; g += (int64_t)gridDim.x * kWaves) {
    const int64_t r0 = g * kRowsPerGroup;
    const int nrows = (int)imin64(kRowsPerGroup, n - r0);
    float* ostream = MODE == 0 ? reinterpret_cast<float*>(out) : nullptr;
    stage_rows<DT, CONTIG>(x, r0, nrows, ld, D, s_sc, s_sh, period, stage, lane, ostream,
                           (r0 >> 4) * (int64_t)(tile_chunks + 1), tile_chunks, src, s_src, vec2 != 0);
    wave_lds_sync();
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int r = lane + 64 * h;
      if (r < nrows) {
        const int a = argmax_row<DT>(stage + r * D, D);
        if (MODE == 0)
          s_arg[r] = (uint8_t)a;
        else
          out[r0 + r] = (uint8_t)a;   // 64 consecutive bytes per instruction
      }
    }
    if (MODE == 0) {
      wave_lds_sync();
      const int ntiles = nrows >> 4;
      if (lane < ntiles) {
        const int64_t t = (r0 >> 4) + lane;
        *reinterpret_cast<uint4*>(out + (t * (tile_chunks + 1) + tile_chunks) * 16) =
            *reinterpret_cast<const uint4*>(s_arg + 16 * lane);
      }
    }
    wave_lds_sync();   // the stage is rewritten by the next group
  }
}

size_t rows_group_lds(int D, bool gather) {
  return (size_t)(8 * D + kWaves * (kRowsPerGroup * D + 32 + (gather ? 2 * kRowsPerGroup : 0))) * sizeof(float);
}

int stream_grid(int64_t groups_of_waves) {
  // enough waves for every CU to keep ~8 groups in flight; grid-stride beyond that
  const int64_t cap = 256 * 8;
  return (int)std::max<int64_t>(1, std::min<int64_t>(cap, (groups_of_waves + kWaves - 1) / kWaves));
}

template <int MODE>
hipError_t launch_rows_group(const float* x, int64_t n, int64_t ld, int D, const float* scale, const float* shift,
                             uint8_t* out, hipStream_t stream, RowSource src = RowSource{nullptr, 0, 0, 0}) {
  const bool gather = src.index != nullptr || src.half > 0;
  const bool contig = !gather && ld == D && (reinterpret_cast<uintptr_t>(x) & 15) == 0;
  const int vec2 = (ld & 1) == 0 && (reinterpret_cast<uintptr_t>(x) & 7) == 0;
  const int64_t groups = (n + kRowsPerGroup - 1) / kRowsPerGroup;
  const dim3 grid(stream_grid(groups)), block(kThreads);
  const size_t lds = rows_group_lds(D, gather);
  if (lds > 160 * 1024) return hipErrorInvalidValue;
  if (lds > 65536) {
    hipError_t e = hipSuccess;
    if (D == 18 && contig)
      e = hipFuncSetAttribute(reinterpret_cast<const void*>(rows_group_kernel<18, true, MODE>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    else if (contig)
      e = hipFuncSetAttribute(reinterpret_cast<const void*>(rows_group_kernel<0, true, MODE>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    else if (D == 18)
      e = hipFuncSetAttribute(reinterpret_cast<const void*>(rows_group_kernel<18, false, MODE>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    else
      e = hipFuncSetAttribute(reinterpret_cast<const void*>(rows_group_kernel<0, false, MODE>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return e;
  }
  if (D == 18 && contig)
    hipLaunchKernelGGL((rows_group_kernel<18, true, MODE>), grid, block, lds, stream, x, n, ld, D, scale, shift, out,
                       src, vec2);
  else if (contig)
    hipLaunchKernelGGL((rows_group_kernel<0, true, MODE>), grid, block, lds, stream, x, n, ld, D, scale, shift, out,
                       src, vec2);
  else if (D == 18)
    hipLaunchKernelGGL((rows_group_kernel<18, false, MODE>), grid, block, lds, stream, x, n, ld, D, scale, shift, out,
                       src, vec2);
  else
    hipLaunchKernelGGL((rows_group_kernel<0, false, MODE>), grid, block, lds, stream, x, n, ld, D, scale, shift, out,
                       src, vec2);
  return hipGetLastError();
}

__global__ __launch_bounds__(256) void perm_indices_kernel(int64_t* __restrict__ out, int64_t start, int64_t count,
                                                           int64_t n, uint64_t key, int half) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i < count) out[i] = sml::perm_row(start + i, n, key, half);
}

// ---------------------------------------------------------------- normalize + filter
constexpr int kChunk = 4096;                  // rows per scatter workgroup (16 x 256)
constexpr int kScanThreads = 1024;

__device__ __forceinline__ bool keep_row(const uint8_t* labels, int64_t r, int keep) {
  return keep < 0 || labels[r] == (uint8_t)keep;
}

__device__ __forceinline__ int count_eq(uint32_t w, uint32_t k4) {
  // bytes of w equal to the byte broadcast in k4: zero-byte detection on w ^ k4
  const uint32_t z = w ^ k4;
  const uint32_t t = ((z & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | z;   // high bit set where byte != 0
  return 4 - __popc(t & 0x80808080u);
}

__global__ __launch_bounds__(kThreads) void filter_count_kernel(const uint8_t* __restrict__ labels, int64_t n,
                                                                int keep, int aligned, int* __restrict__ counts) {
  __shared__ int red[kWaves];
  const int64_t base = (int64_t)blockIdx.x * kChunk;
  const int64_t r = base + 16 * (int64_t)threadIdx.x;   // this lane's 16 labels
  int c = 0;
  if (keep < 0) {
    c = (int)imax64(0, imin64(16, n - r));
  } else if (aligned && r + 16 <= n) {
    const uint4 w = *reinterpret_cast<const uint4*>(labels + r);
    const uint32_t k4 = 0x01010101u * (uint32_t)(uint8_t)keep;
    c = count_eq(w.x, k4) + count_eq(w.y, k4) + count_eq(w.z, k4) + count_eq(w.w, k4);
  } else {
    for (int k = 0; k < 16; ++k) c += (r + k < n && keep_row(labels, r + k, keep)) ? 1 : 0;
  }
  c = (int)sml::wave_sum((float)c);   // exact: <= 1024 per wave
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = c;
  __syncthreads();
  if (threadIdx.x == 0) counts[blockIdx.x] = red[0] + red[1] + red[2] + red[3];
}

// exclusive scan of the per-block counts, in place; total kept rows -> total[0]
__global__ __launch_bounds__(kScanThreads) void filter_scan_kernel(int* __restrict__ counts, int nb,
                                                                   int64_t* __restrict__ total) {
  __shared__ int s_w[kScanThreads / 64];
  __shared__ int s_carry;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  if (threadIdx.x == 0) s_carry = 0;
  __syncthreads();
  for (int base = 0; base < nb; base += kScanThreads) {
    const int i = base + (int)threadIdx.x;
    const int v = i < nb ? counts[i] : 0;
    int s = v;   // inclusive wave scan
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const int u = __shfl_up(s, o, 64);
      if (lane >= o) s += u;
    }
    if (lane == 63) s_w[wid] = s;
    __syncthreads();
    int woff = 0;
    for (int w = 0; w < wid; ++w) woff += s_w[w];
    int btot = 0;
    for (int w = 0; w < kScanThreads / 64; ++w) btot += s_w[w];
    const int carry = s_carry;
    if (i < nb) counts[i] = carry + woff + s - v;
    __syncthreads();
    if (threadIdx.x == 0) s_carry = carry + btot;
    __syncthreads();
  }
  if (threadIdx.x == 0) total[0] = (int64_t)s_carry;
}

template <int DT, bool CONTIG>
__global__ __launch_bounds__(kThreads) void filter_scatter_kernel(
    const float* __restrict__ x, int64_t n, int64_t ld, int Drt, const uint8_t* __restrict__ labels, int keep,
    const float* __restrict__ scale, const float* __restrict__ shift, const int* __restrict__ offsets,
    float* __restrict__ out, int64_t* __restrict__ out_index) {
  const int D = DT > 0 ? DT : Drt;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int period = 4 * D;
  float* s_sc = reinterpret_cast<float*>(smem);
  float* s_sh = s_sc + period;
  int* s_wave = reinterpret_cast<int*>(s_sh + period);          // kWaves (padded to 4)
  int* s_kl = s_wave + 4;                                        // kWaves x 64 kept-row lists
  float* stage0 = reinterpret_cast<float*>(s_kl + kWaves * 64);  // kWaves x 64 rows x D
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  float* stage = stage0 + wid * 64 * D;
  int* kl = s_kl + wid * 64;
  // the scatter normalises on the way out: stage raw rows (identity tables)
  for (int p = threadIdx.x; p < period; p += kThreads) {
    s_sc[p] = 1.0f;
    s_sh[p] = 0.0f;
  }
  __syncthreads();
  int running = offsets[blockIdx.x];
  const int64_t base = (int64_t)blockIdx.x * kChunk;
  for (int k = 0; k < kChunk / kThreads; ++k) {
    const int64_t r0 = base + (int64_t)k * kThreads + wid * 64;
    const int nrows = (int)imax64(0, imin64(64, n - r0));
    if (nrows > 0)
      stage_rows<DT, CONTIG>(x, r0, nrows, ld, D, s_sc, s_sh, period, stage, lane, nullptr, 0, 1);
    const int64_t r = r0 + lane;
    const bool kp = lane < nrows && keep_row(labels, r, keep);
    const uint64_t m = __ballot(kp);
    const int before = __popcll(m & ((1ull << lane) - 1ull));
    const int cnt = __popcll(m);
    if (kp) kl[before] = lane;
    if (lane == 0) s_wave[wid] = cnt;
    __syncthreads();
    int woff = 0;
    for (int w = 0; w < wid; ++w) woff += s_wave[w];
    const int tot = s_wave[0] + s_wave[1] + s_wave[2] + s_wave[3];
    const int64_t dst0 = (int64_t)running + woff;
    SML_DCHECK(dst0 + cnt <= r0 + 64 && dst0 + cnt <= n);   // compaction never moves a row forward
    // the wave's kept rows are one contiguous run of cnt * D floats in out: coalesced stores
    float* o = out + dst0 * D;
    for (int e = lane; e < cnt * D; e += 64) {
      const int j = e / D, col = e - j * D;
      o[e] = scale ? fmaf(stage[kl[j] * D + col], scale[col], shift[col]) : stage[kl[j] * D + col];
    }
    if (out_index && kp) out_index[dst0 + before] = r;
    running += tot;
    __syncthreads();   // s_wave / kl / stage reused next iteration
  }
}

}  // namespace

namespace sml {

int filter_blocks(int64_t n) { return (int)((n + kChunk - 1) / kChunk); }

hipError_t normalize_filter_launch(const float* x, int64_t n, int64_t ld, int D, const uint8_t* labels, int keep,
                                   const float* scale, const float* shift, int* counts, float* out,
                                   int64_t* out_index, int64_t* total, hipStream_t stream) {
  if (D < 1 || D > 64 || n < 0) return hipErrorInvalidValue;
  const int blocks = filter_blocks(n);
  if (blocks == 0) return hipMemsetAsync(total, 0, sizeof(int64_t), stream);
  const int aligned = labels != nullptr && (reinterpret_cast<uintptr_t>(labels) & 15) == 0;
  hipLaunchKernelGGL(filter_count_kernel, dim3(blocks), dim3(kThreads), 0, stream, labels, n, keep, aligned, counts);
  hipLaunchKernelGGL(filter_scan_kernel, dim3(1), dim3(kScanThreads), 0, stream, counts, blocks, total);
  const bool contig = ld == D && (reinterpret_cast<uintptr_t>(x) & 15) == 0;
  const size_t lds = (size_t)(8 * D + 4 + kWaves * 64 + kWaves * 64 * D) * sizeof(float);
  if (D == 18 && contig)
    hipLaunchKernelGGL((filter_scatter_kernel<18, true>), dim3(blocks), dim3(kThreads), lds, stream, x, n, ld, D,
                       labels, keep, scale, shift, counts, out, out_index);
  else if (contig)
    hipLaunchKernelGGL((filter_scatter_kernel<0, true>), dim3(blocks), dim3(kThreads), lds, stream, x, n, ld, D,
                       labels, keep, scale, shift, counts, out, out_index);
  else
    hipLaunchKernelGGL((filter_scatter_kernel<0, false>), dim3(blocks), dim3(kThreads), lds, stream, x, n, ld, D,
                       labels, keep, scale, shift, counts, out, out_index);
  return hipGetLastError();
}

hipError_t pack_tiles_argmax_launch(const float* x, int64_t n, int64_t ld, int D, const float* scale,
                                    const float* shift, uint8_t* out, hipStream_t stream, const int64_t* index,
                                    uint64_t perm_key, int64_t perm_n) {
  if (n <= 0) return hipSuccess;
  if ((n & 15) || D < 1 || D > 64) return hipErrorInvalidValue;
  if (reinterpret_cast<uintptr_t>(out) & 15) return hipErrorInvalidValue;
  if (perm_n > 0 && (index != nullptr || n > perm_n)) return hipErrorInvalidValue;
  const RowSource src{index, perm_key, perm_n, perm_n > 0 ? perm_half_bits(perm_n) : 0};
  return launch_rows_group<0>(x, n, ld, D, scale, shift, out, stream, src);
}

hipError_t perm_indices_launch(int64_t* out, int64_t start, int64_t count, int64_t n, uint64_t key,
                               hipStream_t stream) {
  if (count <= 0) return hipSuccess;
  if (n <= 0 || start < 0 || start + count > n) return hipErrorInvalidValue;
  hipLaunchKernelGGL(perm_indices_kernel, dim3((unsigned)((count + 255) / 256)), dim3(256), 0, stream, out, start,
                     count, n, key, perm_half_bits(n));
  return hipGetLastError();
}

hipError_t row_argmax_launch(const float* x, int64_t n, int64_t ld, int D, const float* scale, const float* shift,
                             uint8_t* out, hipStream_t stream) {
  if (n <= 0) return hipSuccess;
  if (D < 1 || D > 64) return hipErrorInvalidValue;
  return launch_rows_group<1>(x, n, ld, D, scale, shift, out, stream);
}

}  // namespace sml
