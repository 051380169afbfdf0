// K8 normalize_filter: the reference's per-event tf.data graph
//   normalize_fn(...)                      cardata-v3.py:78-168  (per-column affine, 4 zeroed columns)
//   .filter(lambda x, y: y == "false")     cardata-v3.py:212     (train on normal events only)
// as one order-preserving stream compaction on the device, for raw rows that arrive
// through the pinned H2D ring together with their failure_occurred label codes.
//
// Two launches, deterministic and order-preserving:
//   1. count:   each workgroup counts the kept rows of its CHUNK-row slice;
//   2. scatter: each workgroup sums the counts of the slices before it (at most a
//      few hundred 4-byte reads), ranks its kept rows with wave ballots + LDS wave
//      offsets, and writes them normalised (x * scale + shift) to out[rank].
// The last workgroup also stores the total, so the caller can read one int64.
#include "sml_common.h"

namespace {

constexpr int kThreads = 256;
constexpr int kRowsPerThread = 16;
constexpr int kChunk = kThreads * kRowsPerThread;  // rows per workgroup

__device__ __forceinline__ bool keep_row(const uint8_t* labels, int64_t r, int keep) {
  return keep < 0 || labels[r] == (uint8_t)keep;
}

__global__ __launch_bounds__(kThreads) void filter_count_kernel(const uint8_t* __restrict__ labels, int64_t n,
                                                                int keep, int* __restrict__ counts) {
  __shared__ int red[kThreads / 64];
  const int64_t base = (int64_t)blockIdx.x * kChunk;
  int c = 0;
#pragma unroll 4
  for (int k = 0; k < kRowsPerThread; ++k) {
    const int64_t r = base + (int64_t)k * kThreads + threadIdx.x;
    c += (r < n && keep_row(labels, r, keep)) ? 1 : 0;
  }
  c = (int)sml::wave_sum((float)c);  // exact: at most 16 * 64 per wave
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = c;
  __syncthreads();
  if (threadIdx.x == 0) counts[blockIdx.x] = red[0] + red[1] + red[2] + red[3];
}

__global__ __launch_bounds__(kThreads) void filter_scatter_kernel(
    const float* __restrict__ x, int64_t n, int64_t ld, int D, const uint8_t* __restrict__ labels, int keep,
    const float* __restrict__ scale, const float* __restrict__ shift, const int* __restrict__ counts,
    float* __restrict__ out, int64_t* __restrict__ out_index, int64_t* __restrict__ total) {
  __shared__ int s_base;
  __shared__ int s_wave[kThreads / 64];
  __shared__ float s_sc[64], s_sh[64];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  if (threadIdx.x < 64) {
    const int f = (int)threadIdx.x;
    s_sc[f] = f < D ? (scale ? scale[f] : 1.0f) : 0.f;
    s_sh[f] = (f < D && scale) ? shift[f] : 0.f;
  }
  if (threadIdx.x == 0) {
    int b = 0;
    for (int i = 0; i < (int)blockIdx.x; ++i) b += counts[i];
    s_base = b;
    if (blockIdx.x == gridDim.x - 1) total[0] = (int64_t)(b + counts[blockIdx.x]);
  }
  __syncthreads();
  int running = s_base;
  const int64_t base = (int64_t)blockIdx.x * kChunk;
  for (int k = 0; k < kRowsPerThread; ++k) {
    const int64_t r = base + (int64_t)k * kThreads + threadIdx.x;
    const bool kp = r < n && keep_row(labels, r, keep);
    const uint64_t m = __ballot(kp);
    const int before = __popcll(m & ((1ull << lane) - 1ull));
    if (lane == 0) s_wave[wid] = __popcll(m);
    __syncthreads();
    int woff = 0;
    for (int w = 0; w < wid; ++w) woff += s_wave[w];
    const int tot = s_wave[0] + s_wave[1] + s_wave[2] + s_wave[3];
    if (kp) {
      const int64_t dst = (int64_t)(running + woff + before);
      SML_DCHECK(dst <= r && dst < n);   // compaction never moves a row forward
      const float* src = x + r * ld;
      float* o = out + dst * D;
      for (int f = 0; f < D; ++f) o[f] = fmaf(src[f], s_sc[f], s_sh[f]);
      if (out_index) out_index[dst] = r;
    }
    running += tot;
    __syncthreads();  // s_wave reused next iteration
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
  hipLaunchKernelGGL(filter_count_kernel, dim3(blocks), dim3(kThreads), 0, stream, labels, n, keep, counts);
  hipLaunchKernelGGL(filter_scatter_kernel, dim3(blocks), dim3(kThreads), 0, stream, x, n, ld, D, labels, keep, scale,
                     shift, counts, out, out_index, total);
  return hipGetLastError();
}

}  // namespace sml

// Ingest-time argmax of each normalised row (the data half of the accuracy metric,
// tf.argmax(x) of cardata-v3's `metrics=['accuracy']`): one thread per row, the same
// fmaf(x, scale, shift) the training kernels apply, ties to the lowest index.
namespace {
__global__ __launch_bounds__(256) void row_argmax_kernel(const float* __restrict__ x, int64_t n, int64_t ld, int D,
                                                         const float* __restrict__ scale,
                                                         const float* __restrict__ shift, uint8_t* __restrict__ out) {
  const int64_t r = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (r >= n) return;
  const float* row = x + r * ld;
  float best = 0.0f;
  int bi = 0;
  for (int j = 0; j < D; ++j) {
    const float v = scale ? fmaf(row[j], scale[j], shift[j]) : row[j];
    if (j == 0 || v > best) {
      best = v;
      bi = j;
    }
  }
  out[r] = (uint8_t)bi;
}
__device__ __forceinline__ int argmax_norm(const float* row, int D, const float* scale, const float* shift) {
  float best = 0.0f;
  int bi = 0;
  for (int j = 0; j < D; ++j) {
    const float v = scale ? fmaf(row[j], scale[j], shift[j]) : row[j];
    if (j == 0 || v > best) {
      best = v;
      bi = j;
    }
  }
  return bi;
}

__global__ __launch_bounds__(256) void pack_tiles_kernel(const float* __restrict__ x, int64_t n, int64_t ld, int D,
                                                         const float* __restrict__ scale,
                                                         const float* __restrict__ shift, uint8_t* __restrict__ out) {
  const int64_t r = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (r >= n) return;
  const float* row = x + r * ld;
  const int64_t tile_bytes = 64 * (int64_t)D + 16;
  uint8_t* t = out + (r >> 4) * tile_bytes;
  float* dst = reinterpret_cast<float*>(t) + (r & 15) * D;
  // normalize_fn once per event + the argmax of the normalised row
  for (int j = 0; j < D; ++j) dst[j] = scale ? fmaf(row[j], scale[j], shift[j]) : row[j];
  t[64 * D + (r & 15)] = (uint8_t)argmax_norm(row, D, scale, shift);
}
}  // namespace

namespace sml {
hipError_t pack_tiles_argmax_launch(const float* x, int64_t n, int64_t ld, int D, const float* scale,
                                    const float* shift, uint8_t* out, hipStream_t stream) {
  if (n <= 0) return hipSuccess;
  if ((n & 15) || D < 1 || D > 255) return hipErrorInvalidValue;
  hipLaunchKernelGGL(pack_tiles_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, stream, x, n, ld, D, scale,
                     shift, out);
  return hipGetLastError();
}

hipError_t row_argmax_launch(const float* x, int64_t n, int64_t ld, int D, const float* scale, const float* shift,
                             uint8_t* out, hipStream_t stream) {
  if (n <= 0) return hipSuccess;
  if (D < 1 || D > 255) return hipErrorInvalidValue;
  hipLaunchKernelGGL(row_argmax_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, stream, x, n, ld, D, scale,
                     shift, out);
  return hipGetLastError();
}
}  // namespace sml
