// K3 + K6: fused MSE loss forward/backward and categorical-accuracy metric in
// ONE pass (SURVEY.md §2.2 K3 mse_loss_fwd_bwd, K6 cat_accuracy), for the
// layer-by-layer models (LSTM predictor, generic nn.Model).  The fused AE kernel
// has its own in-register copy of the same math.
//
// Keras semantics (reference compile(loss='mean_squared_error', metrics=['accuracy'])):
//   loss     = mean over all elements of (y_pred - y)^2
//   dL/dy_pred = 2 (y_pred - y) / (rows * F)            (times an external scale)
//   accuracy = argmax(y_pred) == argmax(y) per row (first maximal index)
// ``bcast`` > 1 broadcasts one target row over ``bcast`` consecutive prediction
// rows (a [n, T, F] TimeDistributed output against [n, F] next-event targets,
// LSTM-TensorFlow-IO-Kafka/cardata-v2.py:183-206).
//
// One row per lane, rows staged through LDS: a block's RPB rows of y_pred (and of y when
// bcast = 1) are contiguous, so they come in and the gradient goes out as coalesced
// 16-byte accesses (a lane walking its own 72-byte row issued F scalar loads and stores
// per lane, 4-5x slower at F = 18).  Per-block partial sums are reduced with shuffles +
// LDS into one partial per block; a one-block kernel then folds the partials into acc
// [loss_sum, correct] in a fixed order (deterministic).  The earlier one-atomic-per-block
// fold serialised ~1000 same-address float atomics: 17.4 vs 4.4 us for the kernel at
// 65 536 x 18 (profiles/r04, tools/lstm_probe/head_probe.py).  Torch-side this replaces
// ~10 elementwise / reduction kernels per training step.
#include "sml_common.h"
#include "sml_ops.h"

namespace sml {
namespace {

template <int F>
constexpr int rows_per_block() { return F <= 16 ? 256 : (F <= 32 ? 128 : 64); }

template <int F>
__global__ __launch_bounds__(rows_per_block<F>()) void mse_acc_kernel(const float* __restrict__ yp,
                                                                      const float* __restrict__ y, int64_t rows,
                                                                      int bcast, float gscale,
                                                                      float* __restrict__ grad,
                                                                      float* __restrict__ part) {
  constexpr int RPB = rows_per_block<F>(), NW = RPB / 64;
  __shared__ __attribute__((aligned(16))) float sp[RPB * F];
  __shared__ __attribute__((aligned(16))) float st[RPB * F];
  __shared__ float red[2][NW];
  const int64_t r0 = (int64_t)blockIdx.x * RPB;
  const int nr = (int)(rows - r0 < RPB ? rows - r0 : RPB);
  const int n = nr * F;
  const float* pb = yp + r0 * F;
  const float* tb = y + r0 * F;
  const bool vec = ((n & 3) == 0) && ((reinterpret_cast<uintptr_t>(pb) & 15) == 0) &&
                   (bcast != 1 || (reinterpret_cast<uintptr_t>(tb) & 15) == 0) &&
                   (!grad || (reinterpret_cast<uintptr_t>(grad + r0 * F) & 15) == 0);
  if (vec) {
    for (int i = threadIdx.x; i < n / 4; i += RPB) {
      reinterpret_cast<f32x4*>(sp)[i] = reinterpret_cast<const f32x4*>(pb)[i];
      if (bcast == 1) reinterpret_cast<f32x4*>(st)[i] = reinterpret_cast<const f32x4*>(tb)[i];
    }
  } else {
    for (int i = threadIdx.x; i < n; i += RPB) {
      sp[i] = pb[i];
      if (bcast == 1) st[i] = tb[i];
    }
  }
  __syncthreads();
  float se = 0.f, correct = 0.f;
  const int rl = threadIdx.x;
  if (rl < nr) {
    const int64_t r = r0 + rl;
    float* p = sp + rl * F;
    const float* t = bcast == 1 ? st + rl * F : y + (r / bcast) * F;
    float mp = -INFINITY, mt = -INFINITY;
    int ip = 0, it = 0;
#pragma unroll
    for (int j = 0; j < F; ++j) {
      const float a = p[j], b = t[j];
      const float d = a - b;
      se = fmaf(d, d, se);
      p[j] = d * gscale;                      // the gradient, written back in place
      if (a > mp) { mp = a; ip = j; }
      if (b > mt) { mt = b; it = j; }
    }
    correct = ip == it ? 1.f : 0.f;
  }
  if (grad) {
    __syncthreads();
    float* gb = grad + r0 * F;
    if (vec) {
      for (int i = threadIdx.x; i < n / 4; i += RPB) reinterpret_cast<f32x4*>(gb)[i] = reinterpret_cast<const f32x4*>(sp)[i];
    } else {
      for (int i = threadIdx.x; i < n; i += RPB) gb[i] = sp[i];
    }
  }
  if (part) {
    se = wave_sum(se);
    correct = wave_sum(correct);
    const int w = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) {
      red[0][w] = se;
      red[1][w] = correct;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      float a = 0.f, b = 0.f;
#pragma unroll
      for (int i = 0; i < NW; ++i) {
        a += red[0][i];
        b += red[1][i];
      }
      part[2 * blockIdx.x] = a;
      part[2 * blockIdx.x + 1] = b;
    }
  }
}

// acc[k] (+)= sum over the n block partials part[2 i + k], in a fixed order; out (optional):
// out[k] = acc[k] / div[k] -- a train step's loss and accuracy, normalised in this launch
// instead of two torch ops (a division and a copy) on the stream after it
__global__ __launch_bounds__(256) void acc_fold_kernel(const float* __restrict__ part, int n, float* __restrict__ acc,
                                                       int reset, float* __restrict__ out, float div0, float div1,
                                                       int64_t* __restrict__ counter) {
  __shared__ float red[2][4];
  float a = 0.f, b = 0.f;
  for (int i = threadIdx.x; i < n; i += 256) {
    a += part[2 * i];
    b += part[2 * i + 1];
  }
  a = wave_sum(a);
  b = wave_sum(b);
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) {
    red[0][w] = a;
    red[1][w] = b;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    const float sa = (red[0][0] + red[0][1]) + (red[0][2] + red[0][3]);
    const float sb = (red[1][0] + red[1][1]) + (red[1][2] + red[1][3]);
    const float a0 = reset ? sa : acc[0] + sa, a1 = reset ? sb : acc[1] + sb;
    acc[0] = a0;
    acc[1] = a1;
    if (out) {
      out[0] = a0 / div0;
      out[1] = a1 / div1;
    }
    if (counter) counter[0] += 1;   // the optimizer's step count (read by the Adam launch after this)
  }
}

}  // namespace

int mse_acc_blocks(int64_t rows, int F) {
  const int R = F <= 16 ? 256 : (F <= 32 ? 128 : 64);   // rows_per_block<F>()
  return (int)((rows + R - 1) / R);
}

hipError_t mse_acc_launch(const float* yp, const float* y, int64_t rows, int F, int bcast, float gscale, float* grad,
                          float* acc, float* part, int reset, hipStream_t stream, float* out, float div0,
                          float div1, int64_t* counter) {
  if (rows <= 0) return hipSuccess;
  if (bcast < 1 || (acc && !part)) return hipErrorInvalidValue;
  float* pp = acc ? part : nullptr;
#define SML_F(n)                                                                                              \
  case n: {                                                                                                  \
    constexpr int R = rows_per_block<n>();                                                                   \
    hipLaunchKernelGGL(mse_acc_kernel<n>, dim3((unsigned)((rows + R - 1) / R)), dim3(R), 0, stream, yp, y, rows, \
                       bcast, gscale, grad, pp);                                                             \
    break;                                                                                                   \
  }
  switch (F) {
    SML_F(1) SML_F(2) SML_F(4) SML_F(8) SML_F(10) SML_F(16) SML_F(18) SML_F(30) SML_F(32) SML_F(64)
    default: return hipErrorInvalidValue;
  }
#undef SML_F
  if (acc) hipLaunchKernelGGL(acc_fold_kernel, dim3(1), dim3(256), 0, stream, part, mse_acc_blocks(rows, F), acc, reset,
                               out, div0, div1, counter);
  return hipGetLastError();
}

bool mse_acc_supported(int F) {
  switch (F) {
    case 1: case 2: case 4: case 8: case 10: case 16: case 18: case 30: case 32: case 64: return true;
    default: return false;
  }
}

}  // namespace sml
