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
// One row per lane (F <= 64 values in registers), 256-thread blocks, per-block
// partial sums reduced with shuffles + LDS and ONE atomic per block into acc
// [loss_sum, correct]; torch-side this replaces ~10 elementwise / reduction
// kernels per training step.
#include "sml_common.h"
#include "sml_ops.h"

namespace sml {
namespace {

constexpr int kThreads = 256;

template <int F>
__global__ __launch_bounds__(kThreads) void mse_acc_kernel(const float* __restrict__ yp, const float* __restrict__ y,
                                                            int64_t rows, int bcast, float gscale,
                                                            float* __restrict__ grad, float* __restrict__ acc) {
  __shared__ float red[2][kThreads / 64];
  const int64_t r = (int64_t)blockIdx.x * kThreads + threadIdx.x;
  float se = 0.f, correct = 0.f;
  if (r < rows) {
    const float* p = yp + r * F;
    const float* t = y + (r / bcast) * F;
    float mp = -INFINITY, mt = -INFINITY;
    int ip = 0, it = 0;
#pragma unroll
    for (int j = 0; j < F; ++j) {
      const float a = p[j], b = t[j];
      const float d = a - b;
      se = fmaf(d, d, se);
      if (grad) grad[r * F + j] = d * gscale;
      if (a > mp) { mp = a; ip = j; }
      if (b > mt) { mt = b; it = j; }
    }
    correct = ip == it ? 1.f : 0.f;
  }
  if (acc) {
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
      for (int i = 0; i < kThreads / 64; ++i) {
        a += red[0][i];
        b += red[1][i];
      }
      atomicAdd(acc, a);
      atomicAdd(acc + 1, b);
    }
  }
}

}  // namespace

hipError_t mse_acc_launch(const float* yp, const float* y, int64_t rows, int F, int bcast, float gscale, float* grad,
                          float* acc, hipStream_t stream) {
  if (rows <= 0) return hipSuccess;
  if (bcast < 1) return hipErrorInvalidValue;
  const dim3 grid((unsigned)((rows + kThreads - 1) / kThreads));
#define SML_F(n)                                                                                               \
  case n:                                                                                                     \
    hipLaunchKernelGGL(mse_acc_kernel<n>, grid, dim3(kThreads), 0, stream, yp, y, rows, bcast, gscale, grad, acc); \
    break;
  switch (F) {
    SML_F(1) SML_F(2) SML_F(4) SML_F(8) SML_F(10) SML_F(16) SML_F(18) SML_F(30) SML_F(32) SML_F(64)
    default: return hipErrorInvalidValue;
  }
#undef SML_F
  return hipGetLastError();
}

bool mse_acc_supported(int F) {
  switch (F) {
    case 1: case 2: case 4: case 8: case 10: case 16: case 18: case 30: case 32: case 64: return true;
    default: return false;
  }
}

}  // namespace sml
