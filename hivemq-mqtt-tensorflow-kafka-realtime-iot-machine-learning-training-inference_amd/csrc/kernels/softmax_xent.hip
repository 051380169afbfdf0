// K13: fused softmax + sparse categorical cross-entropy, forward AND backward in
// one pass (the MNIST heads of
// python-scripts/tensorflow-kafka-mnist.py:40-47 and
// confluent-tensorflow-io-kafka-simplified.py:10-21:
// Dense(10, softmax) + loss='sparse_categorical_crossentropy', metrics=['accuracy']).
//
// Keras applies softmax in the layer and then takes -log(p[y]) with p clipped
// to [eps, 1-eps]; computing log-softmax directly from the logits is the
// numerically exact form of the same loss (identical wherever the clip is
// inactive, which is every non-saturated row) and gives the textbook gradient
// dL/dz = softmax(z) - onehot(y).
//
// Layout: one row per lane (C <= 32 classes live in VGPRs), 256-thread blocks =
// 4 wave64s; per-block loss / correct sums are reduced with DPP/shuffles + LDS
// and added with one float atomic per block into acc[0..1].  Rows with a label
// outside [0, C) are ignored (no loss, zero gradient) -- the tf.data pipeline
// would have raised; here a poison record must not kill a streaming job.
#include "sml_common.h"
#include "sml_ops.h"

namespace sml {
namespace {

constexpr int kThreads = 256;

template <int C>
__global__ __launch_bounds__(kThreads) void softmax_xent_kernel(const float* __restrict__ logits,
                                                                 const int64_t* __restrict__ labels, int64_t B,
                                                                 float gscale, float* __restrict__ dlogits,
                                                                 float* __restrict__ probs, float* __restrict__ acc) {
  __shared__ float red[2][kThreads / 64];
  const int64_t row = (int64_t)blockIdx.x * kThreads + threadIdx.x;
  float loss = 0.f, correct = 0.f;
  if (row < B) {
    const float* z = logits + row * C;
    float v[C];
#pragma unroll
    for (int j = 0; j < C; ++j) v[j] = z[j];
    float mx = v[0];
    int amax = 0;
#pragma unroll
    for (int j = 1; j < C; ++j) {
      if (v[j] > mx) { mx = v[j]; amax = j; }  // first maximal index (tf.argmax)
    }
    float s = 0.f;
#pragma unroll
    for (int j = 0; j < C; ++j) {
      v[j] = __expf(v[j] - mx);
      s += v[j];
    }
    const float inv = __frcp_rn(s);
    const int64_t y = labels[row];
    const bool ok = y >= 0 && y < C;
    if (ok) {
      float zy = 0.f;
#pragma unroll
      for (int j = 0; j < C; ++j) zy = (j == (int)y) ? z[j] : zy;
      loss = (mx - zy) + __logf(s);
      correct = (amax == (int)y) ? 1.f : 0.f;
    }
    if (probs) {
#pragma unroll
      for (int j = 0; j < C; ++j) probs[row * C + j] = v[j] * inv;
    }
    if (dlogits) {
#pragma unroll
      for (int j = 0; j < C; ++j) {
        const float p = v[j] * inv;
        dlogits[row * C + j] = ok ? (p - (j == (int)y ? 1.f : 0.f)) * gscale : 0.f;
      }
    }
  }
  if (acc) {
    loss = wave_sum(loss);
    correct = wave_sum(correct);
    const int w = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) {
      red[0][w] = loss;
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

template <int C>
hipError_t launch_c(const float* logits, const int64_t* labels, int64_t B, float gscale, float* dlogits, float* probs,
                    float* acc, hipStream_t stream) {
  const int64_t grid = (B + kThreads - 1) / kThreads;
  hipLaunchKernelGGL(softmax_xent_kernel<C>, dim3((unsigned)grid), dim3(kThreads), 0, stream, logits, labels, B,
                     gscale, dlogits, probs, acc);
  return hipGetLastError();
}

}  // namespace

hipError_t softmax_xent_launch(const float* logits, const int64_t* labels, int64_t B, int C, float gscale,
                               float* dlogits, float* probs, float* acc, hipStream_t stream) {
  if (B <= 0) return hipSuccess;
  switch (C) {
    case 2: return launch_c<2>(logits, labels, B, gscale, dlogits, probs, acc, stream);
    case 10: return launch_c<10>(logits, labels, B, gscale, dlogits, probs, acc, stream);
    case 16: return launch_c<16>(logits, labels, B, gscale, dlogits, probs, acc, stream);
    case 32: return launch_c<32>(logits, labels, B, gscale, dlogits, probs, acc, stream);
    default: return hipErrorInvalidValue;
  }
}

}  // namespace sml
