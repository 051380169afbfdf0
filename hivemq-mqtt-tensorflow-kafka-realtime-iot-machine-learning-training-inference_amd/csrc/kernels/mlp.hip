// Wide dense layers of the MNIST classifier on fp32 MFMA with an LDS-tiled K loop.
//
// Reference: python-scripts/tensorflow-kafka-mnist.py:39-47, confluent-tensorflow-io-kafka.py:
// 40-58 -- Flatten(28x28) -> Dense(128 | 512, relu) [-> Dropout(0.2)] -> Dense(10, softmax),
// Adam, sparse categorical cross-entropy.  K1/K2 (dense.hip) keep the whole weight in
// VGPRs and stop at KT*NT <= 32 tiles; the MNIST layers (784 x 128 / 512) need a K loop.
//
// One kernel template covers every GEMM of a training step:
//     C[M, N] = A[M, K] . B[K, N]   (A / B row-major or transposed, A uint8 or fp32)
//   fwd   : H  = dropout(relu(X . W1 + b1)),  Z = H . W2 + b2        (A = X | H)
//   data  : dH = (dZ . W2^T) * [H > 0] / keep                          (B = W2^T)
//   wgrad : [dW ; db] = [X ; 1]^T . dY  (the "ones row" makes the bias gradient row K
//           of the same product, and W, b are adjacent in the flat gradient buffer)
// Workgroup tile 32 x 32 (4 waves of one 16 x 16 MFMA tile each), K staged through LDS
// 16 at a time; v_mfma_f32_16x16x4f32 is exact fp32 (an fmaf chain), so the step
// matches the fp32 torch oracle to accumulation order.  uint8 images are scaled by
// 1/255 as they are staged (tf.image.convert_image_dtype), never materialised as fp32.
//
// Dropout (Keras inverted dropout, rate 1 - keep): the mask is a counter-based hash of
// (seed, step, row, column) evaluated in the forward epilogue; the backward needs no
// mask because H > 0 already implies "kept and active" (H = relu(z) * mask / keep).
#include "sml_common.h"
#include "sml_ops.h"

namespace sml {
namespace {

constexpr int TM = 32, TN = 32, TK = 16;
constexpr int AS = TK + 1, BS = TN + 1;   // LDS strides (odd: conflict-free)

enum AMode { A_F32 = 0, A_U8 = 1, A_F32_T = 2, A_U8_T = 3 };
enum Epi { E_STORE = 0, E_BIAS_ACT = 1, E_RELU_MASK = 2 };

__device__ __forceinline__ uint32_t mix32(uint32_t h) {   // murmur3 finaliser
  h ^= h >> 16;
  h *= 0x85ebca6bu;
  h ^= h >> 13;
  h *= 0xc2b2ae35u;
  h ^= h >> 16;
  return h;
}

// uniform [0, 1) with 24 bits, keyed by (seed, step, row, col)
__device__ __forceinline__ float dropout_u(uint32_t seed, uint32_t step, uint32_t row, uint32_t col) {
  uint32_t h = mix32(seed ^ 0x9e3779b9u);
  h = mix32(h ^ (step * 0x632be5abu));
  h = mix32(h ^ (row * 0x85157af5u));
  h = mix32(h ^ col);
  return (float)(h >> 8) * (1.0f / 16777216.0f);
}

struct GemmArgs {
  const void* A;
  int64_t lda;
  const float* B;
  int64_t ldb;
  float* C;
  int64_t ldc;
  int M, N, K;
  int ones_row;          // A row M-1 reads 1.0 (bias-gradient row)
  const float* bias;     // E_BIAS_ACT
  int relu;              // E_BIAS_ACT
  float keep;            // dropout keep probability (1: none)
  float inv_keep;        // 1 / keep (kept values are multiplied, as tf.nn.dropout does)
  uint32_t seed, step;
  const float* ref;      // E_RELU_MASK: H, same layout as C
  float scale;           // E_RELU_MASK: 1 / keep
};

template <int AM>
__device__ __forceinline__ float load_a(const GemmArgs& g, int i, int k) {
  if (i >= g.M || k >= g.K) return 0.0f;
  if (g.ones_row && i == g.M - 1) return 1.0f;
  if constexpr (AM == A_F32) return static_cast<const float*>(g.A)[(int64_t)i * g.lda + k];
  if constexpr (AM == A_U8) return (float)static_cast<const uint8_t*>(g.A)[(int64_t)i * g.lda + k] * (1.0f / 255.0f);
  if constexpr (AM == A_F32_T) return static_cast<const float*>(g.A)[(int64_t)k * g.lda + i];
  return (float)static_cast<const uint8_t*>(g.A)[(int64_t)k * g.lda + i] * (1.0f / 255.0f);
}

template <bool BT>
__device__ __forceinline__ float load_b(const GemmArgs& g, int k, int j) {
  if (k >= g.K || j >= g.N) return 0.0f;
  return BT ? g.B[(int64_t)j * g.ldb + k] : g.B[(int64_t)k * g.ldb + j];
}

template <int AM, bool BT, int EPI>
__global__ __launch_bounds__(256) void mlp_gemm_kernel(GemmArgs g) {
  __shared__ float As[TM * AS];
  __shared__ float Bs[TK * BS];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int m0 = blockIdx.y * TM, n0 = blockIdx.x * TN;
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  for (int k0 = 0; k0 < g.K; k0 += TK) {
    // stage A [32 x 16] and B [16 x 32]: 512 elements each, 2 per thread
#pragma unroll
    for (int e = 0; e < 2; ++e) {
      const int idx = tid + e * 256;
      // A: transposed sources are read along i (consecutive lanes -> consecutive rows)
      int ai, ak;
      if constexpr (AM == A_F32_T || AM == A_U8_T) {
        ai = idx & (TM - 1);
        ak = idx >> 5;
      } else {
        ai = idx >> 4;
        ak = idx & (TK - 1);
      }
      As[ai * AS + ak] = load_a<AM>(g, m0 + ai, k0 + ak);
      int bk, bj;
      if constexpr (BT) {
        bk = idx & (TK - 1);
        bj = idx >> 4;
      } else {
        bk = idx >> 5;
        bj = idx & (TN - 1);
      }
      Bs[bk * BS + bj] = load_b<BT>(g, k0 + bk, n0 + bj);
    }
    __syncthreads();
#pragma unroll
    for (int kk = 0; kk < TK; kk += 4) {
      const float a = As[(16 * wm + (lane & 15)) * AS + kk + (lane >> 4)];
      const float b = Bs[(kk + (lane >> 4)) * BS + 16 * wn + (lane & 15)];
      acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, acc, 0, 0, 0);
    }
    __syncthreads();
  }
  const int col = n0 + 16 * wn + (lane & 15);
  if (col >= g.N) return;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int row = m0 + 16 * wm + 4 * (lane >> 4) + r;
    if (row >= g.M) continue;
    float v = acc[r];
    const int64_t o = (int64_t)row * g.ldc + col;
    if constexpr (EPI == E_BIAS_ACT) {
      if (g.bias) v += g.bias[col];
      if (g.relu) v = fmaxf(v, 0.0f);
      if (g.keep < 1.0f) v = dropout_u(g.seed, g.step, (uint32_t)row, (uint32_t)col) < g.keep ? v * g.inv_keep : 0.0f;
    } else if constexpr (EPI == E_RELU_MASK) {
      v = g.ref[o] > 0.0f ? v * g.scale : 0.0f;
    }
    g.C[o] = v;
  }
}

template <int AM, bool BT, int EPI>
hipError_t launch(const GemmArgs& g, hipStream_t st) {
  const dim3 grid((unsigned)((g.N + TN - 1) / TN), (unsigned)((g.M + TM - 1) / TM));
  hipLaunchKernelGGL((mlp_gemm_kernel<AM, BT, EPI>), grid, dim3(256), 0, st, g);
  return hipGetLastError();
}

__global__ void dropout_mask_kernel(float* out, int M, int N, float keep, float inv_keep, uint32_t seed,
                                    uint32_t step) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= (int64_t)M * N) return;
  const int r = (int)(i / N), c = (int)(i % N);
  out[i] = dropout_u(seed, step, (uint32_t)r, (uint32_t)c) < keep ? inv_keep : 0.0f;
}

}  // namespace

// the forward epilogue's dropout multipliers (0 or 1/keep) for [M, N] (tests / oracles)
hipError_t mlp_dropout_mask_launch(float* out, int M, int N, float keep, uint32_t seed, uint32_t step,
                                   hipStream_t st) {
  const int64_t n = (int64_t)M * N;
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(dropout_mask_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, out, M, N, keep,
                     1.0f / keep, seed, step);
  return hipGetLastError();
}

hipError_t mlp_fwd_launch(const void* x, int x_u8, int64_t ldx, const float* W, const float* b, float* y, int M,
                          int K, int N, int relu, float keep, uint32_t seed, uint32_t step, hipStream_t st) {
  GemmArgs g{};
  g.A = x; g.lda = ldx; g.B = W; g.ldb = N; g.C = y; g.ldc = N;
  g.M = M; g.N = N; g.K = K; g.bias = b; g.relu = relu; g.keep = keep; g.inv_keep = 1.0f / keep;
  g.seed = seed; g.step = step;
  return x_u8 ? launch<A_U8, false, E_BIAS_ACT>(g, st) : launch<A_F32, false, E_BIAS_ACT>(g, st);
}

hipError_t mlp_bwd_data_launch(const float* dz, const float* W, const float* h, float* dh, int M, int N1, int N2,
                               float inv_keep, hipStream_t st) {
  // dH[M, N1] = dZ[M, N2] . W[N1, N2]^T, gated by H > 0
  GemmArgs g{};
  g.A = dz; g.lda = N2; g.B = W; g.ldb = N2; g.C = dh; g.ldc = N1;
  g.M = M; g.N = N1; g.K = N2; g.ref = h; g.scale = inv_keep;
  return launch<A_F32, true, E_RELU_MASK>(g, st);
}

hipError_t mlp_wgrad_launch(const void* x, int x_u8, int64_t ldx, const float* dy, float* out, int B, int K, int N,
                            hipStream_t st) {
  // out[K + 1, N] = [X ; 1]^T . dY : rows 0..K-1 = dW, row K = db
  GemmArgs g{};
  g.A = x; g.lda = ldx; g.B = dy; g.ldb = N; g.C = out; g.ldc = N;
  g.M = K + 1; g.N = N; g.K = B; g.ones_row = 1;
  return x_u8 ? launch<A_U8_T, false, E_STORE>(g, st) : launch<A_F32_T, false, E_STORE>(g, st);
}

}  // namespace sml
