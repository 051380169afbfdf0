// Fused Dense head of the seq-50 LSTM predictor for gfx950: forward, MSE loss + categorical accuracy,
// and backward (dW, db, dh_T) of Dense(N) on the last LSTM layer's h_T in ONE pass over the rows,
// plus one small fold launch (reference LSTM-TensorFlow-IO-Kafka/cardata-v2.py:183-206: Dense(18)
// after LSTM(16), compile(loss='mean_squared_error', metrics=['accuracy'])).
//
// Why: the per-kernel path ran six launches per train step for this head -- dense_fwd (K1),
// mse_acc + acc_fold (K3 / K6), dense_wgrad + slab_sum (K2), dense_fwd again for dh = dy . W^T --
// 42 us of a 708 us config-3 step under rocprof (profiles/r06), almost all of it small-grid latency
// over ~9 MB of rows.  Here one wave owns 16-row tiles:
//   y^T   = W^T . h^T + b      2 x v_mfma_f32_16x16x16_bf16 (outputs 0..15, 16..31)
//   e     = y - target, loss += e^2, accuracy: first-max argmax over the N outputs (permlane merge)
//   dy    = e * gscale         (fp32; bf16 for the MFMAs, as the per-kernel path's K1 / K2 consume it)
//   dh^T  = W . dy^T           one 16x16x32 over both output tiles -> bf16 [n, 16] rows
//   dW   += h^T . dy, db += colsum(dy) over the wave's rows (two LDS transposes per tile)
// Each workgroup writes one compact partial [K x N | N | 2]; head_fold_kernel sums the partials
// in a fixed order (deterministic), scatters dW / db into the flat gradient through the dense
// slab map, and writes the step's loss / accuracy and the Adam step count, as acc_fold does.
// K = 16 (the LSTM's units), N <= 32.
#include "sml_common.h"
#include "sml_ops.h"

namespace sml {
namespace {

constexpr int HW = 4;   // waves per workgroup
constexpr int WS_ROW = 36;             // per-wave LDS partial: dW rows [16][WS_ROW] (32 used) ...
constexpr int WS_DB = 16 * WS_ROW;     // ... then db [32], loss, correct

struct HeadArgs {
  const __bf16* h;   // [n, 16] bf16, row stride ldh elements
  int64_t ldh;
  const float* W;    // [16, N]
  const float* b;    // [N]
  const float* y;    // [n, N] fp32, row stride ldy elements
  int64_t ldy;
  __bf16* dh;        // [n, 16] bf16 out, row stride 16
  float* part;       // [grid][16 N + N + 2]
  int64_t n;
  int N;
  float gscale;
};

__device__ __forceinline__ void argmax_merge(float& m, int& i, float m2, int i2) {
  if (m2 > m || (m2 == m && i2 < i)) {
    m = m2;
    i = i2;
  }
}

__global__ __launch_bounds__(HW * 64) void lstm_head_kernel(HeadArgs a) {
  const int lane = threadIdx.x & 63, c = lane & 15, g = lane >> 4;
  const int w = threadIdx.x >> 6;
  const int N = a.N;
  const int PS = 16 * N + N + 2;
  __shared__ __attribute__((aligned(16))) char scr[HW][3 * 512];
  __shared__ float slab[HW][WS_DB + 34];
  char* sc = scr[w];
  // A fragments: a1[t] = W^T tile t ([m = output 16t + c][k = unit 4g + j]), a2[t] = W ([m = unit c]
  // [k = output 16t + 4g + j]), bias in the C rows of tile t (outputs 16t + 4g + i)
  bf16x4 a1[2], a2[2];
  f32x4 bias[2];
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    f32x4 u, v;
#pragma unroll
    for (int j = 0; j < 4; ++j) {   // clamped addresses, values selected after the load (no branches)
      const int o1 = 16 * t + c, o2 = 16 * t + 4 * g + j;
      const float wu = a.W[(4 * g + j) * N + (o1 < N ? o1 : 0)], wv = a.W[c * N + (o2 < N ? o2 : 0)];
      const float bb = a.b[o2 < N ? o2 : 0];
      u[j] = o1 < N ? wu : 0.f;
      v[j] = o2 < N ? wv : 0.f;
      bias[t][j] = o2 < N ? bb : 0.f;
    }
    a1[t] = pack4(u);
    a2[t] = pack4(v);
  }
  const f32x4 zero4 = {0.f, 0.f, 0.f, 0.f};
  f32x4 accW[2] = {zero4, zero4}, dbl[2] = {zero4, zero4};
  float se = 0.f, correct = 0.f;
  const int64_t ntile = (a.n + 15) / 16;
  for (int64_t tile = (int64_t)blockIdx.x * HW + w; tile < ntile; tile += (int64_t)gridDim.x * HW) {
    const int64_t row = tile * 16 + c;
    const bool valid = row < a.n;
    const int64_t rc = valid ? row : a.n - 1;
    const bf16x4 hb = *reinterpret_cast<const bf16x4*>(a.h + rc * a.ldh + 4 * g);
    f32x4 yp[2], tg[2], e[2];
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      yp[t] = mfma16(a1[t], hb, bias[t]);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int o = 16 * t + 4 * g + i;
        tg[t][i] = a.y[rc * a.ldy + (o < N ? o : 0)];
        e[t][i] = (valid && o < N) ? yp[t][i] - tg[t][i] : 0.f;
        se = fmaf(e[t][i], e[t][i], se);
      }
    }
    // categorical accuracy: first maximal output of the prediction and of the target, per row
    float mp = -INFINITY, mt = -INFINITY;
    int ip = 0, it = 0;
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int i = 0; i < 4; ++i) {   // selects only: outputs past N compare as -inf
        const int o = 16 * t + 4 * g + i;
        const float pv = o < N ? yp[t][i] : -INFINITY, tv = o < N ? tg[t][i] : -INFINITY;
        const bool bp = pv > mp, bt = tv > mt;
        mp = bp ? pv : mp;
        ip = bp ? o : ip;
        mt = bt ? tv : mt;
        it = bt ? o : it;
      }
#pragma unroll
    for (int s = 16; s <= 32; s <<= 1) {   // merge the 4 lane groups holding the row's outputs
      argmax_merge(mp, ip, __shfl_xor(mp, s, 64), __shfl_xor(ip, s, 64));
      argmax_merge(mt, it, __shfl_xor(mt, s, 64), __shfl_xor(it, s, 64));
    }
    correct += (valid && g == 0 && ip == it) ? 1.f : 0.f;
    bf16x4 dyb[2];
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      f32x4 dy;
#pragma unroll
      for (int i = 0; i < 4; ++i) dy[i] = e[t][i] * a.gscale;
      dbl[t] += dy;
      dyb[t] = pack4(dy);
    }
    // dh^T = W . dy^T: both output tiles as the two K halves of one 16x16x32
    const f32x4 dhT = mfma32(a2[0], a2[1], dyb[0], dyb[1], zero4);
    if (valid) *reinterpret_cast<bf16x4*>(a.dh + row * 16 + 4 * g) = pack4(dhT);
    // dW += h^T . dy over the tile's rows: rows onto K through the LDS transpose
    const bf16x4 hA = lds_transpose(hb, sc, c, g);
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      const bf16x4 dB = lds_transpose(dyb[t], sc + 512 * (1 + t), c, g);
      accW[t] = mfma16(hA, dB, accW[t]);
    }
  }
  // db: fold the 16 row lanes of each output group (xor 1..8 stays inside the 16-lane group)
#pragma unroll
  for (int t = 0; t < 2; ++t)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      float v = dbl[t][i];
#pragma unroll
      for (int o = 1; o < 16; o <<= 1) v += __shfl_xor(v, o, 64);
      dbl[t][i] = v;
    }
  se = wave_sum(se);
  correct = wave_sum(correct);
  // Each wave stores its padded partial unconditionally (row stride WS_ROW: the 4 lane groups land in
  // distinct banks), one barrier, then every entry is the fixed-order sum w0 + w1 + w2 + w3
  // (deterministic; a first version added the waves in turns through guarded LDS read-modify-writes:
  // 4 barriers and 16 dependent LDS round trips per wave).
  float* ws = slab[w];
#pragma unroll
  for (int t = 0; t < 2; ++t)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      ws[(4 * g + i) * WS_ROW + 16 * t + c] = accW[t][i];   // C of accW[t]: [m = unit][n = output]
      if (c == 0) ws[WS_DB + 16 * t + 4 * g + i] = dbl[t][i];
    }
  if (lane == 0) {
    ws[WS_DB + 32] = se;
    ws[WS_DB + 33] = correct;
  }
  __syncthreads();
  float* out = a.part + (int64_t)blockIdx.x * PS;
  for (int i = threadIdx.x; i < PS; i += HW * 64) {
    const int pi = i < 16 * N ? (i / N) * WS_ROW + i % N : WS_DB + (i < 17 * N ? i - 16 * N : 32 + i - 17 * N);
    float v = slab[0][pi];
#pragma unroll
    for (int k = 1; k < HW; ++k) v += slab[k][pi];
    out[i] = v;
  }
}

// One workgroup per partial entry: thread k sums partials k, k + 256, ... in order, then a fixed-order
// LDS tree (deterministic).  dW / db go to grad[map[...]] (the dense slab layout [16][NP] dW then [NP]
// db), the metric sums to acc (this step's), out = acc / div, and the optimizer's step counter + 1.
// (A first version summed each entry with 4 threads over 64 partials: 21.7 us, latency-bound.)
__global__ __launch_bounds__(256) void head_fold_kernel(const float* __restrict__ part, int G, int N,
                                                        float* __restrict__ grad, const int* __restrict__ map,
                                                        float* __restrict__ acc, float* __restrict__ out, float div0,
                                                        float div1, int64_t* __restrict__ counter) {
  const int PS = 16 * N + N + 2;
  const int s = blockIdx.x;
  __shared__ float red[256];
  const int NP = N <= 16 ? 16 : 32;          // the dense slab's padded output width
  // the entry's gradient slot, loaded before the partials (after the tree it was one more round trip)
  int dst = -1;
  if (threadIdx.x == 0 && s < 17 * N) dst = s < 16 * N ? map[(s / N) * NP + s % N] : map[16 * NP + (s - 16 * N)];
  float v = 0.f;
  for (int gi = threadIdx.x; gi < G; gi += 256) v += part[(int64_t)gi * PS + s];
  red[threadIdx.x] = v;
  __syncthreads();
#pragma unroll
  for (int k = 128; k > 0; k >>= 1) {
    if (threadIdx.x < k) red[threadIdx.x] += red[threadIdx.x + k];
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    const float tot = red[0];
    if (s < 17 * N) {                          // dW[unit][output], then db[output]
      if (dst >= 0) grad[dst] = tot;
    } else {
      const int k = s - 17 * N;                // 0: sum of squared errors, 1: correct rows
      acc[k] = tot;
      if (out) out[k] = tot / (k == 0 ? div0 : div1);
      if (k == 0 && counter) counter[0] += 1;
    }
  }
}

int head_grid(int64_t n) {   // one 16-row tile per wave: every tile's loads in flight at once
  const int64_t ntile = (n + 15) / 16;
  return (int)std::max<int64_t>(1, (ntile + HW - 1) / HW);
}

}  // namespace

int lstm_head_partials(int64_t n, int N) { return head_grid(n) * (17 * N + 2); }

hipError_t lstm_head_launch(const void* h, int64_t ldh, const float* W, const float* b, const float* y, int64_t ldy,
                            void* dh, int64_t n, int N, float gscale, float* part, float* grad, const int* map,
                            float* acc, float* out, float div0, float div1, int64_t* counter, hipStream_t st) {
  if (n < 1 || N < 1 || N > 32) return hipErrorInvalidValue;
  const int G = head_grid(n);
  HeadArgs a{(const __bf16*)h, ldh, W, b, y, ldy, (__bf16*)dh, part, n, N, gscale};
  hipLaunchKernelGGL(lstm_head_kernel, dim3(G), dim3(HW * 64), 0, st, a);
  const int PS = 17 * N + 2;
  hipLaunchKernelGGL(head_fold_kernel, dim3(PS), dim3(256), 0, st, part, G, N, grad, map, acc, out, div0, div1,
                     counter);
  return hipGetLastError();
}

}  // namespace sml
