// Persistent Keras-granularity trainer for the reference LSTM stack.
//
// LSTM-TensorFlow-IO-Kafka/cardata-v2.py:172-209 trains
//     LSTM(32, relu, seq) -> LSTM(16, relu) -> RepeatVector(look_back)
//     -> LSTM(16, relu, seq) -> LSTM(32, relu, seq) -> TimeDistributed(Dense(18))
// with look_back = 1 and batch_size = 1: one Adam update per event, 1 000 steps x 5
// epochs.  As an autograd loop that is ~10 dependent launches of a few hundred FLOPs
// each per step.  Here ONE workgroup runs N consecutive Keras steps in one launch
// (the ae_minibatch.hip pattern): the live parameters sit in LDS for the whole launch,
// every thread owns a fixed set of (parameter, Adam m, Adam v) in registers and is the
// only writer of those parameters.
//
// Two kernels.  At batch 1 (the reference's setting, `lstm_ref_train_b1_kernel`, further
// down, with its own design note) wave 0 runs the chain of nine layers alone and waves
// 1..7 run Adam under it, synchronised by LDS counters: no workgroup barrier in the step
// loop.  For batches 2..32 (`lstm_ref_train_kernel`) each step is 10 barrier-separated
// phases:
//     F1-F4   LSTM layer forward  (task = (row, unit): three gate dot products, gate
//             math, c, h; i, g~, o, c saved for backward)
//     D0      head + loss          (wave per row: Dense(18), MSE gradient, loss and
//             argmax accuracy reduced across the wave)
//     D1-D4   LSTM layer backward  (dh from the layer above, gate gradients dz)
//     G       weight gradients + Adam, the next step's rows staged into LDS
//
// look_back = 1 (the reference's setting) makes every LSTM start from h0 = c0 = 0, so
// the recurrent kernels U and the forget-gate columns never receive a gradient: their
// Adam moments stay exactly 0 and Keras' update for them is exactly 0 (0 / (0 + eps)).
// The kernel therefore only carries the i, g, o columns of each W / b ("active"
// columns: 6 450 of the 18 642 parameters) and leaves U and the f columns untouched,
// which is bit-for-bit what Keras does.  The Python side checks the precondition
// (look_back == 1, inactive moments zero).
//
// fp32 everywhere (matches the fp32 torch oracle; the work per step is latency-, not
// throughput-bound, so bf16 MFMA tiles would buy nothing at batch 1).
#include <hip/hip_runtime.h>

#include <cstdint>

#include "sml_common.h"
#include "sml_ops.h"

namespace sml {
namespace {

constexpr int NT = 512;            // 8 waves: ~19 owned parameters per thread
constexpr int MAXB = 32;           // rows per Keras step (reference: 1)

__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// hardware exp / rcp (~1 ulp): the step is latency-bound and libm's accurate forms cost
// several times as many instructions on the serial phase chain
__device__ __forceinline__ float sigm(float z) { return sigmoid_fast(z); }
__device__ __forceinline__ float actf(int a, float z) { return a == 2 ? tanh_fast(z) : fmaxf(z, 0.0f); }
// derivative of the activation, from its OUTPUT value (relu: out > 0; tanh: 1 - out^2)
__device__ __forceinline__ float actd(int a, float out) { return a == 2 ? 1.0f - out * out : (out > 0.0f ? 1.0f : 0.0f); }

// Stack geometry (features F, LSTM units U1..U4) and the two layouts of the parameters.
template <int F_, int U1_, int U2_, int U3_, int U4_>
struct Geo {
  static constexpr int F = F_, U1 = U1_, U2 = U2_, U3 = U3_, U4 = U4_;
  // FlatParams order (models/lstm.py REFERENCE_STACK): W, U, b per LSTM; kernel, bias of the head
  static constexpr int gW1 = 0, gb1 = gW1 + F * 4 * U1 + U1 * 4 * U1;
  static constexpr int gW2 = gb1 + 4 * U1, gb2 = gW2 + U1 * 4 * U2 + U2 * 4 * U2;
  static constexpr int gW3 = gb2 + 4 * U2, gb3 = gW3 + U2 * 4 * U3 + U3 * 4 * U3;
  static constexpr int gW4 = gb3 + 4 * U3, gb4 = gW4 + U3 * 4 * U4 + U4 * 4 * U4;
  static constexpr int gK = gb4 + 4 * U4, gkb = gK + U4 * F;
  static constexpr int NPARAM = gkb + F;
  // LDS: active columns (i | g | o) of each W, odd row strides (conflict-free column and row walks)
  static constexpr int S1 = 3 * U1 + 1, S2 = 3 * U2 + 1, S3 = 3 * U3 + 1, S4 = 3 * U4 + 1, SK = F + 1;
  static constexpr int lW1 = 0, lb1 = lW1 + F * S1;
  static constexpr int lW2 = lb1 + 3 * U1, lb2 = lW2 + U1 * S2;
  static constexpr int lW3 = lb2 + 3 * U2, lb3 = lW3 + U2 * S3;
  static constexpr int lW4 = lb3 + 3 * U3, lb4 = lW4 + U3 * S4;
  static constexpr int lK = lb4 + 3 * U4, lkb = lK + U4 * SK;
  static constexpr int LPARAM = lkb + F;
  // activations (row strides odd)
  static constexpr int XS = F + 1, H1S = U1 + 1, H2S = U2 + 1, H3S = U3 + 1, H4S = U4 + 1;
  static constexpr int G1S = 4 * U1 + 1, G2S = 4 * U2 + 1, G3S = 4 * U3 + 1, G4S = 4 * U4 + 1;
  static constexpr int oX = LPARAM, oY = oX + 2 * MAXB * XS;
  static constexpr int oH1 = oY + 2 * MAXB * XS, oH2 = oH1 + MAXB * H1S, oH3 = oH2 + MAXB * H2S, oH4 = oH3 + MAXB * H3S;
  static constexpr int oG1 = oH4 + MAXB * H4S, oG2 = oG1 + MAXB * G1S, oG3 = oG2 + MAXB * G2S, oG4 = oG3 + MAXB * G3S;
  static constexpr int oZ1 = oG4 + MAXB * G4S, oZ2 = oZ1 + MAXB * S1, oZ3 = oZ2 + MAXB * S2, oZ4 = oZ3 + MAXB * S3;
  static constexpr int oDY = oZ4 + MAXB * S4, oST = oDY + MAXB * XS;
  static constexpr int LDS_FLOATS = oST + 2 * MAXB;
};
using Ref = Geo<18, 32, 16, 16, 32>;
static_assert(Ref::NPARAM == 18642, "reference stack parameter count (cardata-v2.py model.summary)");

struct RefArgs {
  float* flat;
  float* m;
  float* v;
  int64_t* iter;           // Keras Adam iteration counter (device), advanced by nsteps
  const float* x;          // sample rows (row i = input of sample i)
  const float* y;          // target rows
  int64_t ldx, ldy;        // row strides in floats
  const int32_t* order;    // optional sample permutation (nullptr = identity)
  int64_t nrows;           // samples available from row0 on
  int64_t row0;
  int B, nsteps, act;
  float lr, beta1, beta2, eps;
  float* out;              // [nsteps][2]: step loss (mean), correct rows
};

// ---- forward of one LSTM layer at t = 0 (h0 = c0 = 0): task = (row, unit) ----
template <int K, int U>
__device__ __forceinline__ void lstm_fwd(const float* __restrict__ W, const float* __restrict__ bias, int S,
                                         const float* __restrict__ in, int IS, float* __restrict__ h, int HS,
                                         float* __restrict__ gs, int GS, int Bs, int act) {
  for (int task = threadIdx.x; task < Bs * U; task += NT) {
    const int b = task / U, j = task - b * U;
    float zi = bias[j], zg = bias[U + j], zo = bias[2 * U + j];
    const float* xr = in + b * IS;
#pragma unroll
    for (int k = 0; k < K; ++k) {
      const float xv = xr[k];
      zi = fmaf(xv, W[k * S + j], zi);
      zg = fmaf(xv, W[k * S + U + j], zg);
      zo = fmaf(xv, W[k * S + 2 * U + j], zo);
    }
    const float ig = sigm(zi), gt = actf(act, zg), og = sigm(zo);
    const float c = ig * gt;
    const float ac = actf(act, c);
    h[b * HS + j] = og * ac;
    float* g = gs + b * GS;
    g[j] = ig;
    g[U + j] = gt;
    g[2 * U + j] = og;
    g[3 * U + j] = ac;
  }
}

// ---- backward of one LSTM layer: dh[b][j] = sum_n up[b][n] * Wup[j][n], then dz (i | g | o) ----
template <int U, int KN>
__device__ __forceinline__ void lstm_bwd(const float* __restrict__ up, int US, const float* __restrict__ Wup, int WS,
                                         const float* __restrict__ gs, int GS, float* __restrict__ dz, int ZS, int Bs,
                                         int act) {
  for (int task = threadIdx.x; task < Bs * U; task += NT) {
    const int b = task / U, j = task - b * U;
    const float* ur = up + b * US;
    const float* wr = Wup + j * WS;
    float d0 = 0.0f, d1 = 0.0f;
#pragma unroll
    for (int n = 0; n + 1 < KN; n += 2) {
      d0 = fmaf(ur[n], wr[n], d0);
      d1 = fmaf(ur[n + 1], wr[n + 1], d1);
    }
    if (KN & 1) d0 = fmaf(ur[KN - 1], wr[KN - 1], d0);
    const float dh = d0 + d1;
    const float* g = gs + b * GS;
    const float ig = g[j], gt = g[U + j], og = g[2 * U + j], ac = g[3 * U + j];
    const float dc = dh * og * actd(act, ac);
    float* z = dz + b * ZS;
    z[j] = dc * gt * ig * (1.0f - ig);             // input gate
    z[U + j] = dc * ig * actd(act, gt);            // candidate
    z[2 * U + j] = dh * ac * og * (1.0f - og);     // output gate
  }
}

// ---- per-thread parameter ownership: item idx = threadIdx.x + r * NT of each block ----
enum { OWN_LOAD = 0, OWN_STEP = 1, OWN_STORE = 2 };

// One parameter block.  NA = active columns, GATE: LSTM W / b (active column n -> gate
// column n < U ? n : n + U of the 4U-wide Keras kernel), else the Dense head.  BIAS:
// the block is a bias vector (gradient = column sum of dz).
template <int MODE, int SIZE, int NA, bool GATE, bool BIAS, int R0, int R>
__device__ __forceinline__ void own_block(float (&p)[R], float (&mo)[R], float (&vo)[R], const RefArgs& a, int gofs,
                                          int gcols, float* lw, int LS, const float* in, int IS, const float* dz, int ZS,
                                          int Bs, float lr_t) {
  constexpr int N = (SIZE + NT - 1) / NT;
  static_assert(R0 + N <= R, "ownership register budget");
  // opaque copy of the thread id: keeps the compiler from hoisting the ~30 per-item LDS
  // addresses out of the step loop (they would pin ~90 VGPRs for the whole launch)
  int tid = threadIdx.x;
  asm volatile("" : "+v"(tid));
#pragma unroll
  for (int r = 0; r < N; ++r) {
    const int idx = tid + r * NT;
    if (idx < SIZE) {
      const int k = BIAS ? 0 : idx / NA, n = BIAS ? idx : idx - (idx / NA) * NA;
      float* lp = lw + k * LS + n;
      if (MODE == OWN_LOAD || MODE == OWN_STORE) {
        const int U = NA / 3;
        const int col = GATE ? (n < U ? n : n + U) : n;
        const int64_t g = gofs + (int64_t)k * gcols + col;
        if (MODE == OWN_LOAD) {
          p[R0 + r] = a.flat[g];
          mo[R0 + r] = a.m[g];
          vo[R0 + r] = a.v[g];
          *lp = p[R0 + r];
        } else {
          a.flat[g] = p[R0 + r];
          a.m[g] = mo[R0 + r];
          a.v[g] = vo[R0 + r];
        }
      } else {
        float gr = 0.0f;
        for (int b = 0; b < Bs; ++b) gr = fmaf(BIAS ? 1.0f : in[b * IS + k], dz[b * ZS + n], gr);
        const float mm = a.beta1 * mo[R0 + r] + (1.0f - a.beta1) * gr;
        const float vv = a.beta2 * vo[R0 + r] + (1.0f - a.beta2) * gr * gr;
        mo[R0 + r] = mm;
        vo[R0 + r] = vv;
        p[R0 + r] -= lr_t * mm * __builtin_amdgcn_rcpf(__builtin_amdgcn_sqrtf(vv) + a.eps);   // v_sqrt / v_rcp
        *lp = p[R0 + r];
      }
    }
  }
}

template <int SZ>
constexpr int nown() { return (SZ + NT - 1) / NT; }

template <int MODE, typename G, int R>
__device__ __forceinline__ void own_all(float (&p)[R], float (&mo)[R], float (&vo)[R], const RefArgs& a, float* L,
                                        const float* xb, int Bs, float lr_t) {
  constexpr int r0 = 0, r1 = r0 + nown<G::F * 3 * G::U1>(), r2 = r1 + nown<3 * G::U1>();
  constexpr int r3 = r2 + nown<G::U1 * 3 * G::U2>(), r4 = r3 + nown<3 * G::U2>();
  constexpr int r5 = r4 + nown<G::U2 * 3 * G::U3>(), r6 = r5 + nown<3 * G::U3>();
  constexpr int r7 = r6 + nown<G::U3 * 3 * G::U4>(), r8 = r7 + nown<3 * G::U4>();
  constexpr int r9 = r8 + nown<G::U4 * G::F>();
  own_block<MODE, G::F * 3 * G::U1, 3 * G::U1, true, false, r0>(p, mo, vo, a, G::gW1, 4 * G::U1, L + G::lW1, G::S1, xb,
                                                                 G::XS, L + G::oZ1, G::S1, Bs, lr_t);
  own_block<MODE, 3 * G::U1, 3 * G::U1, true, true, r1>(p, mo, vo, a, G::gb1, 0, L + G::lb1, 0, nullptr, 0, L + G::oZ1,
                                                         G::S1, Bs, lr_t);
  own_block<MODE, G::U1 * 3 * G::U2, 3 * G::U2, true, false, r2>(p, mo, vo, a, G::gW2, 4 * G::U2, L + G::lW2, G::S2,
                                                                  L + G::oH1, G::H1S, L + G::oZ2, G::S2, Bs, lr_t);
  own_block<MODE, 3 * G::U2, 3 * G::U2, true, true, r3>(p, mo, vo, a, G::gb2, 0, L + G::lb2, 0, nullptr, 0, L + G::oZ2,
                                                         G::S2, Bs, lr_t);
  own_block<MODE, G::U2 * 3 * G::U3, 3 * G::U3, true, false, r4>(p, mo, vo, a, G::gW3, 4 * G::U3, L + G::lW3, G::S3,
                                                                  L + G::oH2, G::H2S, L + G::oZ3, G::S3, Bs, lr_t);
  own_block<MODE, 3 * G::U3, 3 * G::U3, true, true, r5>(p, mo, vo, a, G::gb3, 0, L + G::lb3, 0, nullptr, 0, L + G::oZ3,
                                                         G::S3, Bs, lr_t);
  own_block<MODE, G::U3 * 3 * G::U4, 3 * G::U4, true, false, r6>(p, mo, vo, a, G::gW4, 4 * G::U4, L + G::lW4, G::S4,
                                                                  L + G::oH3, G::H3S, L + G::oZ4, G::S4, Bs, lr_t);
  own_block<MODE, 3 * G::U4, 3 * G::U4, true, true, r7>(p, mo, vo, a, G::gb4, 0, L + G::lb4, 0, nullptr, 0, L + G::oZ4,
                                                         G::S4, Bs, lr_t);
  own_block<MODE, G::U4 * G::F, G::F, false, false, r8>(p, mo, vo, a, G::gK, G::F, L + G::lK, G::SK, L + G::oH4,
                                                         G::H4S, L + G::oDY, G::XS, Bs, lr_t);
  own_block<MODE, G::F, G::F, false, true, r9>(p, mo, vo, a, G::gkb, 0, L + G::lkb, 0, nullptr, 0, L + G::oDY, G::XS,
                                               Bs, lr_t);
}

template <typename G>
constexpr int own_regs() {
  return nown<G::F * 3 * G::U1>() + nown<3 * G::U1>() + nown<G::U1 * 3 * G::U2>() + nown<3 * G::U2>() +
         nown<G::U2 * 3 * G::U3>() + nown<3 * G::U3>() + nown<G::U3 * 3 * G::U4>() + nown<3 * G::U4>() +
         nown<G::U4 * G::F>() + nown<G::F>();
}

template <typename G>
__device__ __forceinline__ void stage_rows(const RefArgs& a, float* L, int par, int64_t r0, int Bs) {
  float* xs = L + G::oX + par * MAXB * G::XS;
  float* ys = L + G::oY + par * MAXB * G::XS;
  for (int t = threadIdx.x; t < Bs * G::F; t += NT) {
    const int b = t / G::F, f = t - b * G::F;
    const int64_t i = r0 + b;
    const int64_t s = a.order ? (int64_t)a.order[i] : i;
    xs[b * G::XS + f] = a.x[s * a.ldx + f];
    ys[b * G::XS + f] = a.y[s * a.ldy + f];
  }
}

template <typename G>
__global__ __launch_bounds__(NT) void lstm_ref_train_kernel(RefArgs a) {
  extern __shared__ __attribute__((aligned(16))) float L[];
  constexpr int R = own_regs<G>();
  float p[R], mo[R], vo[R];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int64_t it0 = *a.iter;
  own_all<OWN_LOAD, G>(p, mo, vo, a, L, nullptr, 0, 0.0f);
  const int64_t total = a.nrows - a.row0;
  int Bs = (int)(total < a.B ? total : a.B);
  stage_rows<G>(a, L, 0, a.row0, Bs);
  double b1t = pow((double)a.beta1, (double)it0), b2t = pow((double)a.beta2, (double)it0);
  lds_barrier();
  int s = 0;
  for (; s < a.nsteps && Bs > 0; ++s) {
    const int par = s & 1;
    const float* xb = L + G::oX + par * MAXB * G::XS;
    const float* yb = L + G::oY + par * MAXB * G::XS;
    // ---- forward ----
    lstm_fwd<G::F, G::U1>(L + G::lW1, L + G::lb1, G::S1, xb, G::XS, L + G::oH1, G::H1S, L + G::oG1, G::G1S, Bs, a.act);
    lds_barrier();
    lstm_fwd<G::U1, G::U2>(L + G::lW2, L + G::lb2, G::S2, L + G::oH1, G::H1S, L + G::oH2, G::H2S, L + G::oG2, G::G2S, Bs,
                           a.act);
    lds_barrier();
    // RepeatVector(1) is the identity at look_back = 1
    lstm_fwd<G::U2, G::U3>(L + G::lW3, L + G::lb3, G::S3, L + G::oH2, G::H2S, L + G::oH3, G::H3S, L + G::oG3, G::G3S, Bs,
                           a.act);
    lds_barrier();
    lstm_fwd<G::U3, G::U4>(L + G::lW4, L + G::lb4, G::S4, L + G::oH3, G::H3S, L + G::oH4, G::H4S, L + G::oG4, G::G4S, Bs,
                           a.act);
    lds_barrier();
    // ---- D0: TimeDistributed(Dense(F)) + MSE + accuracy, one wave per row ----
    const float gs = 2.0f / (float)(Bs * G::F);   // Keras MSE: mean over rows x features
    for (int b = wave; b < Bs; b += NT / 64) {
      float yp = -3.402823466e38f, yt = -3.402823466e38f, d2 = 0.0f;
      if (lane < G::F) {
        float acc = L[G::lkb + lane];
        const float* hr = L + G::oH4 + b * G::H4S;
#pragma unroll
        for (int k = 0; k < G::U4; ++k) acc = fmaf(hr[k], L[G::lK + k * G::SK + lane], acc);
        yp = acc;
        yt = yb[b * G::XS + lane];
        const float d = yp - yt;
        d2 = d * d;
        L[G::oDY + b * G::XS + lane] = gs * d;
      }
      // argmax (first index on ties, as torch / numpy) of prediction and target
      int ip = lane < G::F ? lane : 1 << 20, it = ip;
      float vp = yp, vt = yt;
#pragma unroll
      for (int o = 32; o >= 1; o >>= 1) {
        const float op = __shfl_xor(vp, o), ot = __shfl_xor(vt, o);
        const int jp = __shfl_xor(ip, o), jt = __shfl_xor(it, o);
        if (op > vp || (op == vp && jp < ip)) { vp = op; ip = jp; }
        if (ot > vt || (ot == vt && jt < it)) { vt = ot; it = jt; }
        d2 += __shfl_xor(d2, o);
      }
      if (lane == 0) {
        L[G::oST + 2 * b] = d2;
        L[G::oST + 2 * b + 1] = ip == it ? 1.0f : 0.0f;
      }
    }
    lds_barrier();
    // ---- backward ----
    lstm_bwd<G::U4, G::F>(L + G::oDY, G::XS, L + G::lK, G::SK, L + G::oG4, G::G4S, L + G::oZ4, G::S4, Bs, a.act);
    lds_barrier();
    lstm_bwd<G::U3, 3 * G::U4>(L + G::oZ4, G::S4, L + G::lW4, G::S4, L + G::oG3, G::G3S, L + G::oZ3, G::S3, Bs, a.act);
    lds_barrier();
    lstm_bwd<G::U2, 3 * G::U3>(L + G::oZ3, G::S3, L + G::lW3, G::S3, L + G::oG2, G::G2S, L + G::oZ2, G::S2, Bs, a.act);
    lds_barrier();
    lstm_bwd<G::U1, 3 * G::U2>(L + G::oZ2, G::S2, L + G::lW2, G::S2, L + G::oG1, G::G1S, L + G::oZ1, G::S1, Bs, a.act);
    lds_barrier();
    // ---- G: weight gradients + Adam; stage the next step's rows ----
    b1t *= (double)a.beta1;
    b2t *= (double)a.beta2;
    const float lr_t = (float)((double)a.lr * sqrt(1.0 - b2t) / (1.0 - b1t));
    own_all<OWN_STEP, G>(p, mo, vo, a, L, xb, Bs, lr_t);
    if (threadIdx.x == 0) {
      float ls = 0.0f, cr = 0.0f;
      for (int b = 0; b < Bs; ++b) {
        ls += L[G::oST + 2 * b];
        cr += L[G::oST + 2 * b + 1];
      }
      a.out[2 * s] = ls / (float)(Bs * G::F);
      a.out[2 * s + 1] = cr;
    }
    const int64_t rn = a.row0 + (int64_t)(s + 1) * a.B;
    const int64_t left = a.nrows - rn;
    const int Bn = (int)(left < a.B ? (left > 0 ? left : 0) : a.B);
    if (s + 1 < a.nsteps && Bn > 0) stage_rows<G>(a, L, par ^ 1, rn, Bn);
    Bs = Bn;
    lds_barrier();
  }
  own_all<OWN_STORE, G>(p, mo, vo, a, L, nullptr, 0, 0.0f);
  if (threadIdx.x == 0) *a.iter = it0 + s;
}

// ===================================================================================
// Batch-1 path (the reference's setting, `lstm_ref_train_b1_kernel`).
//
// Chain.  At B = 1 no layer has more than 32 unit tasks, so the whole forward + backward
// chain of a step runs on wave 0 alone, with NO workgroup barrier inside it.  Lane
// l = j + U * part works on unit j of a U-unit layer and on every P-th input (P = 64 / U);
// the P partial dot products meet through permlane swaps.  A wave's LDS operations
// complete in order, so a value one lane writes is seen by every lane of the same wave
// that reads it afterwards.  The gates a lane computes in the forward pass stay in its
// registers for the backward pass of the same layer (same j mapping).
//   * Weights come from per-lane IMAGES: for every layer each lane finds exactly the
//     weights it multiplies, slot-major (slot s of lane l at s * 64 + l, backward slots in
//     padded, shifted rows -- B1::img; conflict-free,
//     paired into ds_read2st64).  A weight has a forward image (the lane that uses it in
//     its layer's dot product) and, for W2..W4 and the head kernel, a backward image (the
//     lane that uses it in dh of the layer below).  A layer's image is requested one
//     layer ahead, so its latency hides under the current layer's math.
//   * Activations pass between layers through LDS, each written twice: in natural order
//     (the weight gradients read it) and part-major for the consuming layer (each part's
//     inputs contiguous: 16-byte reads).
// Adam, pipelined against the next step's chain.  Wave 0 runs only the chain; waves 1..7
// run Adam.  Thread t' = t - 64 owns column n = t' % NA of a weight block and rows
// k = t' / NA + R * i, with R a multiple of the forward split P, so every image address
// is a per-block base plus a compile-time offset; (p, m, v) stay in its registers and the
// new value goes into both images.  The chain counts its stages in an LDS counter (head,
// D4, D3, D2, D1 of every step), and the Adam waves take the blocks in REVERSE order,
// each as soon as its gradient exists and the chain has read that block's old backward
// image: head after the head layer, W4 after D4, W3 after D3, W2 after D2, W1 after D1.
// So Adam of step s runs under the backward half of the chain of step s, and only W1's
// update sits between the end of one chain and the start of the next (the chain waits on
// a counter of finished W1 blocks before it reads any image).  No workgroup barrier
// remains in the loop.  The activations Adam reads (natural-order h, dz) are double-
// buffered by step
// parity.  A wave's LDS operations complete in order, so "write the images, then bump
// the counter" needs no fence beyond keeping the compiler from reordering them.
// Off the critical path:
//   * the lightest Adam wave computes the loss / argmax accuracy of the step it just
//     updated (from its saved prediction row);
//   * the sample rows arrive 32 steps ahead by asynchronous global -> LDS copies that
//     wave 0 issues and waits for.
// ===================================================================================
constexpr int NB = MAXB;          // steps per prefetched row block
constexpr int NADAM = NT - 64;    // Adam threads (waves 1..7)

constexpr int c4(int v) { return (v + 3) & ~3; }

template <typename G>
struct B1 {
  static constexpr int F = G::F, U1 = G::U1, U2 = G::U2, U3 = G::U3, U4 = G::U4;
  static constexpr int P1 = 64 / U1, P2 = 64 / U2, P3 = 64 / U3, P4 = 64 / U4, PH = 2;
  // inputs per lane (per part) of each chain layer
  static constexpr int KF1 = F / P1, KF2 = U1 / P2, KF3 = U2 / P3, KF4 = U3 / P4, KHD = U4 / PH;
  static constexpr int KB4 = F / P4, KB3 = 3 * U4 / P3, KB2 = 3 * U3 / P2, KB1 = 3 * U2 / P1;
  static_assert(F % P1 == 0 && U1 % P2 == 0 && U2 % P3 == 0 && U3 % P4 == 0 && U4 % PH == 0 && F % P4 == 0 &&
                    (3 * U4) % P3 == 0 && (3 * U3) % P2 == 0 && (3 * U2) % P1 == 0 && F <= 32,
                "even lane splits");
  // image segments (slots per lane): forward = 3 gates x inputs + 3 bias slots (part 0 only)
  static constexpr int sF1 = 0, sF2 = sF1 + 3 * KF1 + 3, sF3 = sF2 + 3 * KF2 + 3, sF4 = sF3 + 3 * KF3 + 3;
  static constexpr int sHD = sF4 + 3 * KF4 + 3, sB4 = sHD + KHD + 1, sB3 = sB4 + KB4, sB2 = sB3 + KB3;
  static constexpr int sB1 = sB2 + KB2, NSLOT = sB1 + KB1;
  // The backward images (slots sB4 .. NSLOT) are written by Adam threads whose lanes walk
  // the OTHER index (lane' = k + K * (n % P') with n running across the wave): in a plain
  // 64-float slot row those writes fall on 2-4 banks.  Each backward slot row is therefore
  // BROW floats long and shifted by (slot & 31): a lane's address stays slot-affine (the
  // chain's reads keep compile-time offsets), and Adam's writes spread over the banks.
  static constexpr int BROW = 96;
  static constexpr int NSLOTF = sB4;                               // forward slots, 64-float rows
  static constexpr int IMG_FLOATS = NSLOTF * 64 + (NSLOT - NSLOTF) * BROW;
  // float offset of (slot, lane) in the images
  static constexpr __host__ __device__ int img(int slot, int lane) {
    return slot < NSLOTF ? slot * 64 + lane : NSLOTF * 64 + (slot - NSLOTF) * BROW + ((slot - NSLOTF) & 31) + lane;
  }
  // natural-order activations of one step (Adam's inputs), double-buffered by step parity
  static constexpr int nH1 = 0, nH2 = nH1 + U1, nH3 = nH2 + U2, nH4 = nH3 + U3;
  static constexpr int nZ1 = nH4 + U4, nZ2 = nZ1 + 3 * U1, nZ3 = nZ2 + 3 * U2, nZ4 = nZ3 + 3 * U3;
  static constexpr int nDY = nZ4 + 3 * U4, NATS = c4(nDY + F);
  // LDS map (floats)
  static constexpr int oROW = IMG_FLOATS;                        // 2 blocks x [NB x rows | NB y rows]
  static constexpr int oNAT = oROW + 4 * NB * F;                 // 2 x NATS
  // part-major copies for the consuming layer (each part's run 16-byte aligned)
  static constexpr int qH1 = oNAT + 2 * NATS, qH2 = qH1 + P2 * c4(KF2), qH3 = qH2 + P3 * c4(KF3);
  static constexpr int qH4 = qH3 + P4 * c4(KF4), qDY = qH4 + PH * c4(KHD), qZ4 = qDY + P4 * c4(KB4);
  static constexpr int qZ3 = qZ4 + P3 * c4(KB3), qZ2 = qZ3 + P2 * c4(KB2);
  static constexpr int oYP = qZ2 + P1 * c4(KB1);                 // [2][F] predictions
  static constexpr int oCNT = c4(oYP + 2 * F);                    // counters: [0..4] Adam blocks, [5] chain
  static constexpr int oSINK = oCNT + 8;                          // per-lane sink for writes a lane must not make
  static constexpr int LDS_FLOATS = oSINK + 64;
  // Adam ownership over the NADAM threads of waves 1..7: rows per pass R (a multiple of the
  // forward split), items per thread N; register pairs per block from r*
  static constexpr int rpass(int na, int p) { return (NADAM / na) / p * p; }
  static constexpr int R1 = rpass(3 * U1, P1), R2 = rpass(3 * U2, P2), R3 = rpass(3 * U3, P3);
  static constexpr int R4 = rpass(3 * U4, P4), RK = rpass(F, PH);
  static constexpr int N1 = (F + R1 - 1) / R1, N2 = (U1 + R2 - 1) / R2, N3 = (U2 + R3 - 1) / R3;
  static constexpr int N4 = (U3 + R4 - 1) / R4, NK = (U4 + RK - 1) / RK;
  static constexpr int r1 = 0, r2 = r1 + (N1 + 1) / 2, r3 = r2 + (N2 + 1) / 2, r4 = r3 + (N3 + 1) / 2;
  static constexpr int rK = r4 + (N4 + 1) / 2, NOWN2 = rK + (NK + 1) / 2;
  static_assert(R1 > 0 && R2 > 0 && R3 > 0 && R4 > 0 && RK > 0, "ownership split");
  static_assert(3 * (U1 + U2 + U3 + U4) + F <= NADAM, "one bias per thread");
  // the W blocks keep R * 3U = 384 of the 448 threads busy; rotated so the idle wave is
  // wave 4, which shares a SIMD with the chain wave under round-robin placement
  static constexpr int WROT = 3 * 64;
};

__device__ __forceinline__ void wave_order() { asm volatile("" ::: "memory"); }

// LDS counters between the chain wave and the Adam waves
__device__ __forceinline__ unsigned cnt_ld(const float* L, int i) {
  return __hip_atomic_load(reinterpret_cast<const unsigned*>(L) + i, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void cnt_wait(const float* L, int i, unsigned target) {
  while (cnt_ld(L, i) < target) __builtin_amdgcn_s_sleep(0);
}
// one lane bumps the counter after the wave's LDS writes (in-order LDS: no fence needed)
__device__ __forceinline__ void cnt_bump(float* L, int i, int lane) {
  wave_order();
  if (lane == 0)
    __hip_atomic_fetch_add(reinterpret_cast<unsigned*>(L) + i, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

// sum of a lane value over the P = 64 / U lane groups of lane = j + U * part
template <int U>
__device__ __forceinline__ float part_sum(float v, int lane) {
  static_assert(U == 16 || U == 32, "chain layouts");
  if (U == 16) v += xor16(v, lane);
  return v + xor32(v, lane);
}

// N consecutive image slots of this lane from slot S0 (slot-major; Bq::img places them)
template <typename Bq, int S0, int N>
__device__ __forceinline__ void img_rd(const float* L, int lane, float (&w)[N]) {
  const float* b = L + lane;
#pragma unroll
  for (int i = 0; i < N; ++i) w[i] = b[Bq::img(S0 + i, 0)];
}
// N floats (N % 4 == 0) of a 16-byte aligned LDS run
template <int N>
__device__ __forceinline__ void vec_rd(const float* v, float (&o)[N]) {
  static_assert(N % 4 == 0, "whole 16-byte reads");
#pragma unroll
  for (int i = 0; i < N; i += 4) {
    const float4 t = *reinterpret_cast<const float4*>(v + i);
    o[i] = t.x;
    o[i + 1] = t.y;
    o[i + 2] = t.z;
    o[i + 3] = t.w;
  }
}

// position of element e of a vector in its consumer's part-major copy (PC parts of KPC)
template <int PC, int KPC>
__device__ __forceinline__ int qpos(int e) { return (e % PC) * c4(KPC) + e / PC; }

template <int ACT>
__device__ __forceinline__ float act_f(float z) { return ACT == 2 ? tanh_fast(z) : fmaxf(z, 0.0f); }
template <int ACT>
__device__ __forceinline__ float act_d(float out) { return ACT == 2 ? 1.0f - out * out : (out > 0.0f ? 1.0f : 0.0f); }

// forward of one LSTM unit from this lane's image (3 gates x KP inputs + bias slots)
template <int KP, int U, int ACT, int NW, int NI>
__device__ __forceinline__ float fwd_unit(const float (&w)[NW], const float (&in)[NI], int lane, float& ig, float& gt,
                                          float& og, float& ac) {
  static_assert(NW == 3 * KP + 3 && NI >= KP, "image / input shapes");
  float zi = w[3 * KP], zg = w[3 * KP + 1], zo = w[3 * KP + 2];
#pragma unroll
  for (int i = 0; i < KP; ++i) {
    zi = fmaf(in[i], w[3 * i], zi);
    zg = fmaf(in[i], w[3 * i + 1], zg);
    zo = fmaf(in[i], w[3 * i + 2], zo);
  }
  zi = part_sum<U>(zi, lane);
  zg = part_sum<U>(zg, lane);
  zo = part_sum<U>(zo, lane);
  ig = sigm(zi);
  gt = act_f<ACT>(zg);
  og = sigm(zo);
  ac = act_f<ACT>(ig * gt);
  return og * ac;
}

// dh of one unit: this lane's image row . its inputs from the layer above
template <int KP, int U, int NI>
__device__ __forceinline__ float bwd_dh(const float (&w)[KP], const float (&up)[NI], int lane) {
  static_assert(NI >= KP, "input shape");
  float d0 = 0.0f, d1 = 0.0f;
#pragma unroll
  for (int i = 0; i + 1 < KP; i += 2) {
    d0 = fmaf(up[i], w[i], d0);
    d1 = fmaf(up[i + 1], w[i + 1], d1);
  }
  if (KP & 1) d0 = fmaf(up[KP - 1], w[KP - 1], d0);
  return part_sum<U>(d0 + d1, lane);
}

// h of a forward layer: part 0 -> natural order, part 1 -> the consumer's copy, rest -> sink
template <typename Bq, int PC, int KPC>
__device__ __forceinline__ void put_h(float* L, int nat, int q, int j, int part, int lane, float h) {
  L[part == 0 ? nat + j : (part == 1 ? q + qpos<PC, KPC>(j) : Bq::oSINK + lane)] = h;
  wave_order();
}

// dz (i | g | o) of unit j: part 0 -> natural, part 1 -> the consumer's copy (QZ), rest -> sink
template <typename Bq, int U, int PC, int KPC, bool QZ>
__device__ __forceinline__ void put_dz(float* L, int nat, int q, int j, int part, int lane, float zi, float zg,
                                       float zo) {
  const int sink = Bq::oSINK + lane;
  L[part == 0 ? nat + j : (part == 1 && QZ ? q + qpos<PC, KPC>(j) : sink)] = zi;
  L[part == 0 ? nat + U + j : (part == 1 && QZ ? q + qpos<PC, KPC>(U + j) : sink)] = zg;
  L[part == 0 ? nat + 2 * U + j : (part == 1 && QZ ? q + qpos<PC, KPC>(2 * U + j) : sink)] = zo;
  wave_order();
}

// gate gradients of one unit from dh and the saved forward gates
template <int ACT>
__device__ __forceinline__ void dz_unit(float dh, float ig, float gt, float og, float ac, float& zi, float& zg,
                                        float& zo) {
  const float dc = dh * og * act_d<ACT>(ac);
  zi = dc * gt * ig * (1.0f - ig);
  zg = dc * ig * act_d<ACT>(gt);
  zo = dh * ac * og * (1.0f - og);
}

#ifdef SML_LREF_PROBE
// the phase probe's clock marks (the kernel and the chain share pc / tq / tn)
#define SML_PROBE_MARK(i) (tn = clock64(), pc[i] += tn - tq, tq = tn)
#define SML_PROBE_ARGS , unsigned long long (&pc)[4], unsigned long long &tq, unsigned long long &tn
#define SML_PROBE_PASS , pc, tq, tn
#else
#define SML_PROBE_MARK(i) ((void)0)
#define SML_PROBE_ARGS
#define SML_PROBE_PASS
#endif

// the whole chain of Keras step s at B = 1 (wave 0)
template <typename G, int ACT>
__device__ __forceinline__ void chain_step(float* L, const float* xb, const float* yb, int nat, float* yp_out,
                                           unsigned step, int lane SML_PROBE_ARGS) {
  using Q = B1<G>;
  const int j1 = lane % G::U1, p1 = lane / G::U1, j2 = lane % G::U2, p2 = lane / G::U2;
  const int j3 = lane % G::U3, p3 = lane / G::U3, j4 = lane % G::U4, p4 = lane / G::U4;
  float i1, g1, o1, a1, i2, g2, o2, a2, i3, g3, o3, a3, i4, g4, o4, a4, h;
  float x[Q::KF1];
#pragma unroll
  for (int i = 0; i < Q::KF1; ++i) x[i] = xb[p1 + Q::P1 * i];
  float w1[3 * Q::KF1 + 3], w2[3 * Q::KF2 + 3];
  cnt_wait(L, Q::oCNT + 0, 7u * step);   // every Adam wave has applied step s - 1 (W1 is its last block)
  SML_PROBE_MARK(1);
  img_rd<Q, Q::sF1>(L, lane, w1);
  img_rd<Q, Q::sF2>(L, lane, w2);
  h = fwd_unit<Q::KF1, G::U1, ACT>(w1, x, lane, i1, g1, o1, a1);
  put_h<Q, Q::P2, Q::KF2>(L, nat + Q::nH1, Q::qH1, j1, p1, lane, h);

  float w3[3 * Q::KF3 + 3], in2[c4(Q::KF2)];
  img_rd<Q, Q::sF3>(L, lane, w3);
  vec_rd(L + Q::qH1 + p2 * c4(Q::KF2), in2);
  h = fwd_unit<Q::KF2, G::U2, ACT>(w2, in2, lane, i2, g2, o2, a2);
  put_h<Q, Q::P3, Q::KF3>(L, nat + Q::nH2, Q::qH2, j2, p2, lane, h);

  float w4[3 * Q::KF4 + 3], in3[c4(Q::KF3)];
  img_rd<Q, Q::sF4>(L, lane, w4);
  vec_rd(L + Q::qH2 + p3 * c4(Q::KF3), in3);
  h = fwd_unit<Q::KF3, G::U3, ACT>(w3, in3, lane, i3, g3, o3, a3);
  put_h<Q, Q::P4, Q::KF4>(L, nat + Q::nH3, Q::qH3, j3, p3, lane, h);

  float wh[Q::KHD + 1], in4[c4(Q::KF4)];
  img_rd<Q, Q::sHD>(L, lane, wh);
  vec_rd(L + Q::qH3 + p4 * c4(Q::KF4), in4);
  h = fwd_unit<Q::KF4, G::U4, ACT>(w4, in4, lane, i4, g4, o4, a4);
  put_h<Q, Q::PH, Q::KHD>(L, nat + Q::nH4, Q::qH4, j4, p4, lane, h);

  float wb4[Q::KB4];
  img_rd<Q, Q::sB4>(L, lane, wb4);
  {  // TimeDistributed(Dense(F)) + the MSE gradient: lane = f + 32 * part
    const int f = lane & 31, ph = lane >> 5, fc = f < G::F ? f : G::F - 1;
    float inh[c4(Q::KHD)];
    vec_rd(L + Q::qH4 + ph * c4(Q::KHD), inh);
    float acc = wh[Q::KHD];
#pragma unroll
    for (int i = 0; i < Q::KHD; ++i) acc = fmaf(inh[i], wh[i], acc);
    const float yp = acc + xor32(acc, lane);
    const float dy = (2.0f / (float)G::F) * (yp - yb[fc]);   // Keras MSE: mean over features
    const int sink = Q::oSINK + lane;
    L[f >= G::F ? sink : (ph == 0 ? nat + Q::nDY + f : Q::qDY + qpos<Q::P4, Q::KB4>(f))] = dy;
    L[f < G::F && ph == 0 ? (int)(yp_out - L) + f : sink] = yp;
    wave_order();
  }
  // stage 1: dY, h4 and the prediction are out and the head's backward image is read (wb4)
  cnt_bump(L, Q::oCNT + 5, lane);
  float wb3[Q::KB3], up4[c4(Q::KB4)], zi, zg, zo;
  img_rd<Q, Q::sB3>(L, lane, wb3);
  vec_rd(L + Q::qDY + p4 * c4(Q::KB4), up4);
  dz_unit<ACT>(bwd_dh<Q::KB4, G::U4>(wb4, up4, lane), i4, g4, o4, a4, zi, zg, zo);
  put_dz<Q, G::U4, Q::P3, Q::KB3, true>(L, nat + Q::nZ4, Q::qZ4, j4, p4, lane, zi, zg, zo);
  cnt_bump(L, Q::oCNT + 5, lane);   // stage: dz and the next layer's backward image read

  float wb2[Q::KB2], up3[c4(Q::KB3)];
  img_rd<Q, Q::sB2>(L, lane, wb2);
  vec_rd(L + Q::qZ4 + p3 * c4(Q::KB3), up3);
  dz_unit<ACT>(bwd_dh<Q::KB3, G::U3>(wb3, up3, lane), i3, g3, o3, a3, zi, zg, zo);
  put_dz<Q, G::U3, Q::P2, Q::KB2, true>(L, nat + Q::nZ3, Q::qZ3, j3, p3, lane, zi, zg, zo);
  cnt_bump(L, Q::oCNT + 5, lane);   // stage: dz and the next layer's backward image read

  float wb1[Q::KB1], up2[c4(Q::KB2)];
  img_rd<Q, Q::sB1>(L, lane, wb1);
  vec_rd(L + Q::qZ3 + p2 * c4(Q::KB2), up2);
  dz_unit<ACT>(bwd_dh<Q::KB2, G::U2>(wb2, up2, lane), i2, g2, o2, a2, zi, zg, zo);
  put_dz<Q, G::U2, Q::P1, Q::KB1, true>(L, nat + Q::nZ2, Q::qZ2, j2, p2, lane, zi, zg, zo);
  cnt_bump(L, Q::oCNT + 5, lane);   // stage: dz and the next layer's backward image read

  float up1[c4(Q::KB1)];
  vec_rd(L + Q::qZ2 + p1 * c4(Q::KB1), up1);
  dz_unit<ACT>(bwd_dh<Q::KB1, G::U1>(wb1, up1, lane), i1, g1, o1, a1, zi, zg, zo);
  put_dz<Q, G::U1, 1, 1, false>(L, nat + Q::nZ1, 0, j1, p1, lane, zi, zg, zo);
  cnt_bump(L, Q::oCNT + 5, lane);   // stage 5: the chain of this step is complete
}

// loss and argmax accuracy of one step from its saved prediction and target rows (one wave)
template <typename G>
__device__ __forceinline__ void step_stats(const float* yp, const float* yt, float* out, int lane) {
  float vp = -3.402823466e38f, vt = -3.402823466e38f, d2 = 0.0f;
  int ip = lane < G::F ? lane : 1 << 20, it = ip;
  if (lane < G::F) {
    vp = yp[lane];
    vt = yt[lane];
    const float d = vp - vt;
    d2 = d * d;
  }
#pragma unroll
  for (int o = 16; o >= 1; o >>= 1) {   // F <= 32: the first half-wave holds every feature
    const float op = __shfl_xor(vp, o), ot = __shfl_xor(vt, o);
    const int jp = __shfl_xor(ip, o), jt = __shfl_xor(it, o);
    if (op > vp || (op == vp && jp < ip)) { vp = op; ip = jp; }
    if (ot > vt || (ot == vt && jt < it)) { vt = ot; it = jt; }
    d2 += __shfl_xor(d2, o);
  }
  if (lane == 0) {
    out[0] = d2 / (float)G::F;
    out[1] = ip == it ? 1.0f : 0.0f;
  }
}

// ---- Adam ownership of the batch-1 kernel ----
enum { B1_LOAD = 0, B1_STEP = 1, B1_STORE = 2 };

struct AdamK {
  float b1, b2, c1, c2, eps, lr_t;
};
__device__ __forceinline__ void adam_item(float& p, float& m, float& v, float g, const AdamK k) {
  m = k.b1 * m + k.c1 * g;
  v = k.b2 * v + k.c2 * g * g;
  p -= k.lr_t * m * __builtin_amdgcn_rcpf(__builtin_amdgcn_sqrtf(v) + k.eps);   // v_sqrt / v_rcp
}
// the same on a register pair (v_pk_mul / v_pk_fma / v_pk_add: two parameters per VALU op)
typedef float f2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ void adam_pair(f2& p, f2& m, f2& v, f2 g, const AdamK k) {
  m = k.b1 * m + k.c1 * g;
  v = k.b2 * v + (k.c2 * g) * g;
  f2 d = {__builtin_amdgcn_sqrtf(v.x), __builtin_amdgcn_sqrtf(v.y)};
  d += k.eps;
  const f2 r = {__builtin_amdgcn_rcpf(d.x), __builtin_amdgcn_rcpf(d.y)};
  p -= (k.lr_t * m) * r;
}

// one parameter (a bias): global offset, image slot, gradient
__device__ __forceinline__ void own_one(int mode, float& p, float& m, float& v, const RefArgs& a, float* L,
                                        int64_t gofs, int img, int dz, const AdamK ak) {
  if (mode == B1_LOAD) {
    p = a.flat[gofs];
    m = a.m[gofs];
    v = a.v[gofs];
  } else if (mode == B1_STORE) {
    a.flat[gofs] = p;
    a.m[gofs] = m;
    a.v[gofs] = v;
  } else {
    adam_item(p, m, v, L[dz], ak);
  }
  if (mode != B1_STORE) L[img] = p;
}

// One weight block: rows K, columns NA, rows per pass R.  Thread u owns column n = u % NA
// and rows k0 + R * i (k0 = u / NA), i < NI, held as register pairs R0 .. R0 + (NI + 1) / 2;
// fwd / bwd are the image addresses of row k0, row k0 + R * i sits fstep * i / bstep * i
// floats further; `in` indexes input k0 (natural order).
template <int MODE, int K, int NA, int R, int NI, int R0, int NR, bool BWD>
__device__ __forceinline__ void own_w(f2 (&p)[NR], f2 (&mo)[NR], f2 (&vo)[NR], const RefArgs& a, float* L, int u,
                                      int64_t gbase, int gstride, int gcol, int fwd, int fstep, int bwd, int bstep,
                                      int in, int dz, const AdamK ak) {
  constexpr int NP = (NI + 1) / 2;
  static_assert(R0 + NP <= NR, "ownership register budget");
  if (u >= R * NA) return;
  const int k0 = u / NA;
  auto valid = [&](int i) { return i < NI && (K % R == 0 || i + 1 < NI || k0 + R * i < K); };
  if (MODE == B1_STEP) {
    // every LDS read of the block first: the image writes below may alias them as far as
    // the compiler knows, and reads issued after a write would each pay a full round trip
    const float dzn = L[dz];
    float inv[2 * NP];
#pragma unroll
    for (int i = 0; i < 2 * NP; ++i) inv[i] = L[in + R * (valid(i) ? i : 0)];
#pragma unroll
    for (int q = 0; q < NP; ++q) {
      const f2 g = {inv[2 * q] * dzn, inv[2 * q + 1] * dzn};
      adam_pair(p[R0 + q], mo[R0 + q], vo[R0 + q], g, ak);
    }
  }
#pragma unroll
  for (int i = 0; i < NI; ++i) {
    if (valid(i)) {
      const int64_t g = gbase + (int64_t)(k0 + R * i) * gstride + gcol;
      f2 &pp = p[R0 + i / 2], &mm = mo[R0 + i / 2], &vv = vo[R0 + i / 2];
      if (MODE == B1_LOAD) {
        pp[i & 1] = a.flat[g];
        mm[i & 1] = a.m[g];
        vv[i & 1] = a.v[g];
      } else if (MODE == B1_STORE) {
        a.flat[g] = pp[i & 1];
        a.m[g] = mm[i & 1];
        a.v[g] = vv[i & 1];
      }
      if (MODE != B1_STORE) {
        L[fwd + fstep * i] = pp[i & 1];
        if (BWD) L[bwd + bstep * i] = pp[i & 1];
      }
    }
  }
}

// Adam (or load / store) of the parameters a thread of waves 1..7 (t = thread - 64) owns in
// block BLK (0..3: W1..W4 with their biases, 4: the head kernel and bias).
// `x_in` / `nat`: LDS offsets of this step's input row and natural-order activations.
template <int MODE, int BLK, typename G, int NR>
__device__ __forceinline__ void own_blk(f2 (&p)[NR], f2 (&mo)[NR], f2 (&vo)[NR], float& pb, float& mb, float& vb,
                                        const RefArgs& a, float* L, int x_in, int nat, const AdamK ak) {
  using Q = B1<G>;
  const int t = (int)threadIdx.x - 64;
  const int u = (t + Q::WROT) % NADAM;
  // W_L[k][n], n = gate * U + j (active columns i | g | o); Keras column col(n) of the 4U-wide kernel.
  // forward image: lane j + U * (k % P), slot sF + 3 * (k / P) + gate
  // backward image (consumer: the layer below, U' = K units, P' = 64 / K): lane k + K * (n % P'), slot sB + n / P'
  // bias b_L[n]: forward image lane j (part 0), slot sF + 3 * KP + gate; owned by thread t = BO + n of the
  // group (the ranges within a group do not overlap: one register slot)
#define SML_W_BLOCK(K_, U_, P_, KP_, R_, N_, R0_, SF, BW, SB, GW, GB_, BO, IN, DZ)                                    \
  {                                                                                                                  \
    constexpr int NA = 3 * U_, PB = 64 / K_;                                                                         \
    const int n = u % NA, k0 = u / NA, gate = n / U_, j = n % U_;                                                    \
    const int fwd = (SF + 3 * (k0 / P_) + gate) * 64 + j + U_ * (k0 % P_);                                           \
    const int bwd = BW ? Q::img(SB + n / PB, k0 + K_ * (n % PB)) : 0;                                              \
    own_w<MODE, K_, NA, R_, N_, R0_, NR, BW>(p, mo, vo, a, L, u, GW, 4 * U_, n < U_ ? n : n + U_, fwd,               \
                                             3 * (R_ / P_) * 64, bwd, R_, (IN) + k0, nat + (DZ) + n, ak);             \
    if (t >= BO && t < BO + NA) {                                                                                    \
      const int e = t - BO, bg = e / U_, bj = e % U_;                                                                \
      own_one(MODE, pb, mb, vb, a, L, GB_ + (e < U_ ? e : e + U_), (SF + 3 * KP_ + bg) * 64 + bj, nat + (DZ) + e,    \
              ak);                                                                                                   \
    }                                                                                                                \
  }
  constexpr int bo1 = 0, bo2 = bo1 + 3 * G::U1, bo3 = bo2 + 3 * G::U2, bo4 = bo3 + 3 * G::U3, bok = bo4 + 3 * G::U4;
  if constexpr (BLK == 0) {
    SML_W_BLOCK(G::F, G::U1, Q::P1, Q::KF1, Q::R1, Q::N1, Q::r1, Q::sF1, false, 0, G::gW1, G::gb1, bo1, x_in, Q::nZ1)
  } else if constexpr (BLK == 1) {
    SML_W_BLOCK(G::U1, G::U2, Q::P2, Q::KF2, Q::R2, Q::N2, Q::r2, Q::sF2, true, Q::sB1, G::gW2, G::gb2, bo2,
                nat + Q::nH1, Q::nZ2)
  } else if constexpr (BLK == 2) {
    SML_W_BLOCK(G::U2, G::U3, Q::P3, Q::KF3, Q::R3, Q::N3, Q::r3, Q::sF3, true, Q::sB2, G::gW3, G::gb3, bo3,
                nat + Q::nH2, Q::nZ3)
  } else if constexpr (BLK == 3) {
    SML_W_BLOCK(G::U3, G::U4, Q::P4, Q::KF4, Q::R4, Q::N4, Q::r4, Q::sF4, true, Q::sB3, G::gW4, G::gb4, bo4,
                nat + Q::nH3, Q::nZ4)
  } else {
    // head kernel K[k][f]: forward lane f + 32 * (k % 2), slot sHD + k / 2; backward (D4) lane k + 32 * (f % 2),
    // slot sB4 + f / 2; head bias: forward lane f, slot sHD + KHD
    const int f = t % G::F, k0 = t / G::F;
    const int fwd = (Q::sHD + k0 / 2) * 64 + f + 32 * (k0 % 2);
    const int bwd = Q::img(Q::sB4 + f / Q::P4, k0 + G::U4 * (f % Q::P4));
    own_w<MODE, G::U4, G::F, Q::RK, Q::NK, Q::rK, NR, true>(p, mo, vo, a, L, t, G::gK, G::F, f, fwd,
                                                            (Q::RK / 2) * 64, bwd, Q::RK, nat + Q::nH4 + k0,
                                                            nat + Q::nDY + f, ak);
    if (t >= bok && t < bok + G::F)
      own_one(MODE, pb, mb, vb, a, L, G::gkb + (t - bok), (Q::sHD + Q::KHD) * 64 + (t - bok), nat + Q::nDY + (t - bok),
              ak);
  }
#undef SML_W_BLOCK
}

// load / store every owned parameter
template <int MODE, typename G, int NR>
__device__ __forceinline__ void own_all_b1(f2 (&p)[NR], f2 (&mo)[NR], f2 (&vo)[NR], float& pb, float& mb, float& vb,
                                           const RefArgs& a, float* L, const AdamK ak) {
  own_blk<MODE, 0, G>(p, mo, vo, pb, mb, vb, a, L, 0, 0, ak);
  own_blk<MODE, 1, G>(p, mo, vo, pb, mb, vb, a, L, 0, 0, ak);
  own_blk<MODE, 2, G>(p, mo, vo, pb, mb, vb, a, L, 0, 0, ak);
  own_blk<MODE, 3, G>(p, mo, vo, pb, mb, vb, a, L, 0, 0, ak);
  own_blk<MODE, 4, G>(p, mo, vo, pb, mb, vb, a, L, 0, 0, ak);
}

// Block `blk` of NB sample rows into row buffer blk & 1 by asynchronous global -> LDS
// copies (global_load_lds_dword: LDS destination = M0 + 4 * lane, no registers held
// while the rows are in flight).  Buffer layout: NB x rows of F floats, then NB y rows.
// Issued from inline asm, so the compiler does not wait on it: the issuing wave orders it
// with an explicit `s_waitcnt vmcnt(0)` before the block is read.  `w0 / wstep`: the waves
// that share the chunks (all 8 for the first block, wave 0 alone afterwards).
#pragma clang diagnostic push
#pragma clang diagnostic ignored "-Winline-asm"  // m0 is deliberately clobbered (no other user here)
__device__ __forceinline__ void glds4(const float* src, unsigned lds_addr) {
  asm volatile("s_mov_b32 m0, %0\n\tglobal_load_lds_dword %1, off" ::"s"(lds_addr), "v"(src) : "memory", "m0");
}
#pragma clang diagnostic pop
__device__ __forceinline__ void wait_vm() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

template <typename G>
__device__ __forceinline__ float* row_block(float* L, int par) { return L + B1<G>::oROW + par * 2 * NB * G::F; }

template <typename G>
__device__ __forceinline__ void block_load(const RefArgs& a, float* L, int64_t blk, int w0, int wstep) {
  static_assert((2 * NB * G::F) % 64 == 0, "whole wave chunks");
  constexpr int CHUNKS = 2 * NB * G::F / 64;
  const int lane = threadIdx.x & 63;
  float* buf = row_block<G>(L, (int)(blk & 1));
  for (int c = w0; c < CHUNKS; c += wstep) {
    const int e = c * 64 + lane;
    const bool yrow = e >= NB * G::F;
    const int rem = yrow ? e - NB * G::F : e;
    const int st = rem / G::F, f = rem - st * G::F;
    const int64_t i = a.row0 + blk * NB + st;
    const unsigned dst = (unsigned)(uintptr_t)((__attribute__((address_space(3))) float*)(buf + c * 64));
    if (i < a.nrows) {
      const int64_t src = a.order ? (int64_t)a.order[i] : i;
      glds4(yrow ? a.y + src * a.ldy + f : a.x + src * a.ldx + f, __builtin_amdgcn_readfirstlane(dst));
    }
  }
}

#ifdef SML_LREF_PROBE
// Phase probe (tools/lref_probe): shader-clock cycles summed over a launch.  Wave 0:
// [0] chain compute, [1] chain waiting for the previous step's Adam; wave 1: [2] Adam busy,
// [3] Adam waiting on the chain; [4] steps.  Built only into the probe binary.
__device__ unsigned long long g_lref_probe[8];
#endif

template <typename G, int ACT>
__global__ __launch_bounds__(NT) void lstm_ref_train_b1_kernel(RefArgs a) {
  extern __shared__ __attribute__((aligned(16))) float L[];
  using Q = B1<G>;
  f2 p[Q::NOWN2], mo[Q::NOWN2], vo[Q::NOWN2];
  float pb = 0.0f, mb = 0.0f, vb = 0.0f;   // the thread's bias (if any)
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int64_t it0 = *a.iter;
  for (int i = threadIdx.x; i < Q::IMG_FLOATS; i += NT) L[i] = 0.0f;   // unused image slots stay 0
  if (threadIdx.x < 8) reinterpret_cast<unsigned*>(L)[Q::oCNT + threadIdx.x] = 0u;
  const int64_t avail = a.nrows - a.row0;
  const int total = (int)(avail < a.nsteps ? avail : a.nsteps);
  block_load<G>(a, L, 0, wave, NT / 64);
  wait_vm();
  lds_barrier();
  const AdamK ak0{a.beta1, a.beta2, 1.0f - a.beta1, 1.0f - a.beta2, a.eps, 0.0f};
  if (wave > 0) {
#pragma unroll
    for (int i = 0; i < Q::NOWN2; ++i) p[i] = mo[i] = vo[i] = f2{0.0f, 0.0f};
    own_all_b1<B1_LOAD, G>(p, mo, vo, pb, mb, vb, a, L, ak0);
  }
  lds_barrier();
#ifdef SML_LREF_PROBE
  unsigned long long pc[4] = {0, 0, 0, 0}, tq = clock64(), tn;
#endif
  if (wave == 0) {
    // ---- the chain ----
    if (total > NB) block_load<G>(a, L, 1, 0, 1);
    for (int s = 0; s < total; ++s) {
      const int slot = s % NB, blk = s / NB;
      if (slot == 0 && s > 0) wait_vm();   // this block was requested ~30 steps ago
      const float* xb = row_block<G>(L, blk & 1) + slot * G::F;
      chain_step<G, ACT>(L, xb, xb + NB * G::F, Q::oNAT + (s & 1) * Q::NATS, L + Q::oYP + (s & 1) * G::F,
                         (unsigned)s, lane SML_PROBE_PASS);
      // block b + 1 reuses block b - 1's buffer: by the end of step b * NB + 1 the chain's
      // wait has seen every Adam wave finish step b * NB (so also step b * NB - 1, the
      // buffer's last reader, and the stats of that step)
      if (slot == 1 && blk > 0 && (blk + 1) * NB < total) block_load<G>(a, L, blk + 1, 0, 1);
      SML_PROBE_MARK(0);
    }
  } else {
    // ---- Adam, one step behind the chain ----
    // Keras' lr_t = lr * sqrt(1 - beta2^t) / (1 - beta1^t), t = it0 + s + 1, in f32 closed form
    // (no loop-carried power: a launch split in two computes the same values)
    const float lg1 = __log2f(a.beta1), lg2 = __log2f(a.beta2);
    for (int s = 0; s < total; ++s) {
      const float t = (float)(it0 + s + 1);
      const AdamK ak{ak0.b1, ak0.b2, ak0.c1, ak0.c2, ak0.eps,
                     a.lr * __builtin_amdgcn_sqrtf(1.0f - exp2f(t * lg2)) / (1.0f - exp2f(t * lg1))};
      const int slot = s % NB, blk = s / NB;
      const float* xb = row_block<G>(L, blk & 1) + slot * G::F;
      const int nat = Q::oNAT + (s & 1) * Q::NATS, xin = (int)(xb - L);
      const unsigned st0 = 5u * (unsigned)s;   // the chain's stage count when step s starts
      // each block as soon as the chain has produced its gradient (and read its old backward
      // image); each finished block is counted for the next chain (oCNT + block)
      SML_PROBE_MARK(2);
      cnt_wait(L, Q::oCNT + 5, st0 + 1u);   // head done
      SML_PROBE_MARK(3);
      if (wave == 4) step_stats<G>(L + Q::oYP + (s & 1) * G::F, xb + NB * G::F, a.out + 2 * s, lane);
      own_blk<B1_STEP, 4, G>(p, mo, vo, pb, mb, vb, a, L, xin, nat, ak);
      SML_PROBE_MARK(2);
      cnt_wait(L, Q::oCNT + 5, st0 + 2u);   // D4 done
      SML_PROBE_MARK(3);
      own_blk<B1_STEP, 3, G>(p, mo, vo, pb, mb, vb, a, L, xin, nat, ak);
      SML_PROBE_MARK(2);
      cnt_wait(L, Q::oCNT + 5, st0 + 3u);   // D3 done
      SML_PROBE_MARK(3);
      own_blk<B1_STEP, 2, G>(p, mo, vo, pb, mb, vb, a, L, xin, nat, ak);
      SML_PROBE_MARK(2);
      cnt_wait(L, Q::oCNT + 5, st0 + 4u);   // D2 done
      SML_PROBE_MARK(3);
      own_blk<B1_STEP, 1, G>(p, mo, vo, pb, mb, vb, a, L, xin, nat, ak);
      SML_PROBE_MARK(2);
      cnt_wait(L, Q::oCNT + 5, st0 + 5u);   // D1 done: the chain of step s is complete
      SML_PROBE_MARK(3);
      own_blk<B1_STEP, 0, G>(p, mo, vo, pb, mb, vb, a, L, xin, nat, ak);
      cnt_bump(L, Q::oCNT + 0, lane);       // step s fully applied (W1 is every wave's last block)
      SML_PROBE_MARK(2);
    }
  }
  SML_PROBE_MARK(wave == 0 ? 0 : 2);
#ifdef SML_LREF_PROBE
  if (lane == 0 && wave <= 1) {
    for (int i = 0; i < 4; ++i) atomicAdd(&g_lref_probe[i], pc[i]);
    if (wave == 0) atomicAdd(&g_lref_probe[4], (unsigned long long)total);
  }
#endif
  wait_vm();   // no copy may still target LDS when the workgroup ends
  lds_barrier();
  if (wave > 0) own_all_b1<B1_STORE, G>(p, mo, vo, pb, mb, vb, a, L, ak0);
  if (threadIdx.x == 0) *a.iter = it0 + (total > 0 ? total : 0);
}

}  // namespace

int lstm_ref_train_params() { return Ref::NPARAM; }

#ifdef SML_LREF_PROBE
hipError_t lstm_ref_probe_read(unsigned long long* host8, bool reset) {
  hipError_t e = hipMemcpyFromSymbol(host8, HIP_SYMBOL(g_lref_probe), 8 * sizeof(unsigned long long));
  if (e == hipSuccess && reset) {
    const unsigned long long z[8] = {};
    e = hipMemcpyToSymbol(HIP_SYMBOL(g_lref_probe), z, sizeof z);
  }
  return e;
}
#endif

hipError_t lstm_ref_train_launch(float* flat, float* m, float* v, int64_t* iter, const float* x, int64_t ldx,
                                 const float* y, int64_t ldy, const int32_t* order, int64_t nrows, int64_t row0, int B,
                                 int nsteps, int act, float lr, float beta1, float beta2, float eps, float* out,
                                 hipStream_t stream) {
  if (B < 1 || B > MAXB || nsteps < 1 || row0 < 0 || row0 >= nrows) return hipErrorInvalidValue;
  RefArgs a{flat, m, v, iter, x, y, ldx, ldy, order, nrows, row0, B, nsteps, act, lr, beta1, beta2, eps, out};
  auto k = B > 1 ? lstm_ref_train_kernel<Ref> : act == 2 ? lstm_ref_train_b1_kernel<Ref, 2> : lstm_ref_train_b1_kernel<Ref, 1>;
  const size_t lds = sizeof(float) * (B == 1 ? B1<Ref>::LDS_FLOATS : Ref::LDS_FLOATS);
  if (lds > 65536) {
    const hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(k),
                                             hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return e;
  }
  hipLaunchKernelGGL(k, dim3(1), dim3(NT), lds, stream, a);
  return hipGetLastError();
}

}  // namespace sml
