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
// Two kernels share that ownership scheme.  At batch 1 (the reference's setting,
// `lstm_ref_train_b1_kernel`, further down) the chain of nine layers runs on ONE wave with
// no workgroup barrier inside it, and a step has two barriers.  For batches 2..32
// (`lstm_ref_train_kernel`) each step is 10 barrier-separated phases:
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
//     weights it multiplies, slot-major (slot s of lane l at s * 64 + l: conflict-free,
//     paired into ds_read2st64).  A weight has a forward image (the lane that uses it in
//     its layer's dot product) and, for W2..W4 and the head kernel, a backward image (the
//     lane that uses it in dh of the layer below).  A layer's image is requested one
//     layer ahead, so its latency hides under the current layer's math.
//   * Activations pass between layers through LDS, each written twice: in natural order
//     (the weight gradients read it) and part-major for the consuming layer (each part's
//     inputs contiguous: 16-byte reads).
// Adam.  All 8 waves, between the step's two barriers.  Thread t owns column n = t % NA
// of a weight block and rows k = t / NA + R * i, with R a multiple of the forward split
// P, so every image address is a per-block base plus a compile-time offset.  It keeps
// (p, m, v) in registers and writes the new value into both images.
// Off the critical path, while wave 0 runs the chain:
//   * wave 1 computes the Adam step size lr_t and the loss / argmax accuracy of the
//     PREVIOUS step (from its saved prediction row);
//   * the sample rows arrive 32 steps ahead by asynchronous global -> LDS copies.
// ===================================================================================
constexpr int NB = MAXB;          // steps per prefetched row block

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
  // LDS map (floats)
  static constexpr int oROW = NSLOT * 64;                        // 2 blocks x [NB x rows | NB y rows]
  static constexpr int oH1 = oROW + 4 * NB * F, oH2 = oH1 + U1, oH3 = oH2 + U2, oH4 = oH3 + U3;   // natural order
  static constexpr int oZ1 = oH4 + U4, oZ2 = oZ1 + 3 * U1, oZ3 = oZ2 + 3 * U2, oZ4 = oZ3 + 3 * U3;
  static constexpr int oDY = oZ4 + 3 * U4;
  // part-major copies for the consuming layer (each part's run 16-byte aligned)
  static constexpr int qH1 = c4(oDY + F), qH2 = qH1 + P2 * c4(KF2), qH3 = qH2 + P3 * c4(KF3);
  static constexpr int qH4 = qH3 + P4 * c4(KF4), qDY = qH4 + PH * c4(KHD), qZ4 = qDY + P4 * c4(KB4);
  static constexpr int qZ3 = qZ4 + P3 * c4(KB3), qZ2 = qZ3 + P2 * c4(KB2);
  static constexpr int oYP = qZ2 + P1 * c4(KB1);                 // [2][F] predictions (stats of the previous step)
  static constexpr int oLR = oYP + 2 * F;                         // Adam step size of the current step
  static constexpr int oSINK = c4(oLR + 1);                       // per-lane sink for writes a lane must not make
  static constexpr int LDS_FLOATS = oSINK + 64;
  // Adam ownership: rows per pass R (a multiple of the forward split), items per thread
  static constexpr int rpass(int na, int p) { return (NT / na) / p * p; }
  static constexpr int R1 = rpass(3 * U1, P1), R2 = rpass(3 * U2, P2), R3 = rpass(3 * U3, P3);
  static constexpr int R4 = rpass(3 * U4, P4), RK = rpass(F, PH);
  static constexpr int N1 = (F + R1 - 1) / R1, N2 = (U1 + R2 - 1) / R2, N3 = (U2 + R3 - 1) / R3;
  static constexpr int N4 = (U3 + R4 - 1) / R4, NK = (U4 + RK - 1) / RK;
  static constexpr int NBIAS = 3 * (U1 + U2 + U3 + U4) + F;
  static_assert(NBIAS <= NT, "one bias per thread");
  static constexpr int NOWN = N1 + N2 + N3 + N4 + NK + 1;
};

__device__ __forceinline__ void wave_order() { asm volatile("" ::: "memory"); }

// sum of a lane value over the P = 64 / U lane groups of lane = j + U * part
template <int U>
__device__ __forceinline__ float part_sum(float v, int lane) {
  static_assert(U == 16 || U == 32, "chain layouts");
  if (U == 16) v += xor16(v, lane);
  return v + xor32(v, lane);
}

// N consecutive image slots of this lane from slot s0 (slot-major: stride 64 floats)
template <int N>
__device__ __forceinline__ void img_rd(const float* L, int s0, int lane, float (&w)[N]) {
  const float* b = L + s0 * 64 + lane;
#pragma unroll
  for (int i = 0; i < N; ++i) w[i] = b[i * 64];
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

// forward of one LSTM unit from this lane's image (3 gates x KP inputs + bias slots)
template <int KP, int U, int NW, int NI>
__device__ __forceinline__ float fwd_unit(const float (&w)[NW], const float (&in)[NI], int act, int lane, float& ig,
                                          float& gt, float& og, float& ac) {
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
  gt = actf(act, zg);
  og = sigm(zo);
  ac = actf(act, ig * gt);
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
__device__ __forceinline__ void dz_unit(float dh, float ig, float gt, float og, float ac, int act, float& zi,
                                        float& zg, float& zo) {
  const float dc = dh * og * actd(act, ac);
  zi = dc * gt * ig * (1.0f - ig);
  zg = dc * ig * actd(act, gt);
  zo = dh * ac * og * (1.0f - og);
}

// the whole chain of one Keras step at B = 1 (wave 0)
template <typename G>
__device__ __forceinline__ void chain_step(float* L, const float* xb, const float* yb, float* yp_out, int act,
                                           int lane) {
  using Q = B1<G>;
  const int j1 = lane % G::U1, p1 = lane / G::U1, j2 = lane % G::U2, p2 = lane / G::U2;
  const int j3 = lane % G::U3, p3 = lane / G::U3, j4 = lane % G::U4, p4 = lane / G::U4;
  float i1, g1, o1, a1, i2, g2, o2, a2, i3, g3, o3, a3, i4, g4, o4, a4, h;
  float x[Q::KF1];
#pragma unroll
  for (int i = 0; i < Q::KF1; ++i) x[i] = xb[p1 + Q::P1 * i];
  float w1[3 * Q::KF1 + 3], w2[3 * Q::KF2 + 3];
  img_rd(L, Q::sF1, lane, w1);
  img_rd(L, Q::sF2, lane, w2);
  h = fwd_unit<Q::KF1, G::U1>(w1, x, act, lane, i1, g1, o1, a1);
  put_h<Q, Q::P2, Q::KF2>(L, Q::oH1, Q::qH1, j1, p1, lane, h);

  float w3[3 * Q::KF3 + 3], in2[c4(Q::KF2)];
  img_rd(L, Q::sF3, lane, w3);
  vec_rd(L + Q::qH1 + p2 * c4(Q::KF2), in2);
  h = fwd_unit<Q::KF2, G::U2>(w2, in2, act, lane, i2, g2, o2, a2);
  put_h<Q, Q::P3, Q::KF3>(L, Q::oH2, Q::qH2, j2, p2, lane, h);

  float w4[3 * Q::KF4 + 3], in3[c4(Q::KF3)];
  img_rd(L, Q::sF4, lane, w4);
  vec_rd(L + Q::qH2 + p3 * c4(Q::KF3), in3);
  h = fwd_unit<Q::KF3, G::U3>(w3, in3, act, lane, i3, g3, o3, a3);
  put_h<Q, Q::P4, Q::KF4>(L, Q::oH3, Q::qH3, j3, p3, lane, h);

  float wh[Q::KHD + 1], in4[c4(Q::KF4)];
  img_rd(L, Q::sHD, lane, wh);
  vec_rd(L + Q::qH3 + p4 * c4(Q::KF4), in4);
  h = fwd_unit<Q::KF4, G::U4>(w4, in4, act, lane, i4, g4, o4, a4);
  put_h<Q, Q::PH, Q::KHD>(L, Q::oH4, Q::qH4, j4, p4, lane, h);

  float wb4[Q::KB4];
  img_rd(L, Q::sB4, lane, wb4);
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
    L[f >= G::F ? sink : (ph == 0 ? Q::oDY + f : Q::qDY + qpos<Q::P4, Q::KB4>(f))] = dy;
    yp_out[f < G::F && ph == 0 ? f : sink - (int)(yp_out - L)] = yp;
    wave_order();
  }
  float wb3[Q::KB3], up4[c4(Q::KB4)], zi, zg, zo;
  img_rd(L, Q::sB3, lane, wb3);
  vec_rd(L + Q::qDY + p4 * c4(Q::KB4), up4);
  dz_unit(bwd_dh<Q::KB4, G::U4>(wb4, up4, lane), i4, g4, o4, a4, act, zi, zg, zo);
  put_dz<Q, G::U4, Q::P3, Q::KB3, true>(L, Q::oZ4, Q::qZ4, j4, p4, lane, zi, zg, zo);

  float wb2[Q::KB2], up3[c4(Q::KB3)];
  img_rd(L, Q::sB2, lane, wb2);
  vec_rd(L + Q::qZ4 + p3 * c4(Q::KB3), up3);
  dz_unit(bwd_dh<Q::KB3, G::U3>(wb3, up3, lane), i3, g3, o3, a3, act, zi, zg, zo);
  put_dz<Q, G::U3, Q::P2, Q::KB2, true>(L, Q::oZ3, Q::qZ3, j3, p3, lane, zi, zg, zo);

  float wb1[Q::KB1], up2[c4(Q::KB2)];
  img_rd(L, Q::sB1, lane, wb1);
  vec_rd(L + Q::qZ3 + p2 * c4(Q::KB2), up2);
  dz_unit(bwd_dh<Q::KB2, G::U2>(wb2, up2, lane), i2, g2, o2, a2, act, zi, zg, zo);
  put_dz<Q, G::U2, Q::P1, Q::KB1, true>(L, Q::oZ2, Q::qZ2, j2, p2, lane, zi, zg, zo);

  float up1[c4(Q::KB1)];
  vec_rd(L + Q::qZ2 + p1 * c4(Q::KB1), up1);
  dz_unit(bwd_dh<Q::KB1, G::U1>(wb1, up1, lane), i1, g1, o1, a1, act, zi, zg, zo);
  put_dz<Q, G::U1, 1, 1, false>(L, Q::oZ1, 0, j1, p1, lane, zi, zg, zo);
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
// One weight block: rows K, columns NA, forward split P (rows per pass R).  Thread t owns
// column n = t % NA and rows k0 + R * i (k0 = t / NA).  fwd(k0, n) / bwd(k0, n) give the
// image addresses of row k0; row k0 + R * i sits FSTEP * i / BSTEP * i floats further.
enum { B1_LOAD = 0, B1_STEP = 1, B1_STORE = 2 };

struct AdamK {
  float b1, b2, c1, c2, eps, lr_t;
};
__device__ __forceinline__ void adam_item(float& p, float& m, float& v, float g, const AdamK& k) {
  m = k.b1 * m + k.c1 * g;
  v = k.b2 * v + k.c2 * g * g;
  p -= k.lr_t * m * __builtin_amdgcn_rcpf(__builtin_amdgcn_sqrtf(v) + k.eps);   // v_sqrt / v_rcp
}

template <int MODE, int K, int NA, int R, int NI, int R0, int NR, bool BWD>
__device__ __forceinline__ void own_w(float (&p)[NR], float (&mo)[NR], float (&vo)[NR], const RefArgs& a, float* L,
                                      int t, int64_t gbase, int gstride, int gcol, int fwd, int fstep, int bwd,
                                      int bstep, int in, int dz, const AdamK& ak) {
  static_assert(R0 + NI <= NR, "ownership register budget");
  if (t >= R * NA) return;
  const int k0 = t / NA;
  float dzn = 0.0f;
  if (MODE == B1_STEP) dzn = L[dz];
#pragma unroll
  for (int i = 0; i < NI; ++i) {
    const int k = k0 + R * i;
    if ((K % R == 0 || i + 1 < NI) || k < K) {
      const int64_t g = gbase + (int64_t)k * gstride + gcol;
      if (MODE == B1_LOAD) {
        p[R0 + i] = a.flat[g];
        mo[R0 + i] = a.m[g];
        vo[R0 + i] = a.v[g];
      } else if (MODE == B1_STORE) {
        a.flat[g] = p[R0 + i];
        a.m[g] = mo[R0 + i];
        a.v[g] = vo[R0 + i];
      } else {
        adam_item(p[R0 + i], mo[R0 + i], vo[R0 + i], L[in + R * i] * dzn, ak);
      }
      if (MODE != B1_STORE) {
        L[fwd + fstep * i] = p[R0 + i];
        if (BWD) L[bwd + bstep * i] = p[R0 + i];
      }
    }
  }
}

template <int MODE, typename G, int NR>
__device__ __forceinline__ void own_b1(float (&p)[NR], float (&mo)[NR], float (&vo)[NR], const RefArgs& a, float* L,
                                       const float* xb, const AdamK& ak) {
  using Q = B1<G>;
  const int t = threadIdx.x;
  const int x_in = (int)(xb - L);
  // W_L[k][n], n = gate * U + j (active columns i | g | o); Keras column col(n) of the 4U-wide kernel
  // forward image: lane j + U * (k % P), slot sF + 3 * (k / P) + gate
  // backward image (consumer: the layer below, U' = K units, P' = 64 / K): lane k + K * (n % P'), slot sB + n / P'
#define SML_W_BLOCK(K_, U_, P_, R_, N_, R0_, SF, BW, SB, GW, IN, DZ)                                                 \
  {                                                                                                                  \
    constexpr int NA = 3 * U_, PB = 64 / K_;                                                                         \
    const int n = t % NA, k0 = t / NA, gate = n / U_, j = n % U_;                                                    \
    const int fwd = (SF + 3 * (k0 / P_) + gate) * 64 + j + U_ * (k0 % P_);                                           \
    const int bwd = BW ? (SB + n / PB) * 64 + k0 + K_ * (n % PB) : 0;                                                \
    own_w<MODE, K_, NA, R_, N_, R0_, NR, BW>(p, mo, vo, a, L, t, GW, 4 * U_, n < U_ ? n : n + U_, fwd,               \
                                             3 * (R_ / P_) * 64, bwd, R_, (IN) + k0, DZ + n, ak);                     \
  }
  constexpr int r1 = 0, r2 = r1 + Q::N1, r3 = r2 + Q::N2, r4 = r3 + Q::N3, rk = r4 + Q::N4, rb = rk + Q::NK;
  SML_W_BLOCK(G::F, G::U1, Q::P1, Q::R1, Q::N1, r1, Q::sF1, false, 0, G::gW1, x_in, Q::oZ1)
  SML_W_BLOCK(G::U1, G::U2, Q::P2, Q::R2, Q::N2, r2, Q::sF2, true, Q::sB1, G::gW2, Q::oH1, Q::oZ2)
  SML_W_BLOCK(G::U2, G::U3, Q::P3, Q::R3, Q::N3, r3, Q::sF3, true, Q::sB2, G::gW3, Q::oH2, Q::oZ3)
  SML_W_BLOCK(G::U3, G::U4, Q::P4, Q::R4, Q::N4, r4, Q::sF4, true, Q::sB3, G::gW4, Q::oH3, Q::oZ4)
#undef SML_W_BLOCK
  {  // head kernel K[k][f]: forward lane f + 32 * (k % 2), slot sHD + k / 2; backward (D4) lane k + 32 * (f % 2), slot sB4 + f / 2
    const int f = t % G::F, k0 = t / G::F;
    const int fwd = (Q::sHD + k0 / 2) * 64 + f + 32 * (k0 % 2);
    const int bwd = (Q::sB4 + f / Q::P4) * 64 + k0 + G::U4 * (f % Q::P4);
    own_w<MODE, G::U4, G::F, Q::RK, Q::NK, rk, NR, true>(p, mo, vo, a, L, t, G::gK, G::F, f, fwd, (Q::RK / 2) * 64,
                                                         bwd, Q::RK, Q::oH4 + k0, Q::oDY + f, ak);
  }
  if (t < Q::NBIAS) {   // one bias per thread: b1 | b2 | b3 | b4 | head bias
    int gofs, img, dz;
    auto pick = [&](int e, int U, int sF, int KP, int gb, int oz) {
      const int gate = e / U, j = e % U;
      gofs = gb + (e < U ? e : e + U);
      img = (sF + 3 * KP + gate) * 64 + j;
      dz = oz + e;
    };
    constexpr int e1 = 3 * G::U1, e2 = e1 + 3 * G::U2, e3 = e2 + 3 * G::U3, e4 = e3 + 3 * G::U4;
    if (t < e1) pick(t, G::U1, Q::sF1, Q::KF1, G::gb1, Q::oZ1);
    else if (t < e2) pick(t - e1, G::U2, Q::sF2, Q::KF2, G::gb2, Q::oZ2);
    else if (t < e3) pick(t - e2, G::U3, Q::sF3, Q::KF3, G::gb3, Q::oZ3);
    else if (t < e4) pick(t - e3, G::U4, Q::sF4, Q::KF4, G::gb4, Q::oZ4);
    else {
      const int f = t - e4;
      gofs = G::gkb + f;
      img = (Q::sHD + Q::KHD) * 64 + f;
      dz = Q::oDY + f;
    }
    if (MODE == B1_LOAD) {
      p[rb] = a.flat[gofs];
      mo[rb] = a.m[gofs];
      vo[rb] = a.v[gofs];
    } else if (MODE == B1_STORE) {
      a.flat[gofs] = p[rb];
      a.m[gofs] = mo[rb];
      a.v[gofs] = vo[rb];
    } else {
      adam_item(p[rb], mo[rb], vo[rb], L[dz], ak);
    }
    if (MODE != B1_STORE) L[img] = p[rb];
  }
}

// Block `blk` of NB sample rows into row buffer blk & 1 by asynchronous global -> LDS
// copies (global_load_lds_dword: LDS destination = M0 + 4 * lane, no registers held
// while the rows are in flight).  Buffer layout: NB x rows of F floats, then NB y rows.
// Issued from inline asm, so the compiler does not wait on it: the caller orders it with
// an explicit `s_waitcnt vmcnt(0)` and a barrier before the block is read.
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
__device__ __forceinline__ void block_load(const RefArgs& a, float* L, int64_t blk) {
  static_assert((2 * NB * G::F) % 64 == 0, "whole wave chunks");
  constexpr int CHUNKS = 2 * NB * G::F / 64;
  const int lane = threadIdx.x & 63;
  float* buf = row_block<G>(L, (int)(blk & 1));
  for (int c = threadIdx.x >> 6; c < CHUNKS; c += NT / 64) {
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
// Phase probe (tools/lref_probe): shader-clock cycles summed over the steps of a launch,
// measured by wave 0: [0] chain, [1] chain end -> past barrier 1, [2] Adam, [3] -> past
// barrier 2, [4] steps.  Built only into the probe binary.
__device__ unsigned long long g_lref_probe[8];
#endif

template <typename G>
__global__ __launch_bounds__(NT) void lstm_ref_train_b1_kernel(RefArgs a) {
  extern __shared__ __attribute__((aligned(16))) float L[];
  using Q = B1<G>;
  float p[Q::NOWN], mo[Q::NOWN], vo[Q::NOWN];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int64_t it0 = *a.iter;
  for (int i = threadIdx.x; i < Q::NSLOT * 64; i += NT) L[i] = 0.0f;   // unused image slots stay 0
  lds_barrier();
  AdamK ak{a.beta1, a.beta2, 1.0f - a.beta1, 1.0f - a.beta2, a.eps, 0.0f};
  own_b1<B1_LOAD, G>(p, mo, vo, a, L, row_block<G>(L, 0), ak);
  const int64_t avail = a.nrows - a.row0;
  const int total = (int)(avail < a.nsteps ? avail : a.nsteps);
  block_load<G>(a, L, 0);
  wait_vm();
  if (total > NB) block_load<G>(a, L, 1);
  double b1t = pow((double)a.beta1, (double)it0), b2t = pow((double)a.beta2, (double)it0);
  float* const yp_buf = L + Q::oYP;
  lds_barrier();
#ifdef SML_LREF_PROBE
  unsigned long long pc[4] = {0, 0, 0, 0}, tq = clock64(), tn;
#define SML_PROBE_MARK(i) (tn = clock64(), pc[i] += tn - tq, tq = tn)
#else
#define SML_PROBE_MARK(i) ((void)0)
#endif
  for (int s = 0; s < total; ++s) {
    const int slot = s % NB, par = (s / NB) & 1;
    const float* xb = row_block<G>(L, par) + slot * G::F;
    const float* yb = xb + NB * G::F;
    b1t *= (double)a.beta1;
    b2t *= (double)a.beta2;
    if (wave == 0) {
      chain_step<G>(L, xb, yb, yp_buf + (s & 1) * G::F, a.act, lane);
      SML_PROBE_MARK(0);
    } else if (wave == 1) {
      if (lane == 0) L[Q::oLR] = (float)((double)a.lr * sqrt(1.0 - b2t) / (1.0 - b1t));
      if (s > 0) {
        const int sp = s - 1;
        step_stats<G>(yp_buf + (sp & 1) * G::F, row_block<G>(L, (sp / NB) & 1) + (NB + sp % NB) * G::F,
                      a.out + 2 * sp, lane);
      }
    }
    lds_barrier();
    SML_PROBE_MARK(1);
    ak.lr_t = L[Q::oLR];
    own_b1<B1_STEP, G>(p, mo, vo, a, L, xb, ak);
    SML_PROBE_MARK(2);
    // block b + 1 was requested 32 steps ago: land it before the barrier that ends block b.
    // Block b + 2 reuses block b's buffer once the stats of b's last step are out (slot 0).
    if (slot == NB - 1) wait_vm();
    if (slot == 0 && s > 0 && (s / NB + 1) * NB < total) block_load<G>(a, L, s / NB + 1);
    lds_barrier();
    SML_PROBE_MARK(3);
  }
#ifdef SML_LREF_PROBE
  if (threadIdx.x == 0) {
    for (int i = 0; i < 4; ++i) atomicAdd(&g_lref_probe[i], pc[i]);
    atomicAdd(&g_lref_probe[4], (unsigned long long)total);
  }
#endif
#undef SML_PROBE_MARK
  if (total > 0 && wave == 1) {
    const int sp = total - 1;
    step_stats<G>(yp_buf + (sp & 1) * G::F, row_block<G>(L, (sp / NB) & 1) + (NB + sp % NB) * G::F, a.out + 2 * sp,
                  lane);
  }
  wait_vm();   // no copy may still target LDS when the workgroup ends
  own_b1<B1_STORE, G>(p, mo, vo, a, L, nullptr, ak);
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
  auto k = B == 1 ? lstm_ref_train_b1_kernel<Ref> : lstm_ref_train_kernel<Ref>;
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
