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
// Batch-1 path (the reference's setting).  At B = 1 no phase of the chain has more than
// 32 (unit) tasks, so the whole forward + backward chain runs on wave 0 alone with
// lane-split dot products (lane = j + U * part, the P = 64 / U parts each take every
// P-th input and meet through permlane swaps) and NO workgroup barrier between its nine
// layers: a wave's LDS operations complete in order, so a value one lane writes is seen
// by every lane of the same wave that reads it afterwards.  The gates each lane saves
// in the forward pass stay in its registers for the backward pass (same j mapping).
// Per step there are two barriers: chain -> Adam on all 8 waves -> next step.
// Off the critical path, while wave 0 runs the chain:
//   * wave 1 computes the Adam step size lr_t and the loss / argmax accuracy of the
//     PREVIOUS step (from its saved prediction row);
//   * the sample rows arrive 32 steps ahead: every 32nd step the workgroup writes the
//     block it prefetched into registers 32 steps earlier to LDS and issues the loads of
//     the block after it, so no step waits on a global load.
// ===================================================================================
constexpr int NB = MAXB;          // steps per prefetched row block (reuses the two row buffers)

__device__ __forceinline__ void wave_order() { asm volatile("" ::: "memory"); }

// sum of a lane value over the P = 64 / U lane groups of lane = j + U * part
template <int U>
__device__ __forceinline__ float part_sum(float v, int lane) {
  static_assert(U == 16 || U == 32, "chain layouts");
  if (U == 16) v += xor16(v, lane);
  return v + xor32(v, lane);
}

// forward of one LSTM layer for one row on one wave: h[j] = o * act(i * g~)
template <int K, int U>
__device__ __forceinline__ void chain_fwd(const float* __restrict__ W, const float* __restrict__ bias, int S,
                                          const float* in, float* h, int act, int lane, float& ig, float& gt,
                                          float& og, float& ac) {
  constexpr int P = 64 / U;
  const int j = lane % U, part = lane / U;
  float zi = 0.0f, zg = 0.0f, zo = 0.0f;
#pragma unroll
  for (int k0 = 0; k0 < K; k0 += P) {
    const int k = k0 + part;
    if (K % P == 0 || k < K) {
      const float xv = in[k];
      const float* w = W + k * S + j;
      zi = fmaf(xv, w[0], zi);
      zg = fmaf(xv, w[U], zg);
      zo = fmaf(xv, w[2 * U], zo);
    }
  }
  zi = part_sum<U>(zi, lane) + bias[j];
  zg = part_sum<U>(zg, lane) + bias[U + j];
  zo = part_sum<U>(zo, lane) + bias[2 * U + j];
  ig = sigm(zi);
  gt = actf(act, zg);
  og = sigm(zo);
  ac = actf(act, ig * gt);
  if (part == 0) h[j] = og * ac;
  wave_order();
}

// backward of one LSTM layer for one row: dh[j] = up . Wup[j], then dz (i | g | o)
template <int U, int KN>
__device__ __forceinline__ void chain_bwd(const float* up, const float* __restrict__ Wup, int WS, float ig, float gt,
                                          float og, float ac, float* dz, int act, int lane) {
  constexpr int P = 64 / U;
  const int j = lane % U, part = lane / U;
  const float* wr = Wup + j * WS;
  float d0 = 0.0f, d1 = 0.0f;
#pragma unroll
  for (int n0 = 0; n0 < KN; n0 += 2 * P) {
    const int n = n0 + part;
    if (KN % P == 0 || n < KN) d0 = fmaf(up[n], wr[n], d0);
    if (n + P < KN) d1 = fmaf(up[n + P], wr[n + P], d1);
  }
  const float dh = part_sum<U>(d0 + d1, lane);
  const float dc = dh * og * actd(act, ac);
  if (part == 0) dz[j] = dc * gt * ig * (1.0f - ig);
  if (part == (P > 2 ? 1 : 0)) dz[U + j] = dc * ig * actd(act, gt);
  if (part == (P > 2 ? 2 : 1)) dz[2 * U + j] = dh * ac * og * (1.0f - og);
  wave_order();
}

// the whole chain of one Keras step at B = 1 (wave 0)
template <typename G>
__device__ __forceinline__ void chain_step(float* L, const float* xb, const float* yb, float* yp_out, int act,
                                           int lane) {
  float i1, g1, o1, a1, i2, g2, o2, a2, i3, g3, o3, a3, i4, g4, o4, a4;
  chain_fwd<G::F, G::U1>(L + G::lW1, L + G::lb1, G::S1, xb, L + G::oH1, act, lane, i1, g1, o1, a1);
  chain_fwd<G::U1, G::U2>(L + G::lW2, L + G::lb2, G::S2, L + G::oH1, L + G::oH2, act, lane, i2, g2, o2, a2);
  chain_fwd<G::U2, G::U3>(L + G::lW3, L + G::lb3, G::S3, L + G::oH2, L + G::oH3, act, lane, i3, g3, o3, a3);
  chain_fwd<G::U3, G::U4>(L + G::lW4, L + G::lb4, G::S4, L + G::oH3, L + G::oH4, act, lane, i4, g4, o4, a4);
  {  // TimeDistributed(Dense(F)) + the MSE gradient: lane = f + 32 * part, k split in halves
    const int f = lane & 31, part = lane >> 5;
    float acc = 0.0f;
    if (f < G::F) {
#pragma unroll
      for (int k0 = 0; k0 < G::U4; k0 += 2) acc = fmaf(L[G::oH4 + k0 + part], L[G::lK + (k0 + part) * G::SK + f], acc);
    }
    acc += xor32(acc, lane);
    if (f < G::F) {
      const float yp = acc + L[G::lkb + f];
      if (part == 0) L[G::oDY + f] = (2.0f / (float)G::F) * (yp - yb[f]);   // Keras MSE: mean over features
      else yp_out[f] = yp;
    }
    wave_order();
  }
  chain_bwd<G::U4, G::F>(L + G::oDY, L + G::lK, G::SK, i4, g4, o4, a4, L + G::oZ4, act, lane);
  chain_bwd<G::U3, 3 * G::U4>(L + G::oZ4, L + G::lW4, G::S4, i3, g3, o3, a3, L + G::oZ3, act, lane);
  chain_bwd<G::U2, 3 * G::U3>(L + G::oZ3, L + G::lW3, G::S3, i2, g2, o2, a2, L + G::oZ2, act, lane);
  chain_bwd<G::U1, 3 * G::U2>(L + G::oZ2, L + G::lW2, G::S2, i1, g1, o1, a1, L + G::oZ1, act, lane);
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

// Block `blk` of NB sample rows into LDS buffer blk & 1 by asynchronous global -> LDS
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
__device__ __forceinline__ float* row_block(float* L, int par) { return L + G::oX + par * 2 * NB * G::F; }

template <typename G>
__device__ __forceinline__ void block_load(const RefArgs& a, float* L, int64_t blk) {
  static_assert(2 * 2 * NB * G::F <= 4 * MAXB * G::XS, "two row blocks fit the batch path's row buffers");
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

template <typename G>
__global__ __launch_bounds__(NT) void lstm_ref_train_b1_kernel(RefArgs a) {
  extern __shared__ __attribute__((aligned(16))) float L[];
  constexpr int R = own_regs<G>();
  static_assert(G::U1 <= 32 && G::U2 <= 32 && G::U3 <= 32 && G::U4 <= 32 && G::F <= 32, "one-wave chain");
  float p[R], mo[R], vo[R];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int64_t it0 = *a.iter;
  own_all<OWN_LOAD, G>(p, mo, vo, a, L, nullptr, 0, 0.0f);
  const int64_t avail = a.nrows - a.row0;
  const int total = (int)(avail < a.nsteps ? avail : a.nsteps);
  block_load<G>(a, L, 0);
  wait_vm();
  if (total > NB) block_load<G>(a, L, 1);
  double b1t = pow((double)a.beta1, (double)it0), b2t = pow((double)a.beta2, (double)it0);
  float* const yp_buf = L + G::oG1;   // [2][F] prediction rows (the batch path's gate saves are unused here)
  float* const lr_slot = L + G::oST;
  lds_barrier();
  for (int s = 0; s < total; ++s) {
    const int slot = s % NB, par = (s / NB) & 1;
    const float* xb = row_block<G>(L, par) + slot * G::F;
    const float* yb = xb + NB * G::F;
    b1t *= (double)a.beta1;
    b2t *= (double)a.beta2;
    if (wave == 0) {
      chain_step<G>(L, xb, yb, yp_buf + (s & 1) * G::F, a.act, lane);
    } else if (wave == 1) {
      if (lane == 0) *lr_slot = (float)((double)a.lr * sqrt(1.0 - b2t) / (1.0 - b1t));
      if (s > 0) {
        const int sp = s - 1;
        step_stats<G>(yp_buf + (sp & 1) * G::F, row_block<G>(L, (sp / NB) & 1) + (NB + sp % NB) * G::F,
                      a.out + 2 * sp, lane);
      }
    }
    lds_barrier();
    own_all<OWN_STEP, G>(p, mo, vo, a, L, xb, 1, *lr_slot);
    // block b + 1 was requested 32 steps ago: land it before the barrier that ends block b.
    // Block b + 2 reuses block b's buffer once the stats of b's last step are out (slot 0).
    if (slot == NB - 1) wait_vm();
    if (slot == 0 && s > 0 && (s / NB + 1) * NB < total) block_load<G>(a, L, s / NB + 1);
    lds_barrier();
  }
  if (total > 0 && wave == 1) {
    const int sp = total - 1;
    step_stats<G>(yp_buf + (sp & 1) * G::F, row_block<G>(L, (sp / NB) & 1) + (NB + sp % NB) * G::F, a.out + 2 * sp,
                  lane);
  }
  wait_vm();   // no copy may still target LDS when the workgroup ends
  own_all<OWN_STORE, G>(p, mo, vo, a, L, nullptr, 0, 0.0f);
  if (threadIdx.x == 0) *a.iter = it0 + (total > 0 ? total : 0);
}

}  // namespace

int lstm_ref_train_params() { return Ref::NPARAM; }

hipError_t lstm_ref_train_launch(float* flat, float* m, float* v, int64_t* iter, const float* x, int64_t ldx,
                                 const float* y, int64_t ldy, const int32_t* order, int64_t nrows, int64_t row0, int B,
                                 int nsteps, int act, float lr, float beta1, float beta2, float eps, float* out,
                                 hipStream_t stream) {
  if (B < 1 || B > MAXB || nsteps < 1 || row0 < 0 || row0 >= nrows) return hipErrorInvalidValue;
  RefArgs a{flat, m, v, iter, x, y, ldx, ldy, order, nrows, row0, B, nsteps, act, lr, beta1, beta2, eps, out};
  auto k = B == 1 ? lstm_ref_train_b1_kernel<Ref> : lstm_ref_train_kernel<Ref>;
  const size_t lds = sizeof(float) * Ref::LDS_FLOATS;
  if (lds > 65536) {
    const hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(k),
                                             hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return e;
  }
  hipLaunchKernelGGL(k, dim3(1), dim3(NT), lds, stream, a);
  return hipGetLastError();
}

}  // namespace sml
