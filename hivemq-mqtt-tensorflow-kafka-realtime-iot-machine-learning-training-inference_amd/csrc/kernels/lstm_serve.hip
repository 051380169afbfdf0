// Persistent per-event LSTM scorer (BASELINE config 3 model, served like config 5).
//
// The reference LSTM job predicts each next car event from a window of the last
// `look_back` events and streams the predictions through a Python OutputCallback
// (LSTM-TensorFlow-IO-Kafka/cardata-v2.py:220-273).  Here one resident workgroup polls
// the host-mapped request ring exactly like the autoencoder scorer (ae_serve.hip: LL
// framed slots, no launch and no hipMemcpy per event) and keeps, on the device, the last
// T normalised events of every car key (a per-key ring in HBM: 100 000 cars x 50 x 18
// floats = 360 MB of 288 GB) plus the key's previous prediction.  Per event:
//   1. append the event to its key's window;
//   2. score it: mean squared error against the prediction made at the key's previous
//      event (the LSTM's own anomaly signal: how far the car moved from its forecast);
//   3. once T events are known, run the whole stack (LSTM layers, RepeatVector, Dense /
//      TimeDistributed head) over the window from zero state -- Keras' stateless
//      semantics, as the model was trained -- and emit the forecast of the next event.
//
// Execution: 4 waves.  An LSTM step is z = [x_t ; h] . [W ; U] + b for 4u <= 128 gates:
// wave w owns gates 32w..32w+31, lane half k (lane >> 5) one 32-long half of the
// concatenated input, with its 32 weights in registers (every layer's, loaded once at
// launch); the two halves meet through a permlane32 swap, the gates through LDS, and
// threads t < u update unit t's cell state in a register.  Two workgroup barriers per
// step.  Weights, biases, the window and the activations live in LDS.
//
// Stacks of up to four LSTM layers (every one but the last returning sequences) under
// one Dense head -- BASELINE config 3's LSTM(32) -> LSTM(16) -> Dense(18) at look_back 50
// -- take the PIPELINED variant instead: wave l runs LSTM layer l over the window with no
// workgroup barrier inside the recurrence.  Lane (p, j) = (lane >> 5, lane & 31) computes
// two gates of unit j -- (i, g~) on p = 0, (f, o) on p = 1 -- as one packed-fp32 dot
// product (v_pk_fma_f32) against its [W ; U] columns held in registers; the halves meet
// through one permlane32 swap.  h_t goes to the layer's LDS sequence buffer, then a
// release fence and the layer's step counter; layer l + 1 spins on that counter
// (acquire) and consumes h_t while layer l computes step t + 1, so an event costs
// ~T + L - 1 step latencies instead of L x T steps with two barriers each.  The last
// layer's wave applies the Dense head to h_{T-1}.
//
// Exit conditions every wave reaches: the host's stop flag or `idle` without a request
// (decided by wave 0, broadcast through LDS at the next barrier).
#include <cstdlib>

#include "sml_common.h"
#include "sml_ops.h"
#include "sml_serve_dev.h"

namespace sml {
namespace {

using namespace serve_dev;

constexpr int NT = 256;
constexpr int MAXW = 32;       // widest layer input / output
constexpr int MAXT = 64;       // longest window
constexpr int MAXLSTM = 4;     // LSTM layers with register-resident weights
constexpr int KEY_WORD = 31;   // request word carrying the car key
constexpr int ZX_RING = 8;     // PIPE: steps of input projection buffered ahead of a recurrence

__device__ __forceinline__ float sigm(float z) { return 1.0f / (1.0f + __expf(-z)); }

// The per-key state (window ring, count, forecast) is written by one wave and read by the
// others in later events: agent-scope relaxed atomics go around the per-CU L1, so no wave
// can hit a stale line of an older event.
template <typename T>
__device__ __forceinline__ T ld_agent(const T* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
template <typename T>
__device__ __forceinline__ void st_agent(T* p, T v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ float act_lstm(int a, float z) { return a == ACT_RELU ? fmaxf(z, 0.f) : tanhf(z); }

struct Smem {
  float* H;       // PIPE: [MAXLSTM][MAXT][MAXW] per-layer h sequences
  float* w;       // all parameters, Keras order
  float* seqa;    // [MAXT][MAXW]
  float* seqb;    // [MAXT][MAXW]
  float* v;       // [64]: [x_t ; h]
  float* z;       // [128] gate pre-activations
  float* pred;    // [MAXW]
  float* xrow;    // [MAXW]
  float* sc;      // [MAXW]
  float* sh;      // [MAXW]
  int* ctl;       // [8]: quit, key, count, seen sequence, t_seen lo / hi
};

// a.L is a pipelinable stack: n LSTM layers (u, in <= 32, n <= MAXLSTM, all but the last
// returning sequences), then exactly one Dense head; returns n (0: not pipelinable)
__host__ __device__ inline int pipe_layers(const LstmServeArgs& a) {
  int n = 0;
  while (n < a.nl && a.L[n].kind == LS_LSTM) ++n;
  if (n < 1 || n > MAXLSTM || n + 1 != a.nl || a.L[n].kind != LS_DENSE || a.L[n].u > MAXW) return 0;
  for (int l = 0; l < n; ++l)
    if (a.L[l].u > 32 || a.L[l].in > 32 || (l + 1 < n && !a.L[l].ret)) return 0;
  return n;
}

typedef float f32x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ f32x2 fma2(float x, f32x2 w, f32x2 acc) {
  return __builtin_elementwise_fma(f32x2{x, x}, w, acc);
}

template <bool PIPE>
__global__ __launch_bounds__(NT) void lstm_serve_kernel(LstmServeArgs a) {
  extern __shared__ __attribute__((aligned(16))) float smem_f[];
  // PIPE step counters and the zero h_{-1} row: static LDS, so volatile accesses stay ds_*
  // operations (a generic pointer into the dynamic block made them flat system-scope ones)
  __shared__ int s_rdy[MAXLSTM];
  __shared__ int s_prj[2];   // PIPE with projection waves: steps each layer's x-projection has published
  __shared__ __attribute__((aligned(16))) float s_zrow[MAXW];
  __shared__ __attribute__((aligned(16))) f32x2 s_zx[2][ZX_RING][64];   // x . W + b per lane, ring of steps
  Smem S;
  S.w = smem_f;
  const int nwp = (a.nw + 3) & ~3;
  S.seqa = S.w + nwp;
  S.seqb = S.seqa + MAXT * MAXW;
  S.v = S.seqb + MAXT * MAXW;
  S.z = S.v + 64;
  S.pred = S.z + 128;
  S.xrow = S.pred + MAXW;
  S.sc = S.xrow + MAXW;
  S.sh = S.sc + MAXW;
  S.ctl = reinterpret_cast<int*>(S.sh + MAXW);
  S.H = reinterpret_cast<float*>(S.ctl + 8);
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int half = lane >> 5;
  const int gate = wid * 32 + (lane & 31);
  const int D = a.D, T = a.T;
  for (int i = tid; i < a.nw; i += NT) S.w[i] = a.wts[i];
  for (int i = tid; i < MAXW; i += NT) {
    S.sc[i] = (i < D && a.scale) ? a.scale[i] : 1.f;
    S.sh[i] = (i < D && a.shift) ? a.shift[i] : 0.f;
  }
  if (tid < 64) S.v[tid] = 0.f;   // [x ; h] past I + u stays 0 (its weights are 0: no 0 * garbage)
  if (tid < 8) S.ctl[tid] = 0;
  if constexpr (PIPE) {
    // padded columns (past a layer's width) are read against zero weights: keep them 0
    for (int i = tid; i < MAXLSTM * MAXT * MAXW; i += NT) S.H[i] = 0.f;
    for (int i = tid; i < MAXT * MAXW; i += NT) S.seqa[i] = 0.f;
    if (tid < MAXW) s_zrow[tid] = 0.f;
  }
  __syncthreads();
  const int npipe = PIPE ? pipe_layers(a) : 0;
  // PIPE roles.  Stacks of one or two LSTM layers split every layer over two waves: wave l
  // runs layer l's recurrence (h_{t-1} . U + the gates), wave 2 + l its input projection
  // x_t . W + b, published per step through a ring in LDS -- the recurrence's critical chain
  // then holds only the u recurrent terms.  Deeper stacks: wave l does both for layer l.
  const bool split = npipe <= 2;
  const int role_layer = !PIPE ? -1 : wid < npipe ? wid : (split && wid >= 2 && wid - 2 < npipe) ? wid - 2 : -1;
  const bool role_proj = PIPE && split && wid >= 2;
  // PIPE: the role's layer, lane (p, j): wp[k] = ([W ; U][k][gate A], [W ; U][k][gate B]),
  // k < 32 input rows, 32 + k recurrent rows; gates A | B = i | g~ (p = 0), f | o (p = 1).
  // A split recurrence wave keeps only the U rows, a projection wave only the W rows and b.
  f32x2 wp[64], bp = {0.f, 0.f};
  if constexpr (PIPE) {
    if (role_layer >= 0) {
      const LstmServeLayer& L = a.L[role_layer];
      const bool want_w = !split || role_proj, want_u = !split || !role_proj;
      const int G = 4 * L.u, j = lane & 31, p = lane >> 5;
      const int ca = p * L.u + j, cb = (2 + p) * L.u + j;
      const bool ok = j < L.u;
      // Gate scales folded into the columns (both waves of a split layer load the same ones):
      // sigmoid gates i, f, o carry -log2(e), so sigm(z) = 1 / (1 + 2^z') is one v_exp + add +
      // v_rcp; a tanh layer's g~ carries -2 log2(e) (tanh(z) = 2 sigm(2z) - 1), so every lane
      // activates both of its gates with the same three instructions before the halves swap.
      // A relu layer's g~ stays unscaled.
      constexpr float L2E = 1.4426950408889634f;
      const float sa = -L2E, sb = p ? -L2E : (L.act == ACT_RELU ? 1.f : -2.f * L2E);
#pragma unroll
      for (int k = 0; k < 32; ++k) {
        wp[k] = (want_w && ok && k < L.in) ? f32x2{S.w[L.woff + k * G + ca] * sa, S.w[L.woff + k * G + cb] * sb}
                                           : f32x2{0.f, 0.f};
        wp[32 + k] = (want_u && ok && k < L.u)
                         ? f32x2{S.w[L.uoff + k * G + ca] * sa, S.w[L.uoff + k * G + cb] * sb}
                         : f32x2{0.f, 0.f};
      }
      if (want_w && ok) bp = f32x2{S.w[L.boff + ca] * sa, S.w[L.boff + cb] * sb};
    }
  }
  // register-resident weight halves of every LSTM layer: k = 32 * half + i of [W ; U]
  float wr[MAXLSTM][32], br[MAXLSTM];
  if constexpr (!PIPE) {
    int li = 0;
    for (int l = 0; l < a.nl; ++l) {
      const LstmServeLayer& L = a.L[l];
      if (L.kind != LS_LSTM) continue;
#pragma unroll
      for (int q = 0; q < MAXLSTM; ++q) {
        if (q != li) continue;
        const int G = 4 * L.u;
#pragma unroll
        for (int i = 0; i < 32; ++i) {
          const int k = 32 * half + i;
          float wv = 0.f;
          if (gate < G) {
            if (k < L.in) wv = S.w[L.woff + k * G + gate];
            else if (k - L.in < L.u) wv = S.w[L.uoff + (k - L.in) * G + gate];
          }
          wr[q][i] = wv;
        }
        br[q] = gate < G ? S.w[L.boff + gate] : 0.f;
      }
      ++li;
    }
  }

  uint64_t tail = ld_sys(&a.ctl->done);
  uint64_t last = __builtin_amdgcn_s_memrealtime();
  if (tid == 0) st_sys32(&a.ctl->alive, 1u);
  for (;;) {
    // ---------------- all four waves poll the next request slot, staggered by a quarter
    // of a PCIe round trip so their samples interleave.  Each poll is one synchronous
    // cache-bypassing load whose wait the compiler places (no load result is ever in flight
    // across statements: an asm-issued pipelined poll let the compiler copy a destination
    // register before its data landed).  The first wave that sees the whole request
    // publishes the row and key to LDS, then its sequence number; the others see that.
    const int slot = (int)(tail % (uint64_t)a.nslots);
    const uint32_t want = (uint32_t)(tail + 1);
    {
      typedef __attribute__((address_space(3))) volatile int lds_vint;   // ds_* accesses, not flat
      lds_vint* seen = (lds_vint*)&S.ctl[3];
      lds_vint* quit_f = (lds_vint*)&S.ctl[0];
      const uint64_t* wp = &a.req[slot].w[lane & 31];
      // ~0.25 / 0.5 / 0.75 us: s_sleep takes an immediate
      if (wid == 1) __builtin_amdgcn_s_sleep(10);
      else if (wid == 2) __builtin_amdgcn_s_sleep(20);
      else if (wid == 3) __builtin_amdgcn_s_sleep(30);
      for (uint32_t it = 0;; ++it) {
        if (*seen == (int)want || *quit_f) break;
        const uint64_t w = ld_sys(wp);
        const bool ok = (lane >= D && lane != KEY_WORD) || lane >= 32 || (uint32_t)(w >> 32) == want;
        if (__ballot(ok) == ~0ull) {
          if (lane < D) S.xrow[lane] = fmaf(__uint_as_float((uint32_t)w), S.sc[lane], S.sh[lane]);
          if (lane == KEY_WORD) S.ctl[1] = (int)(uint32_t)w;
          if (lane == 0) {
            const uint64_t ts = __builtin_amdgcn_s_memrealtime();
            S.ctl[4] = (int)(uint32_t)ts;
            S.ctl[5] = (int)(uint32_t)(ts >> 32);
          }
          asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // row and key before the sequence
          if (lane == 0) *seen = (int)want;
          break;
        }
        if ((it & 63) == 63 && wid == 0) {   // exit conditions every wave reaches
          if (ld_sys32(&a.ctl->stop) || __builtin_amdgcn_s_memrealtime() - last > a.idle_ticks) {
            if (lane == 0) *quit_f = 1;
            break;
          }
        }
      }
    }
    __syncthreads();
    if (S.ctl[0]) break;
    int key = S.ctl[1];
    key = key < 0 ? 0 : (key >= a.nkeys ? a.nkeys - 1 : key);   // the host validates; never leave the table
    float* hist = a.hist + (int64_t)key * T * D;
    float* lastp = a.lastpred + (int64_t)key * D;
    // events of this key before this one: read once, broadcast, so every wave takes the same
    // branches (the stack below has barriers).  The key's previous forecast is read in the
    // same round trip (used only once the key has T events), not after the count.
    float prev = 0.f;
    if (tid == 0) S.ctl[2] = ld_agent(&a.hcount[key]);
    if (tid >= 64 && tid < 64 + D) prev = ld_agent(&lastp[tid - 64]);
    // The key's whole window ring, in storage order, in the same round trip as its count: the
    // ring always holds the key's last T events, only its rotation depends on the count, so
    // the rows are placed (rotated) once the count is known instead of read after it.
    constexpr int WPT = MAXT * MAXW / NT;   // ring elements per thread (T * D <= MAXT * MAXW)
    float rv[WPT];
#pragma unroll
    for (int i = 0; i < WPT; ++i) rv[i] = (tid + i * NT < T * D) ? ld_agent(&hist[tid + i * NT]) : 0.f;
    if (tid >= 64 && tid < 64 + D) S.pred[tid - 64] = prev;   // parked until the count is known
    __syncthreads();
    const int cnt = S.ctl[2];
    const bool full = cnt + 1 >= T;
    // ---------------- append the event, score it against the previous forecast
    float err = 0.f;
    if (tid < D) {
      const float xn = S.xrow[tid];
      st_agent(&hist[(cnt % T) * D + tid], xn);
      if (cnt >= T) {
        const float d = xn - S.pred[tid];
        err = d * d;
      }
    }
    if (wid == 0) err = wave_sum(err);
    if (PIPE && tid < MAXLSTM) s_rdy[tid] = 0;
    if (PIPE && tid < 2) s_prj[tid] = 0;
    // ---------------- the window, oldest first, into seqa [t][k] (the newest row from LDS)
    if (full) {
      // storage slot r holds events n = r (mod T); window step t holds event cnt + 1 - T + t, so
      // t = (r - cnt - 1) mod T, and step T - 1 is this event (its slot still holds the evicted one)
      const int rot = (cnt + 1) % T;
#pragma unroll
      for (int i = 0; i < WPT; ++i) {
        const int e = tid + i * NT;
        if (e < T * D) {
          const int r = e / D, k = e - r * D;
          const int t = r >= rot ? r - rot : r - rot + T;
          S.seqa[t * MAXW + k] = t == T - 1 ? S.xrow[k] : rv[i];
        }
      }
    }
    __syncthreads();
    const uint64_t t_rec = __builtin_amdgcn_s_memrealtime();   // key state + window gathered
    if (PIPE && full) {
      // the wave's layer as a scalar: layer fields in SGPRs, uniform branches
      const int lw = __builtin_amdgcn_readfirstlane(wid);
      typedef __attribute__((address_space(3))) volatile int lds_vint;
      lds_vint* rdy = (lds_vint*)s_rdy;   // ds_read / ds_write, never a flat access
      lds_vint* prj = (lds_vint*)s_prj;
      // Dot products run over a compile-time number of float4 input groups (4 or 8; the
      // padded columns and their weights are zero): a runtime trip count under `#pragma
      // unroll` became a v_cndmask per accumulator per group (8 selects per 4 packed FMAs).
      using I4 = std::integral_constant<int, 4>;
      using I8 = std::integral_constant<int, 8>;
      if (split && lw >= 2 && lw - 2 < npipe) {
        // ---- input projection of layer pl: zx_t = x_t . W + b into the ring
        const int pl = lw - 2;
        const LstmServeLayer& L = a.L[pl];
        const float* xin = pl == 0 ? S.seqa : S.H + (pl - 1) * MAXT * MAXW;
        auto project = [&](auto ni4c) {
          constexpr int NI4 = decltype(ni4c)::value;
          int below = pl > 0 ? 0 : T, freed = ZX_RING;   // producer / consumer counters seen
          for (int t = 0; t < T; ++t) {
            if (below <= t || freed <= t) {
              if (pl > 0)   // the layer below has published h_t
                while ((below = rdy[pl - 1]) <= t) {
                }
              // ring slot free: the recurrence has finished step t - ZX_RING
              while ((freed = rdy[pl] + ZX_RING) <= t) {
              }
              __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
            }
            const float4* x4 = reinterpret_cast<const float4*>(xin + t * MAXW);
            float4 xv[NI4];
#pragma unroll
            for (int k4 = 0; k4 < NI4; ++k4) xv[k4] = x4[k4];
            f32x2 acc[4] = {bp, {0.f, 0.f}, {0.f, 0.f}, {0.f, 0.f}};
#pragma unroll
            for (int k4 = 0; k4 < NI4; ++k4) {
              acc[0] = fma2(xv[k4].x, wp[4 * k4 + 0], acc[0]);
              acc[1] = fma2(xv[k4].y, wp[4 * k4 + 1], acc[1]);
              acc[2] = fma2(xv[k4].z, wp[4 * k4 + 2], acc[2]);
              acc[3] = fma2(xv[k4].w, wp[4 * k4 + 3], acc[3]);
            }
            s_zx[pl][t % ZX_RING][lane] = (acc[0] + acc[1]) + (acc[2] + acc[3]);
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
            if (lane == 0) prj[pl] = t + 1;
          }
        };
        if (L.in > 16) project(I8{});
        else project(I4{});
      } else if (lw < npipe) {
        const LstmServeLayer& L = a.L[lw];
        const int u = L.u;
        const float* xin = lw == 0 ? S.seqa : S.H + (lw - 1) * MAXT * MAXW;
        float* hout = S.H + lw * MAXT * MAXW;
        // NI4: input groups of the x . W part (0: split, the projection wave does it); NU4: of h . U
        auto recur = [&](auto ni4c, auto nu4c, auto reluc) {
          constexpr int NI4 = decltype(ni4c)::value, NU4 = decltype(nu4c)::value;
          constexpr bool RELU = decltype(reluc)::value;
          float c = 0.f;   // a tanh layer carries c scaled by 2 log2(e) (below)
          int avail = 0;   // steps the producer (projection ring or the layer below) has published
          for (int t = 0; t < T; ++t) {
            // The producer runs ahead, so its counter is re-read only once the steps already
            // seen are used up: no LDS round trip on the recurrence's chain in the common case.
            if (avail <= t) {
              if (NI4 == 0) {   // this step's input projection is in the ring
                while ((avail = prj[lw]) <= t) {
                }
              } else if (lw > 0) {   // the layer below has published h_t
                while ((avail = rdy[lw - 1]) <= t) {
                }
              } else {
                avail = T;
              }
              __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
            }
            // every LDS read first (padded columns are zero), then the FMAs: one LDS wait per step
            const float4* x4 = reinterpret_cast<const float4*>(xin + t * MAXW);
            const float4* h4 = reinterpret_cast<const float4*>(t > 0 ? hout + (t - 1) * MAXW : s_zrow);
            float4 xv[NI4 ? NI4 : 1], hv[NU4];
            f32x2 acc[4];   // four chains: at most 8 + 8 dependent packed FMAs each, under the issue time
            if constexpr (NI4 == 0) {
              acc[0] = s_zx[lw][t % ZX_RING][lane];
            } else {
              acc[0] = bp;
#pragma unroll
              for (int k4 = 0; k4 < NI4; ++k4) xv[k4] = x4[k4];
            }
#pragma unroll
            for (int k4 = 0; k4 < NU4; ++k4) hv[k4] = h4[k4];
#pragma unroll
            for (int q = 1; q < 4; ++q) acc[q] = f32x2{0.f, 0.f};
#pragma unroll
            for (int k4 = 0; k4 < NI4; ++k4) {
              acc[0] = fma2(xv[k4].x, wp[4 * k4 + 0], acc[0]);
              acc[1] = fma2(xv[k4].y, wp[4 * k4 + 1], acc[1]);
              acc[2] = fma2(xv[k4].z, wp[4 * k4 + 2], acc[2]);
              acc[3] = fma2(xv[k4].w, wp[4 * k4 + 3], acc[3]);
            }
#pragma unroll
            for (int k4 = 0; k4 < NU4; ++k4) {
              acc[0] = fma2(hv[k4].x, wp[32 + 4 * k4 + 0], acc[0]);
              acc[1] = fma2(hv[k4].y, wp[32 + 4 * k4 + 1], acc[1]);
              acc[2] = fma2(hv[k4].z, wp[32 + 4 * k4 + 2], acc[2]);
              acc[3] = fma2(hv[k4].w, wp[32 + 4 * k4 + 3], acc[3]);
            }
            const f32x2 z = (acc[0] + acc[1]) + (acc[2] + acc[3]);   // scaled pre-activations
            // Each lane activates its own two gates, then ONE swap per value brings the (f, o)
            // of lane + 32 to the p = 0 lanes (the only ones that keep c and write h):
            //   p = 0: ea = sigm(i), eb = sigm(2 g~) (tanh layer; unused by relu)
            //   p = 1: ea = sigm(f), eb = sigm(o)
            const float ea = rcp_fast(1.f + __builtin_amdgcn_exp2f(z.x));
            const float eb = rcp_fast(1.f + __builtin_amdgcn_exp2f(z.y));
            const float fg = __uint_as_float(
                __builtin_amdgcn_permlane32_swap(__float_as_uint(ea), __float_as_uint(ea), false, false)[1]);
            const float og = __uint_as_float(
                __builtin_amdgcn_permlane32_swap(__float_as_uint(eb), __float_as_uint(eb), false, false)[1]);
            float h;
            if constexpr (RELU) {
              c = fmaf(fg, c, ea * relu_fast(z.y));
              h = og * relu_fast(c);
            } else {
              // c' = K c with K = 2 log2(e): c' = f c' + i (K tanh(g~)), K tanh(g~) = 2K sigm(2g~) - K,
              // and tanh(c) = 1 - 2 / (1 + 2^c'), so h = o - 2 o / (1 + 2^c')
              constexpr float K = 2.8853900817779268f;
              c = fmaf(fg, c, ea * fmaf(eb, 2.f * K, -K));
              h = fmaf(-2.f * og, rcp_fast(1.f + __builtin_amdgcn_exp2f(c)), og);
            }
            if (lane < u) hout[t * MAXW + lane] = h;
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
            if (lane == 0) rdy[lw] = t + 1;
          }
        };
        auto with_u = [&](auto ni4c, auto reluc) {
          if (u > 16) recur(ni4c, I8{}, reluc);
          else recur(ni4c, I4{}, reluc);
        };
        auto with_i = [&](auto reluc) {
          if (split) with_u(std::integral_constant<int, 0>{}, reluc);
          else if (L.in > 16) with_u(I8{}, reluc);
          else with_u(I4{}, reluc);
        };
        if (L.act == ACT_RELU) with_i(std::true_type{});
        else with_i(std::false_type{});
        if (lw == npipe - 1) {   // Dense head on h_{T-1}
          const LstmServeLayer& Hd = a.L[npipe];
          const float* hl = hout + (T - 1) * MAXW;
          if (lane < Hd.u) {
            float acc = S.w[Hd.boff + lane];
#pragma unroll
            for (int k = 0; k < 32; ++k)
              if (k < Hd.in) acc = fmaf(hl[k], S.w[Hd.woff + k * Hd.u + lane], acc);
            S.pred[lane] = acc;
          }
        }
      }
      __syncthreads();
    } else if (full) {
      float* cur = S.seqa;
      float* nxt = S.seqb;
      int tcur = T, dim = D, li = 0;
      for (int l = 0; l < a.nl; ++l) {
        const LstmServeLayer& L = a.L[l];
        if (L.kind == LS_LSTM) {
          const int I = L.in, u = L.u, G = 4 * u;
          float c = 0.f, h = 0.f;
          if (tid < u) S.v[I + tid] = 0.f;
          for (int t = 0; t < tcur; ++t) {
            if (tid < I) S.v[tid] = cur[t * MAXW + tid];
            __syncthreads();
            float s = 0.f;
#pragma unroll
            for (int q = 0; q < MAXLSTM; ++q) {
              if (q != li) continue;
              const float4* v4 = reinterpret_cast<const float4*>(S.v + 32 * half);
#pragma unroll
              for (int i4 = 0; i4 < 8; ++i4) {
                const float4 vv = v4[i4];
                s = fmaf(vv.x, wr[q][4 * i4 + 0], s);
                s = fmaf(vv.y, wr[q][4 * i4 + 1], s);
                s = fmaf(vv.z, wr[q][4 * i4 + 2], s);
                s = fmaf(vv.w, wr[q][4 * i4 + 3], s);
              }
              s += xor32(s, lane) + br[q];
            }
            if (half == 0 && gate < G) S.z[gate] = s;
            __syncthreads();
            if (tid < u) {
              const float ig = sigm(S.z[tid]), fg = sigm(S.z[u + tid]);
              const float gg = act_lstm(L.act, S.z[2 * u + tid]), og = sigm(S.z[3 * u + tid]);
              c = fmaf(fg, c, ig * gg);
              h = og * act_lstm(L.act, c);
              S.v[I + tid] = h;
              if (L.ret) nxt[t * MAXW + tid] = h;
            }
          }
          if (!L.ret && tid < u) nxt[tid] = h;
          tcur = L.ret ? tcur : 1;
          dim = u;
          ++li;
        } else if (L.kind == LS_REPEAT) {
          for (int e = tid; e < L.n * dim; e += NT) {
            const int t = e / dim, k = e - t * dim;
            nxt[t * MAXW + k] = cur[k];   // cur holds one vector (the previous layer's h_T)
          }
          tcur = L.n;
        } else {   // dense / TimeDistributed(Dense): only the last step is the forecast
          const int U = L.u;
          if (tid < U) {
            float acc = S.w[L.boff + tid];
            const float* xin = cur + (tcur - 1) * MAXW;
            // unrolled to the widest input: every LDS read is issued before the FMA chain
#pragma unroll
            for (int k = 0; k < MAXW; ++k)
              if (k < dim) acc = fmaf(xin[k], S.w[L.woff + k * U + tid], acc);
            nxt[(tcur - 1) * MAXW + tid] = acc;
            if (l == a.nl - 1) S.pred[tid] = acc;
          }
          dim = U;
        }
        __syncthreads();
        float* tmp = cur;
        cur = nxt;
        nxt = tmp;
      }
    }
    const uint64_t t_comp = __builtin_amdgcn_s_memrealtime();
    const uint64_t t_seen = (uint64_t)(uint32_t)S.ctl[4] | ((uint64_t)(uint32_t)S.ctl[5] << 32);
    // ---------------- results (wave 0), the key's state, completion counter
    if (wid == 0) {
      ServeResult* r = a.res + slot;
      const float p = (full && lane < D) ? S.pred[lane] : 0.f;
      if (lane < D) {
        st_sys(&r->w[lane], tagged(want, p));
        if (full) st_agent(&lastp[lane], p);
      }
      if (lane == 0) {
        const float score = cnt >= T ? err / (float)D : __builtin_nanf("");
        const uint32_t flag = cnt >= T ? (score > a.threshold ? 1u : 0u) : 2u;
        st_agent(&a.hcount[key], cnt + 1);
        st_sys(&r->w[kServeScore], tagged(want, score));
        st_sys(&r->w[kServeFlag], tagged_u(want, flag));
        st_sys(&r->w[kServeTLoad], tagged_u(want, (uint32_t)(t_rec - t_seen)));
        st_sys(&r->w[kServeTComp], tagged_u(want, (uint32_t)(t_comp - t_seen)));
        st_sys(&r->w[kServeTDone], tagged_u(want, (uint32_t)(__builtin_amdgcn_s_memrealtime() - t_seen)));
        st_sys(&a.ctl->done, tail + 1);
      }
    }
    tail += 1;
    last = __builtin_amdgcn_s_memrealtime();
    __syncthreads();   // key state stored before the next event may read it
  }
  __syncthreads();
  wait_stores();
  if (tid == 0) st_sys32(&a.ctl->alive, 0u);
}


// ===================================================================================
// The reference stack at look_back 1 (LSTM-TensorFlow-IO-Kafka/cardata-v2.py:172-209:
// LSTM 32 -> LSTM 16 -> RepeatVector(1) -> LSTM 16 -> LSTM 32 -> TimeDistributed(Dense 18)).
// With a one-event window every LSTM runs one step from h0 = c0 = 0, so only the i, g~, o
// columns of each kernel matter and the whole forecast is a nine-stage chain of small dot
// products.  ONE wave does all of it, with every weight it multiplies held in registers
// for the kernel's life: lane l = j + U * part owns unit j of a U-unit layer and every
// P-th input (P = 64 / U); the partial sums meet through permlane swaps, and a layer's
// output passes to the next through LDS (one wave: no barrier, LDS operations complete in
// order), written part-major so the consumer's inputs are 16-byte reads.  The key's event
// count and previous forecast are requested right after the request is picked up and are
// first needed after the chain, so their global round trip hides under it.
// ===================================================================================
constexpr int R1F = 18, R1U1 = 32, R1U2 = 16, R1U3 = 16, R1U4 = 32;

template <int U>
__device__ __forceinline__ float r1_part_sum(float v, int lane) {
  if (U == 16) v += xor16(v, lane);
  return v + xor32(v, lane);
}
template <int RELU>
__device__ __forceinline__ float r1_act(float z) { return RELU ? fmaxf(z, 0.f) : tanh_fast(z); }

// this lane's weights of one LSTM layer (K inputs, U units): w[3i + g] = W[k = part + P i][gate g],
// gates i | g~ | o (Keras columns 0, 2U, 3U), then the 3 biases (part 0; 0 elsewhere)
template <int K, int U, int NW>
__device__ __forceinline__ void r1_load_lstm(const float* wts, const LstmServeLayer& L, int lane, float (&w)[NW]) {
  constexpr int P = 64 / U, KP = K / P;
  static_assert(NW == 3 * KP + 3 && K % P == 0, "image shape");
  const int j = lane % U, part = lane / U;
#pragma unroll
  for (int i = 0; i < KP; ++i) {
    const int k = part + P * i;
    w[3 * i + 0] = wts[L.woff + k * 4 * U + j];
    w[3 * i + 1] = wts[L.woff + k * 4 * U + 2 * U + j];
    w[3 * i + 2] = wts[L.woff + k * 4 * U + 3 * U + j];
  }
  w[3 * KP + 0] = part == 0 ? wts[L.boff + j] : 0.f;
  w[3 * KP + 1] = part == 0 ? wts[L.boff + 2 * U + j] : 0.f;
  w[3 * KP + 2] = part == 0 ? wts[L.boff + 3 * U + j] : 0.f;
}

template <int KP, int U, int RELU, int NW, int NI>
__device__ __forceinline__ float r1_unit(const float (&w)[NW], const float (&in)[NI], int lane) {
  float zi = w[3 * KP], zg = w[3 * KP + 1], zo = w[3 * KP + 2];
#pragma unroll
  for (int i = 0; i < KP; ++i) {
    zi = fmaf(in[i], w[3 * i], zi);
    zg = fmaf(in[i], w[3 * i + 1], zg);
    zo = fmaf(in[i], w[3 * i + 2], zo);
  }
  zi = r1_part_sum<U>(zi, lane);
  zg = r1_part_sum<U>(zg, lane);
  zo = r1_part_sum<U>(zo, lane);
  return sigm(zo) * r1_act<RELU>(sigm(zi) * r1_act<RELU>(zg));   // c = i * g~ (c0 = 0), h = o * act(c)
}

// h[j] of part-0 lanes into the consumer's part-major copy (PC parts of KPC), others to the sink
template <int PC, int KPC>
__device__ __forceinline__ void r1_put(float* q, float* sink, int j, int part, int lane, float h) {
  constexpr int RUN = (KPC + 3) & ~3;
  float* dst = part == 0 ? q + (j % PC) * RUN + j / PC : sink + lane;
  *dst = h;
  asm volatile("" ::: "memory");
}
template <int N>
__device__ __forceinline__ void r1_vec(const float* v, float (&o)[N]) {
#pragma unroll
  for (int i = 0; i < N; i += 4) {
    const float4 t = *reinterpret_cast<const float4*>(v + i);
    o[i] = t.x;
    o[i + 1] = t.y;
    o[i + 2] = t.z;
    o[i + 3] = t.w;
  }
}

template <int RELU>
__global__ __launch_bounds__(64) void lstm_serve_ref1_kernel(LstmServeArgs a) {
  constexpr int P1 = 64 / R1U1, P2 = 64 / R1U2, P3 = 64 / R1U3, P4 = 64 / R1U4;
  constexpr int K1 = R1F / P1, K2 = R1U1 / P2, K3 = R1U2 / P3, K4 = R1U3 / P4, KH = R1U4 / 2;
  __shared__ __attribute__((aligned(16))) float xrow[32], q1[64], q2[64], q3[64], q4[64], sink[64], sc[32], sh[32];
  const int lane = threadIdx.x;
  const int D = a.D;
  sc[lane & 31] = ((lane & 31) < D && a.scale) ? a.scale[lane & 31] : 1.f;
  sh[lane & 31] = ((lane & 31) < D && a.shift) ? a.shift[lane & 31] : 0.f;
  // every weight this lane multiplies, for the kernel's life (~120 registers)
  float w1[3 * K1 + 3], w2[3 * K2 + 3], w3[3 * K3 + 3], w4[3 * K4 + 3], wh[KH + 1];
  r1_load_lstm<R1F, R1U1>(a.wts, a.L[0], lane, w1);
  r1_load_lstm<R1U1, R1U2>(a.wts, a.L[1], lane, w2);
  r1_load_lstm<R1U2, R1U3>(a.wts, a.L[3], lane, w3);
  r1_load_lstm<R1U3, R1U4>(a.wts, a.L[4], lane, w4);
  {  // head: lane f + 32 * part, k = part + 2 i
    const int f = lane & 31, part = lane >> 5;
    const LstmServeLayer& H = a.L[5];
#pragma unroll
    for (int i = 0; i < KH; ++i) wh[i] = f < R1F ? a.wts[H.woff + (part + 2 * i) * R1F + f] : 0.f;
    wh[KH] = (f < R1F && part == 0) ? a.wts[H.boff + f] : 0.f;
  }
  const int j1 = lane % R1U1, p1 = lane / R1U1, j2 = lane % R1U2, p2 = lane / R1U2;
  const int j3 = lane % R1U3, p3 = lane / R1U3, j4 = lane % R1U4, p4 = lane / R1U4;
  __syncthreads();

  uint64_t tail = ld_sys(&a.ctl->done);
  uint64_t last = __builtin_amdgcn_s_memrealtime();
  if (lane == 0) st_sys32(&a.ctl->alive, 1u);
  for (;;) {
    const int slot = (int)(tail % (uint64_t)a.nslots);
    const uint32_t want = (uint32_t)(tail + 1);
    bool quit = false;
    uint32_t keyw = 0;
    uint64_t t_seen = 0;
    {
      const uint64_t* wp = &a.req[slot].w[lane & 31];
      for (uint32_t it = 0;; ++it) {
        const uint64_t w = ld_sys(wp);
        const bool ok = (lane >= D && lane != KEY_WORD) || lane >= 32 || (uint32_t)(w >> 32) == want;
        if (__ballot(ok) == ~0ull) {
          t_seen = __builtin_amdgcn_s_memrealtime();
          if (lane < D) xrow[lane] = fmaf(__uint_as_float((uint32_t)w), sc[lane], sh[lane]);
          keyw = (uint32_t)__shfl((int)(uint32_t)w, KEY_WORD);
          break;
        }
        if ((it & 63) == 63 &&
            (ld_sys32(&a.ctl->stop) || __builtin_amdgcn_s_memrealtime() - last > a.idle_ticks)) {
          quit = true;
          break;
        }
      }
    }
    if (quit) break;
    int key = (int)keyw;
    key = key < 0 ? 0 : (key >= a.nkeys ? a.nkeys - 1 : key);   // the host validates; never leave the table
    // the key's state: requested now, first used after the chain
    const int cnt = ld_agent(&a.hcount[key]);
    const float prev = lane < D ? ld_agent(&a.lastpred[(int64_t)key * D + lane]) : 0.f;
    asm volatile("" ::: "memory");
    // ---------------- the chain
    float x[K1];
#pragma unroll
    for (int i = 0; i < K1; ++i) x[i] = xrow[p1 + P1 * i];
    r1_put<P2, K2>(q1, sink, j1, p1, lane, r1_unit<K1, R1U1, RELU>(w1, x, lane));
    float in2[(K2 + 3) & ~3];
    r1_vec(q1 + p2 * ((K2 + 3) & ~3), in2);
    r1_put<P3, K3>(q2, sink, j2, p2, lane, r1_unit<K2, R1U2, RELU>(w2, in2, lane));
    float in3[(K3 + 3) & ~3];
    r1_vec(q2 + p3 * ((K3 + 3) & ~3), in3);
    r1_put<P4, K4>(q3, sink, j3, p3, lane, r1_unit<K3, R1U3, RELU>(w3, in3, lane));
    float in4[(K4 + 3) & ~3];
    r1_vec(q3 + p4 * ((K4 + 3) & ~3), in4);
    r1_put<2, KH>(q4, sink, j4, p4, lane, r1_unit<K4, R1U4, RELU>(w4, in4, lane));
    float inh[KH];
    r1_vec(q4 + (lane >> 5) * ((KH + 3) & ~3), inh);
    float acc = wh[KH];
#pragma unroll
    for (int i = 0; i < KH; ++i) acc = fmaf(inh[i], wh[i], acc);
    const float pred = acc + xor32(acc, lane);   // lanes f < D (either half) hold forecast f
    const uint64_t t_comp = __builtin_amdgcn_s_memrealtime();
    // ---------------- score against the previous forecast, results, the key's state
    float err = 0.f;
    if (lane < D && cnt >= 1) {
      const float d = xrow[lane] - prev;
      err = d * d;
    }
    err = wave_sum(err);
    ServeResult* r = a.res + slot;
    if (lane < D) {
      st_sys(&r->w[lane], tagged(want, pred));
      st_agent(&a.lastpred[(int64_t)key * D + lane], pred);
      st_agent(&a.hist[(int64_t)key * a.T * D + lane], xrow[lane]);
    }
    if (lane == 0) {
      const float score = cnt >= 1 ? err / (float)D : __builtin_nanf("");
      const uint32_t flag = cnt >= 1 ? (score > a.threshold ? 1u : 0u) : 2u;
      st_agent(&a.hcount[key], cnt + 1);
      st_sys(&r->w[kServeScore], tagged(want, score));
      st_sys(&r->w[kServeFlag], tagged_u(want, flag));
      st_sys(&r->w[kServeTLoad], tagged_u(want, 0u));
      st_sys(&r->w[kServeTComp], tagged_u(want, (uint32_t)(t_comp - t_seen)));
      st_sys(&r->w[kServeTDone], tagged_u(want, (uint32_t)(__builtin_amdgcn_s_memrealtime() - t_seen)));
      st_sys(&a.ctl->done, tail + 1);
    }
    tail += 1;
    last = __builtin_amdgcn_s_memrealtime();
  }
  wait_stores();
  if (lane == 0) st_sys32(&a.ctl->alive, 0u);
}

// the launch arguments describe exactly the reference stack at look_back 1
bool lstm_serve_is_ref1(const LstmServeArgs& x) {
  if (x.T != 1 || x.D != R1F || x.nl != 6) return false;
  const LstmServeLayer* L = x.L;
  const bool shape = L[0].kind == LS_LSTM && L[0].in == R1F && L[0].u == R1U1 && L[1].kind == LS_LSTM &&
                     L[1].in == R1U1 && L[1].u == R1U2 && L[1].ret == 0 && L[2].kind == LS_REPEAT && L[2].n == 1 &&
                     L[3].kind == LS_LSTM && L[3].in == R1U2 && L[3].u == R1U3 && L[4].kind == LS_LSTM &&
                     L[4].in == R1U3 && L[4].u == R1U4 && L[5].kind == LS_DENSE && L[5].in == R1U4 && L[5].u == R1F;
  const int act = L[0].act;
  return shape && (act == ACT_RELU || act == ACT_TANH) && L[1].act == act && L[3].act == act && L[4].act == act;
}
}  // namespace

size_t lstm_serve_lds_bytes(int nw) {
  const int nwp = (nw + 3) & ~3;
  return (size_t)(nwp + 2 * MAXT * MAXW + 64 + 128 + 4 * MAXW) * sizeof(float) + 8 * sizeof(int) +
         (size_t)MAXLSTM * MAXT * MAXW * sizeof(float) + MAXLSTM * sizeof(int);   // PIPE sequences + counters
}

hipError_t lstm_serve_launch(const LstmServeArgs& args, hipStream_t stream) {
  // shape contract of the kernel (also checked by the host class): every layer fits
  if (args.D < 1 || args.D > 31 || args.T < 1 || args.T > MAXT || args.nl < 1 || args.nl > LS_MAXLAYERS ||
      args.nslots < 64 || args.nkeys < 1)
    return hipErrorInvalidValue;
  int nlstm = 0, dim = args.D, tlen = args.T;
  for (int l = 0; l < args.nl; ++l) {
    const LstmServeLayer& L = args.L[l];
    if (L.kind == LS_LSTM) {
      if (L.in != dim || L.u < 1 || L.u > 32 || L.in > 32 || ++nlstm > MAXLSTM) return hipErrorInvalidValue;
      dim = L.u;
      tlen = L.ret ? tlen : 1;
    } else if (L.kind == LS_REPEAT) {
      if (tlen != 1 || L.n < 1 || L.n > MAXT) return hipErrorInvalidValue;
      tlen = L.n;
    } else if (L.kind == LS_DENSE) {
      if (L.in != dim || L.u < 1 || L.u > MAXW) return hipErrorInvalidValue;
      dim = L.u;
    } else {
      return hipErrorInvalidValue;
    }
  }
  if (args.L[args.nl - 1].kind != LS_DENSE || dim != args.D) return hipErrorInvalidValue;
  // the reference stack at look_back 1 takes the one-wave register-resident path, unless
  // SML_LSTM_SERVE_GENERIC=1 asks for the general kernel (A/B and cross-checks)
  const char* gen = getenv("SML_LSTM_SERVE_GENERIC");
  if (lstm_serve_is_ref1(args) && !(gen && gen[0] == '1')) {
    auto k = args.L[0].act == ACT_RELU ? lstm_serve_ref1_kernel<1> : lstm_serve_ref1_kernel<0>;
    hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, stream, args);
    return hipGetLastError();
  }
  const size_t lds = lstm_serve_lds_bytes(args.nw);
  if (lds + 9 * 1024 > 160 * 1024) return hipErrorInvalidValue;   // + the PIPE kernel's static LDS (8.2 KB)
  // stacks of LSTM layers under one Dense head: the pipelined variant (one wave per layer);
  // SML_LSTM_SERVE_GENERIC=1 keeps the barrier-per-step kernel (A/B, cross-checks)
  const bool pipe = pipe_layers(args) > 0 && !(gen && gen[0] == '1');
  auto kern = pipe ? lstm_serve_kernel<true> : lstm_serve_kernel<false>;
  if (lds > 65536) {
    const hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(kern),
                                             hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return e;
  }
  hipLaunchKernelGGL(kern, dim3(1), dim3(NT), lds, stream, args);
  return hipGetLastError();
}

}  // namespace sml
