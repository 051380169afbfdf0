// Persistent per-event anomaly scorer (BASELINE config 5).
//
// The reference scores events through model.predict on tf.data batches and a
// Python OutputCallback (cardata-v3.py:235-280); per-event latency is not even
// measurable there.  The launch-per-event path here (H2D copy + fused forward
// kernel + D2H copy) costs three runtime round trips per event.  This kernel
// removes all of them: ONE wave stays resident and polls the host-mapped request
// ring (fine-grained pinned memory, cache-bypassing system-scope loads).
//
// Slots are LL-framed (sml_ops.h): each 8-byte word is 4 payload bytes + a 4-byte
// event tag.  The wave polls the next slot's words THEMSELVES, so the poll that finds
// the event also delivers its row -- no separate "head moved, now fetch the row" PCIe
// round trip -- and it writes tagged result words that the host polls in its own
// memory, so there is no wait for the stores' acknowledgement either.  A single
// event (the common case at a fixed QPS) is spread over 16 lanes, one output unit
// each; a backlog of more than 4 (seen through the host's head counter) is scored one
// event per lane, up to 64 per pass.
//
// Weights (Keras order W1 b1 .. W4 b4, <= 31/15/15/15 units) and the input
// normaliser live in LDS; every lane reads the same weight address, so the LDS
// reads are broadcasts.
//
// Exit conditions every wave reaches: the host's stop flag, or `idle_us` without
// a request (measured on the 100 MHz s_memrealtime counter) -- a forgotten
// server never keeps the GPU busy, and the host relaunches on demand.
#include "sml_common.h"
#include "sml_ops.h"
#include "sml_serve_dev.h"

namespace sml {
namespace {

constexpr int MAXD = 32, MAXH = 16;

using namespace serve_dev;

template <int IN, int OUT>
__device__ __forceinline__ void dense_lane(const float* __restrict__ W, const float* __restrict__ b, int in_n,
                                           int out_n, const float* x, float* y, int act) {
#pragma unroll
  for (int o = 0; o < OUT; ++o) {
    float acc = 0.f;
    if (o < out_n) {
      acc = b[o];
#pragma unroll
      for (int i = 0; i < IN; ++i)
        if (i < in_n) acc = fmaf(x[i], W[i * out_n + o], acc);
      acc = act_fwd(act, acc);
    }
    y[o] = acc;
  }
}

// CD / C1 / C2 > 0 fix (D, n1, n2) at compile time (compact straight-line code for
// the reference configs: car data 18-14-7, credit card 30-14-7); 0 = runtime dims.
template <int CD, int C1, int C2>
__global__ __launch_bounds__(64) void ae_serve_kernel(ServeCtl* ctl, const ServeReq* __restrict__ req,
                                                       ServeResult* res, int nslots, const float* __restrict__ wts,
                                                       const float* __restrict__ scale,
                                                       const float* __restrict__ shift, int D_, int n1_, int n2_,
                                                       int a1, int a2, int a3, int a4, float threshold,
                                                       uint64_t idle_ticks) {
  constexpr int XD = CD > 0 ? CD : MAXD, X1 = C1 > 0 ? C1 : MAXH, X2 = C2 > 0 ? C2 : MAXH;
  const int D = CD > 0 ? CD : D_, n1 = C1 > 0 ? C1 : n1_, n2 = C2 > 0 ? C2 : n2_;
  __shared__ float lw[MAXD * MAXH + MAXH + MAXH * MAXH + MAXH + MAXH * MAXH + MAXH + MAXH * MAXD + MAXD];
  __shared__ float lsc[MAXD], lsh[MAXD];
  const int lane = threadIdx.x;
  const int nw = D * n1 + n1 + n1 * n2 + n2 + n2 * n2 + n2 + n2 * D + D;
  for (int i = lane; i < nw; i += 64) lw[i] = wts[i];
  for (int i = lane; i < D; i += 64) {
    lsc[i] = scale ? scale[i] : 1.f;
    lsh[i] = shift ? shift[i] : 0.f;
  }
  __syncthreads();
  const float* W1 = lw;
  const float* b1 = W1 + D * n1;
  const float* W2 = b1 + n1;
  const float* b2 = W2 + n1 * n2;
  const float* W3 = b2 + n2;
  const float* b3 = W3 + n2 * n2;
  const float* W4 = b3 + n2;
  const float* b4 = W4 + n2 * D;
  // latency path: lane u keeps column u of every layer's weights (and its biases) in registers
  float rw1[XD], rw2[X1], rw3[X2], rw4[X2], rb[4];
#pragma unroll
  for (int i = 0; i < XD; ++i) rw1[i] = (i < D && lane < n1) ? W1[i * n1 + lane] : 0.f;
#pragma unroll
  for (int i = 0; i < X1; ++i) rw2[i] = (i < n1 && lane < n2) ? W2[i * n2 + lane] : 0.f;
#pragma unroll
  for (int i = 0; i < X2; ++i) rw3[i] = (i < n2 && lane < n2) ? W3[i * n2 + lane] : 0.f;
#pragma unroll
  for (int i = 0; i < X2; ++i) rw4[i] = (i < n2 && lane < D) ? W4[i * D + lane] : 0.f;
  rb[0] = lane < n1 ? b1[lane] : 0.f;
  rb[1] = lane < n2 ? b2[lane] : 0.f;
  rb[2] = lane < n2 ? b3[lane] : 0.f;
  rb[3] = lane < D ? b4[lane] : 0.f;

  uint64_t tail = ld_sys(&ctl->done);
  uint64_t last = __builtin_amdgcn_s_memrealtime();
  if (lane == 0) st_sys32(&ctl->alive, 1u);
  bool quit = false;
  while (!quit) {
    // Pipelined polling: three polls of the next slot (word `lane` + the head counter)
    // in flight, spaced about a third of a PCIe round trip apart, so an event is seen
    // ~RTT/3 after its row lands instead of up to a whole round trip later.  Each
    // consumed poll is re-issued at once, which keeps the spacing.  The polls are issued
    // and waited for by separate asm statements, so the compiler may copy a poll register
    // before its data lands (a loop phi copy; lstm_serve.hip was bitten by it): that is
    // harmless here because the tag and the payload are the SAME 8-byte word -- a stale
    // copy can only fail the tag test (the wave polls again), never pair a new tag with
    // old data -- and the row used afterwards is exactly the word that passed the test.
    const int slot0 = (int)(tail % (uint64_t)nslots);
    SML_DCHECK(slot0 >= 0 && slot0 < nslots);
    const uint32_t want = (uint32_t)(tail + 1);
    const uint64_t* wp = &req[slot0].w[lane & (MAXD - 1)];
    const uint64_t* hp = &ctl->head;
    uint64_t w0, h0, w1, h1, w2, h2;
    poll_issue(w0, h0, wp, hp);
    __builtin_amdgcn_s_sleep(8);
    poll_issue(w1, h1, wp, hp);
    __builtin_amdgcn_s_sleep(8);
    poll_issue(w2, h2, wp, hp);
    uint64_t wv = 0, head = 0;
    auto ready = [&](uint64_t w, uint64_t hd) {
      const bool ok = lane >= D || (uint32_t)(w >> 32) == want;
      return __ballot(ok) == ~0ull || hd > tail + 4;
    };
    for (uint32_t it = 0;; ++it) {
      asm volatile("s_waitcnt vmcnt(4)" : "+v"(w0), "+v"(h0)::"memory");
      if (ready(w0, h0)) { wv = w0; head = h0; break; }
      poll_issue(w0, h0, wp, hp);
      asm volatile("s_waitcnt vmcnt(4)" : "+v"(w1), "+v"(h1)::"memory");
      if (ready(w1, h1)) { wv = w1; head = h1; break; }
      poll_issue(w1, h1, wp, hp);
      asm volatile("s_waitcnt vmcnt(4)" : "+v"(w2), "+v"(h2)::"memory");
      if (ready(w2, h2)) { wv = w2; head = h2; break; }
      poll_issue(w2, h2, wp, hp);
      if ((it & 63) == 63) {   // exit conditions every wave reaches
        if (ld_sys32(&ctl->stop) || __builtin_amdgcn_s_memrealtime() - last > idle_ticks) { quit = true; break; }
      }
    }
    // the polls still in flight must land before their registers are reused
    asm volatile("s_waitcnt vmcnt(0)" : "+v"(w0), "+v"(h0), "+v"(w1), "+v"(h1), "+v"(w2), "+v"(h2)::"memory");
    if (quit) break;
    const bool ok = lane >= D || (uint32_t)(wv >> 32) == want;
    if (__ballot(ok) == ~0ull && head <= tail + 4) {
      // latency path: the row arrived with the poll, x_i in lane i.  Lane u computes
      // output unit u of every layer from its register-resident weight column, taking
      // the previous layer's activations straight from their lanes (v_readlane into an
      // SGPR operand): no LDS round trip, no barrier, no second pass.
      const uint64_t t_seen = __builtin_amdgcn_s_memrealtime();
      const int li = lane < MAXD ? lane : MAXD - 1;
      const float xv = lane < D ? fmaf(__uint_as_float((uint32_t)wv), lsc[li], lsh[li]) : 0.f;
      auto layer = [&](float in, const float* w_col, float bias, int in_n, int out_n, int act, auto INC) {
        constexpr int IN_MAX = decltype(INC)::value;
        float acc0 = bias, acc1 = 0.f;
#pragma unroll
        for (int i = 0; i < IN_MAX; i += 2) {
          if (i < in_n) acc0 = fmaf(__int_as_float(__builtin_amdgcn_readlane(__float_as_int(in), i)), w_col[i], acc0);
          if (i + 1 < in_n)
            acc1 = fmaf(__int_as_float(__builtin_amdgcn_readlane(__float_as_int(in), i + 1)), w_col[i + 1], acc1);
        }
        return lane < out_n ? act_fwd(act, acc0 + acc1) : 0.f;
      };
      const float v1 = layer(xv, rw1, rb[0], D, n1, a1, std::integral_constant<int, XD>{});
      const float v2 = layer(v1, rw2, rb[1], n1, n2, a2, std::integral_constant<int, X1>{});
      const float v3 = layer(v2, rw3, rb[2], n2, n2, a3, std::integral_constant<int, X2>{});
      const float yv = layer(v3, rw4, rb[3], n2, D, a4, std::integral_constant<int, X2>{});
      const uint64_t t_comp = __builtin_amdgcn_s_memrealtime();
      const float d = lane < D ? yv - xv : 0.f;
      const float se = wave_sum(d * d);
      ServeResult* r = res + slot0;
      if (lane < D) st_sys(&r->w[lane], tagged(want, yv));
      if (lane == 0) {
        const float score = se / (float)D;
        st_sys(&r->w[kServeScore], tagged(want, score));
        st_sys(&r->w[kServeFlag], tagged_u(want, score > threshold ? 1u : 0u));
        st_sys(&r->w[kServeTLoad], tagged_u(want, 0u));
        st_sys(&r->w[kServeTComp], tagged_u(want, (uint32_t)(t_comp - t_seen)));
        st_sys(&r->w[kServeTDone], tagged_u(want, (uint32_t)(__builtin_amdgcn_s_memrealtime() - t_seen)));
      }
      tail += 1;
      if (lane == 0) st_sys(&ctl->done, tail);   // back-pressure hint only: results carry their own tags
      last = __builtin_amdgcn_s_memrealtime();
    } else if (head > tail + 4) {
      // backlog: one event per lane, up to 64 per pass (rows were published before head)
      const uint64_t t_seen = __builtin_amdgcn_s_memrealtime();
      const uint64_t k = head - tail < 64 ? head - tail : 64;
      if ((uint64_t)lane < k) {
        const uint64_t ev = tail + lane;
        const uint32_t tag = (uint32_t)(ev + 1);
        const int slot = (int)(ev % (uint64_t)nslots);
        SML_DCHECK(slot >= 0 && slot < nslots);
        float x[MAXD], h1[MAXH], h2[MAXH], h3[MAXH], y[XD];
        u32x4 q[MAXD / 2];
        static_assert(MAXD == 32, "ld_sys_row32 loads 32 words");
        ld_sys_row32(&req[slot].w[0], q);   // slot padding readable
#pragma unroll
        for (int i = 0; i < MAXD; ++i) {
          uint32_t bits = q[i / 2][2 * (i % 2)], t = q[i / 2][2 * (i % 2) + 1];
          if (i < D && t != tag) {
            // the host publishes head after the rows, so this normally never runs; bounded
            // so that a wave always reaches the exit conditions
            uint64_t v = ld_sys(&req[slot].w[i]);
            for (int spin = 0; (uint32_t)(v >> 32) != tag && spin < (1 << 20); ++spin) v = ld_sys(&req[slot].w[i]);
            bits = (uint32_t)v;
          }
          x[i] = i < D ? fmaf(__uint_as_float(bits), lsc[i], lsh[i]) : 0.f;
        }
        const uint64_t t_loaded = __builtin_amdgcn_s_memrealtime();
        dense_lane<XD, X1>(W1, b1, D, n1, x, h1, a1);
        dense_lane<X1, X2>(W2, b2, n1, n2, h1, h2, a2);
        dense_lane<X2, X2>(W3, b3, n2, n2, h2, h3, a3);
        dense_lane<X2, XD>(W4, b4, n2, D, h3, y, a4);
        const uint64_t t_comp = __builtin_amdgcn_s_memrealtime();
        float se = 0.f;
#pragma unroll
        for (int i = 0; i < MAXD; ++i) {
          if (i < D) {
            const float d = y[i] - x[i];
            se = fmaf(d, d, se);
          }
        }
        ServeResult* r = res + slot;
#pragma unroll
        for (int i = 0; i < XD; ++i)
          if (i < D) st_sys(&r->w[i], tagged(tag, y[i]));
        const float score = se / (float)D;
        st_sys(&r->w[kServeScore], tagged(tag, score));
        st_sys(&r->w[kServeFlag], tagged_u(tag, score > threshold ? 1u : 0u));
        st_sys(&r->w[kServeTLoad], tagged_u(tag, (uint32_t)(t_loaded - t_seen)));
        st_sys(&r->w[kServeTComp], tagged_u(tag, (uint32_t)(t_comp - t_seen)));
        st_sys(&r->w[kServeTDone], tagged_u(tag, (uint32_t)(__builtin_amdgcn_s_memrealtime() - t_seen)));
      }
      __syncthreads();
      tail += k;
      if (lane == 0) st_sys(&ctl->done, tail);
      last = __builtin_amdgcn_s_memrealtime();
    }
  }
  __syncthreads();
  wait_stores();
  if (lane == 0) st_sys32(&ctl->alive, 0u);
}

}  // namespace

hipError_t ae_serve_launch(ServeCtl* ctl, const ServeReq* req, ServeResult* res, int nslots, const float* wts,
                           const float* scale, const float* shift, const int* dims, const int* acts, float threshold,
                           double idle_seconds, hipStream_t stream) {
  if (dims[0] < 1 || dims[0] > MAXD || dims[1] < 1 || dims[1] > MAXH || dims[2] < 1 || dims[2] > MAXH)
    return hipErrorInvalidValue;
  if (nslots < 64) return hipErrorInvalidValue;
  const uint64_t ticks = (uint64_t)(idle_seconds * 100e6);   // s_memrealtime runs at 100 MHz
#define SML_SERVE(a, b, c)                                                                                    \
  hipLaunchKernelGGL((ae_serve_kernel<a, b, c>), dim3(1), dim3(64), 0, stream, ctl, req, res, nslots, wts, scale, \
                     shift, dims[0], dims[1], dims[2], acts[0], acts[1], acts[2], acts[3], threshold, ticks)
  if (dims[0] == 18 && dims[1] == 14 && dims[2] == 7) SML_SERVE(18, 14, 7);
  else if (dims[0] == 30 && dims[1] == 14 && dims[2] == 7) SML_SERVE(30, 14, 7);
  else SML_SERVE(0, 0, 0);
#undef SML_SERVE
  return hipGetLastError();
}

}  // namespace sml
