// Host-side launcher declarations for the streamml gfx950 kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace sml {

// ---- dense autoencoder (ae_fused.hip) ----
int ae_nslot();
int ae_train_blocks_per_cu();  // most resident 256-thread workgroups per CU of any train variant (4)
int ae_nparam();
int ae_waves_per_block();
int ae_train_grid(int64_t n, int max_blocks);
hipError_t ae_train_launch(const float* x, int64_t n, int64_t ld, const float* scale, const float* shift,
                           const float* params, float* partials, int64_t* iter, const int64_t* cursor,
                           const int* dims, const int* acts, float l1, int want_acc, int grid, const uint8_t* xpack,
                           hipStream_t stream, int* grid_used);  // grid_used <= grid: slabs written
// metrics (optional, 4 floats): += (sum sq err, sum |h1|, correct argmax, rows) -- evaluate()
hipError_t ae_forward_launch(const float* x, int64_t n, int64_t ld, const float* scale, const float* shift,
                             const float* params, float* recon, float* score, uint8_t* flag, float threshold,
                             const int* dims, const int* acts, int max_blocks, hipStream_t stream,
                             float* metrics = nullptr);
hipError_t reduce_adam_launch(const float* partials, int G, int S, int nparam, float* grad_out, float* params,
                              float* m, float* v, const int64_t* iter, float lr, float beta1, float beta2, float eps,
                              float gscale, float* metrics_acc, int flags, int64_t* cursor, int64_t cursor_step,
                              int64_t cursor_ring, hipStream_t stream);
// the slab level sum + reduce_adam in one launch (counters: slab_adam_columns(S) zeroed uint32,
// re-armed by the kernel; scratch: ceil(G / 32) * S floats); bit-identical to the two launches
int slab_adam_columns(int S);
hipError_t slab_adam_launch(const float* partials, int G, int S, int nparam, float* scratch, unsigned* counters,
                            float* grad_out, float* params, float* m, float* v, const int64_t* iter, float lr,
                            float beta1, float beta2, float eps, float gscale, float* metrics_acc, int flags,
                            int64_t* cursor, int64_t cursor_step, int64_t cursor_ring, hipStream_t stream);

// ---- persistent small-batch AE trainer (ae_minibatch.hip): nsteps Keras steps in one launch ----
int ae_minibatch_max_batch();
// streaming epoch counters (host-mapped device pointers, runtime/stream_ring.h)
struct MBStream {
  const int64_t* avail;      // rows in the ring so far (absolute)
  const int64_t* total;      // -1 until the stream ended, then the row count
  int64_t* consumed;         // rows the kernel no longer needs
  int* status;               // 1 = timed out waiting for rows
  long long timeout_ticks;   // s_memrealtime (100 MHz)
};
hipError_t ae_minibatch_launch(const float* x, int64_t ld, int64_t ring, int64_t* cursor, const float* scale,
                               const float* shift, float* params, float* m, float* v, int64_t* iter, float* metrics,
                               int B, int nsteps, const int* dims, const int* acts, float l1, float lr, float beta1,
                               float beta2, float eps, float gscale, int want_acc, unsigned long long* prof,
                               int nmodels, int64_t xmodel, const float* lrs, const int64_t* ragged,
                               uint64_t* const* dp_peers, int dp_ranks, int dp_rank0, int* dp_status,
                               long long dp_timeout, hipStream_t stream, const MBStream* sr = nullptr,
                               int precision = -1);   // 1 bf16 contractions, 0 fp32, -1 SML_MB_BF16

// ---- LSTM recurrence (lstm.hip) ----
hipError_t lstm_fwd_launch(const float* zx, const float* Uw, const float* h0, const float* c0, float* hseq,
                           float* cseq, float* gates, int64_t B, int T, int U, int act, hipStream_t stream);
hipError_t lstm_bwd_launch(const float* dh, const float* gates, const float* cseq, const float* c0, const float* Uw,
                           float* dz, float* dh0, float* dc0, int64_t B, int T, int U, int act, hipStream_t stream);

// ---- softmax + sparse categorical cross-entropy (softmax_xent.hip) ----
hipError_t softmax_xent_launch(const float* logits, const int64_t* labels, int64_t B, int C, float gscale,
                               float* dlogits, float* probs, float* acc, hipStream_t stream);

// ---- tall-skinny dense layers (dense.hip) ----
int dense_tiles(int d);
bool dense_supported(int K, int N);
int dense_wgrad_slab(int K, int N);
int dense_wgrad_grid(int64_t M, int max_blocks);
int slab_sum_scratch(int G, int S);
int slab_sum_level_launch(const float* in, int G, int S, float* out, hipStream_t stream);
// map (optional, S ints): the final level writes element s to out[map[s]] (< 0: dropped)
// two mapped slab sets reduced into one flat output in ONE launch (one-pass reduction, G <= 4096 each)
// Adam fused into slab_sum2 (the last reduction of a train step): every mapped slot is updated where its
// gradient becomes final, the `nrest` slots listed in `rest` (no slab covers them) from out[] as it
// stands.  Bit-identical to slab_sum2 + reduce_adam (sml_adam.h).
struct SlabAdam {
  float* params = nullptr;
  float* m = nullptr;
  float* v = nullptr;
  const int64_t* iter = nullptr;   // already advanced for this step
  float lr = 0.f, b1 = 0.f, b2 = 0.f, eps = 0.f, gscale = 1.f;
  const int* rest = nullptr;
  int nrest = 0;
};
hipError_t slab_sum2_launch(const float* p0, int G0, int S0, const int* map0, const float* p1, int G1, int S1,
                            const int* map1, float* out, hipStream_t stream, const SlabAdam* adam = nullptr);
hipError_t slab_sum_launch(const float* partials, int G, int S, float* scratch, float* out, hipStream_t stream,
                           const int* map = nullptr);
// w_t: W is the row-major [N, K] weight used transposed (Y = X . W^T)
hipError_t rowgemm_launch(const void* X, int x_bf16, int64_t M, int K, int64_t ldx, const float* W, const float* bias,
                          int N, int act, void* Y, int y_bf16, int64_t ldy, int max_blocks, hipStream_t stream,
                          int w_t = 0);
hipError_t wgrad_launch(const void* X, int x_bf16, int64_t M, int K, int64_t ldx, int shift_T, const void* DY,
                        int dy_bf16, int N, int64_t ldy, int want_db, float* partials, int grid, hipStream_t stream);

// ---- general LDS-tiled MFMA GEMM (gemm.hip) ----
// C[M, N] = act(op(A)[M, K] . op(B)[K, N] + bias), operands fp32 or bf16:
//   a_kc: A element (m, k) at A[m * lda + k] (else A[k * lda + m]);
//   b_kc: B element (k, n) at B[n * ldb + k] (else B[k * ldb + n]).
// splits > 1: split-K into `partials` ([splits, M, round4(N)] fp32; bias / act / C unused),
// reduced by slab_sum_launch.
hipError_t gemm_launch(const void* A, int a_bf16, int64_t lda, int a_kc, const void* B, int b_bf16, int64_t ldb,
                       int b_kc, int64_t M, int64_t N, int64_t K, const float* bias, int act, void* C, int c_bf16,
                       int64_t ldc, float* partials, int splits, hipStream_t stream);
int gemm_auto_splits(int64_t M, int64_t N, int64_t K, int cus);


// ---- fully fused LSTM layer (lstm_fused.hip) ----
bool lstm_fused_supported(int U, int IN);
int lstm_fused_slab(int U, int IN);
int lstm_fused_dx_ld(int IN);     // row stride of the padded dx buffer the backward kernel writes
int lstm_fused_waves(int64_t B);
int64_t lstm_fused_dz_bytes(int64_t B, int T, int U);   // dz scratch of the backward (U >= 64 layers), else 0
int lstm_fused_slabs(int64_t B, int U, bool dx);  // backward workgroups = weight-gradient slabs (persistent grid)
// x: fp32 or bf16 (x_bf16); h and dh are bf16 (lstm_fused.hip header), dx has x's dtype
hipError_t lstm_fused_fwd_launch(const void* x, bool x_bf16, const float* W, const float* Uw, const float* b,
                                 const float* h0, const float* c0, void* hseq_bf16, void* cseq_bf16, int64_t B, int T,
                                 int IN, int U, int act, int64_t x_seq, hipStream_t stream);
// two stacked layers in one forward (lstm_fused_fwd.hip): x fp32 [B, T, IN1] -> layer 1 (U1 32) ->
// layer 2 (U2 16); saves both layers' h / c exactly as two lstm_fused_fwd_launch calls do
bool lstm_fused_fwd2_supported(int IN1, int U1, int U2, int act1, int act2);
int lstm_fused_fwd2_rows(int64_t B);   // sequences the h / c buffers of lstm_fused_fwd2_launch must hold
// hlast2 non-null: h1 / h2 stored fragment-native (the backward's fragment mode) and layer 2's h_T
// as [B16, U2] bf16 rows into hlast2
hipError_t lstm_fused_fwd2_launch(const float* x, const float* W1, const float* U1, const float* b1, const float* W2,
                                  const float* U2, const float* b2, void* hseq1, void* cseq1, void* hseq2, void* cseq2,
                                  void* hlast2, int64_t B, int T, int IN1, int act1, int act2, int64_t x_seq,
                                  hipStream_t stream);
// two stacked layers' backward in one launch (lstm_fused_stack.hip): layer 2's dX feeds layer 1's
// dh in registers; one slab per workgroup per layer (partials1 [grid, S1], partials2 [grid, S2])
bool lstm_fused_bwd2_supported(int IN1, int U1, int U2, int act1, int act2);
int lstm_fused_bwd2_grid(int64_t B);
hipError_t lstm_fused_bwd2_launch(const float* x, int64_t x_seq, int IN1, const void* h1, const void* c1, const void* h2,
                                  const void* c2, const void* dh2, int dh2_last_only, const float* W1, const float* U1,
                                  const float* b1, const float* W2, const float* U2, const float* b2, float* partials1,
                                  float* partials2, int64_t B, int T, int act, hipStream_t stream);
hipError_t lstm_fused_bwd_launch(const void* dh_bf16, const void* cseq_bf16, const void* hseq_bf16, const void* x,
                                 bool x_bf16, const float* h0, const float* c0, const float* W, const float* Uw,
                                 const float* b, void* dx, float* dh0, float* dc0, float* partials, int64_t B, int T,
                                 int IN, int U, int act, int dh_last_only, int64_t x_seq, void* dz_scratch,
                                 int frag, hipStream_t stream);
// unit-block split backward (lstm_fused_split.hip): U = 32 layers without dX (fp32 x, dh every step) in the
// BX / DB bias modes run
// with two waves per 16-sequence tile; lstm_fused_bwd_launch routes them there, and the caller sizes
// the partials by lstm_fused_bwd_slabs (the split kernel's grid differs from lstm_fused_slabs)
bool lstm_split_applies(int U, int IN, bool dx, bool x_bf16, bool dh_last_only);
int lstm_split_grid(int64_t B);
hipError_t lstm_split_bwd_launch(const void* dh, const void* cseq, const void* hseq, const void* x, bool x_bf16,
                                 const float* h0, const float* c0, const float* W, const float* Uw, const float* b,
                                 float* dh0, float* dc0, float* partials, int64_t B, int T, int IN, int act,
                                 int dh_last_only, int64_t x_seq, int frag, hipStream_t st);
inline int lstm_fused_bwd_slabs(int64_t B, int U, int IN, bool dx, bool x_bf16, bool dh_last_only) {
  return lstm_split_applies(U, IN, dx, x_bf16, dh_last_only) ? lstm_split_grid(B) : lstm_fused_slabs(B, U, dx);
}
// fused Dense head of the LSTM predictor (lstm_head.hip): forward, MSE + accuracy, dW / db (scattered
// into grad through the dense slab map) and dh = dy . W^T (bf16 [n, 16]) in one pass + one fold launch;
// h [n, 16] bf16 rows (stride ldh), W [16, N], N <= 32; part holds lstm_head_partials(n, N) floats
int lstm_head_partials(int64_t n, int N);
hipError_t lstm_head_launch(const void* h, int64_t ldh, const float* W, const float* b, const float* y, int64_t ldy,
                            void* dh, int64_t n, int N, float gscale, float* part, float* grad, const int* map,
                            float* acc, float* out, float div0, float div1, int64_t* counter, hipStream_t st);
// fragment mode (frag = 1): h, a bf16 x and dh (unless dh_last_only) read fragment-native, dx written so;
// instances for the stacked model's two layers (U 32 without dX from fp32 x, U 16 with dX from bf16 x)
bool lstm_fused_frag_supported(int U, int IN, bool x_bf16, bool want_dx);

// tile-packed training ring: per 16-row tile the normalised rows (x * scale + shift, 64*D
// bytes) then their 16 argmax bytes; out holds n/16 * (64*D + 16) bytes (n % 16 == 0).
// index (optional, n int64): packed row r is x[index[r]]; perm_n > 0: packed row r is
// x[perm_row(r, perm_n, perm_key)], a keyed bijection of [0, perm_n) (an epoch's shuffle
// fused into the pack with no permutation array)
hipError_t pack_tiles_argmax_launch(const float* x, int64_t n, int64_t ld, int D, const float* scale,
                                    const float* shift, uint8_t* out, hipStream_t stream,
                                    const int64_t* index = nullptr, uint64_t perm_key = 0, int64_t perm_n = 0);
// out[i] = perm_row(start + i, n, key): the same bijection, materialised (short batches, tests)
hipError_t perm_indices_launch(int64_t* out, int64_t start, int64_t count, int64_t n, uint64_t key,
                               hipStream_t stream);
// argmax (lowest index on ties) of each normalised row x * scale + shift over D features
hipError_t row_argmax_launch(const float* x, int64_t n, int64_t ld, int D, const float* scale, const float* shift,
                             uint8_t* out, hipStream_t stream);

// ---- MNIST MLP GEMMs (mlp.hip): fp32 MFMA, LDS-tiled K loop, fused epilogues ----
hipError_t mlp_fwd_launch(const void* x, int x_u8, int64_t ldx, const float* W, const float* b, float* y, int M,
                          int K, int N, int relu, float keep, uint32_t seed, uint32_t step, hipStream_t st);
hipError_t mlp_bwd_data_launch(const float* dz, const float* W, const float* h, float* dh, int M, int N1, int N2,
                               float inv_keep, hipStream_t st);
hipError_t mlp_wgrad_launch(const void* x, int x_u8, int64_t ldx, const float* dy, float* out, int B, int K, int N,
                            hipStream_t st);
hipError_t mlp_dropout_mask_launch(float* out, int M, int N, float keep, uint32_t seed, uint32_t step,
                                   hipStream_t st);

// ---- persistent Keras-step trainer for the reference LSTM stack (lstm_ref_train.hip) ----
int lstm_ref_train_params();
hipError_t lstm_ref_train_launch(float* flat, float* m, float* v, int64_t* iter, const float* x, int64_t ldx,
                                 const float* y, int64_t ldy, const int32_t* order, int64_t nrows, int64_t row0, int B,
                                 int nsteps, int act, float lr, float beta1, float beta2, float eps, float* out,
                                 hipStream_t stream);

// ---- persistent per-event scorer (ae_serve.hip); structures live in host-mapped memory ----
struct alignas(128) ServeCtl {
  uint64_t head;            // host: events published (monotonic)
  uint64_t pad0[15];
  uint64_t done;            // device: events completed (monotonic)
  uint64_t pad1[15];
  uint32_t stop;            // host: ask the kernel to exit
  uint32_t alive;           // device: 1 while the kernel runs
  uint32_t pad2[30];
};
// Request and result slots use low-latency ("LL") framing: every 8-byte word carries
// 4 bytes of payload and a 4-byte tag = (uint32)(event + 1).  One 8-byte-atomic PCIe
// read then tells whether the word already belongs to the event being waited for, so
// neither side needs a separate ready flag, fence or acknowledgement round trip: the
// GPU polls the request words themselves and has the row in registers the moment the
// tags match; the host polls the result words in its own memory.
struct ServeReq {
  uint64_t w[32];           // w[i] = tag << 32 | float bits of x[i]  (i < D)
};
enum : int {                // ServeResult word indices
  kServeScore = 32,         // mean squared reconstruction error
  kServeFlag = 33,          // score > threshold
  kServeTLoad = 34,         // device ticks (100 MHz) from pick-up to row in registers
  kServeTComp = 35,         // ... to forward pass done
  kServeTDone = 36,         // ... to result stores issued
  kServeWords = 37
};
struct ServeResult {
  uint64_t w[40];           // [0, D): reconstruction, then the fields above; all tagged
};
hipError_t ae_serve_launch(ServeCtl* ctl, const ServeReq* req, ServeResult* res, int nslots, const float* wts,
                           const float* scale, const float* shift, const int* dims, const int* acts, float threshold,
                           double idle_seconds, hipStream_t stream);

// ---- persistent per-event LSTM scorer (lstm_serve.hip): same rings as ae_serve ----
// request word 31 carries the car key (uint32 payload); result words [0, D) the forecast of
// the key's next event, kServeScore the MSE of this event against the key's previous
// forecast, kServeFlag 0 normal / 1 anomaly / 2 no forecast yet (fewer than T + 1 events)
enum : int { LS_LSTM = 0, LS_REPEAT = 1, LS_DENSE = 2, LS_MAXLAYERS = 8 };
struct LstmServeLayer {
  int kind;            // LS_*
  int in, u;           // input width, units (Dense: output width)
  int act, ret, n;     // LSTM activation code, return_sequences; RepeatVector n
  int woff, uoff, boff;   // float offsets of kernel / recurrent kernel / bias in the weights
};
struct LstmServeArgs {
  ServeCtl* ctl;
  const ServeReq* req;
  ServeResult* res;
  int nslots;
  const float* wts;
  int nw;
  int nl;
  LstmServeLayer L[LS_MAXLAYERS];
  const float* scale;
  const float* shift;
  int D, T;
  float* hist;         // [nkeys][T][D] per-key window ring (device)
  int* hcount;         // [nkeys] events seen per key
  float* lastpred;     // [nkeys][D] the key's latest forecast
  int nkeys;
  float threshold;
  uint64_t idle_ticks;
};
size_t lstm_serve_lds_bytes(int nw);
hipError_t lstm_serve_launch(const LstmServeArgs& args, hipStream_t stream);

// ---- fused MSE + categorical accuracy (loss.hip) ----
bool mse_acc_supported(int F);
// acc != null needs part: 2 * mse_acc_blocks(rows, F) floats of scratch (the block partials,
// folded into acc by a one-block kernel: acc = partials (reset) or acc += partials); out
// (optional, needs acc): out[k] = acc[k] / div_k after the fold; counter (optional, needs acc):
// an int64 step count advanced by one in the same launch
int mse_acc_blocks(int64_t rows, int F);
hipError_t mse_acc_launch(const float* yp, const float* y, int64_t rows, int F, int bcast, float gscale, float* grad,
                          float* acc, float* part, int reset, hipStream_t stream, float* out = nullptr,
                          float div0 = 1.f, float div1 = 1.f, int64_t* counter = nullptr);

// ---- utilities (util.hip) ----
hipError_t lane_xor_probe_launch(float* out, hipStream_t stream);

// K8 normalize + label filter + order-preserving compaction (preprocess.hip)
int filter_blocks(int64_t n);
hipError_t normalize_filter_launch(const float* x, int64_t n, int64_t ld, int D, const uint8_t* labels, int keep,
                                   const float* scale, const float* shift, int* counts, float* out,
                                   int64_t* out_index, int64_t* total, hipStream_t stream);

}  // namespace sml
