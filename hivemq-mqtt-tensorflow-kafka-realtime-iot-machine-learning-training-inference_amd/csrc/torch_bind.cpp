// PyTorch binding for the gfx950 kernels (module streamml._C).
//
// Every op here requires ROCm device tensors; there is deliberately no CPU
// fallback inside the extension (the torch-CPU reference path lives in Python
// and is only used for the CPU plumbing configuration / numerics oracles).
#include <torch/extension.h>
#include <c10/hip/HIPStream.h>
#include <c10/hip/HIPGuard.h>
#include <hip/hip_runtime.h>

#include "sml_ops.h"
#include "../runtime/p2p.h"
#include "sml_p2p.h"
#include "sml_scorer_api.h"
#include "../runtime/ring.h"
#include "../runtime/serve.h"
#include "../runtime/stream_ring.h"
#include "../runtime/queues.h"

#include <pybind11/numpy.h>
#include <cstdlib>
#include <cstring>

namespace {

// SML_SYNC_CHECK=1: launch-blocking debug mode -- every launch is
// followed by a device synchronize, so an asynchronous kernel fault is reported
// against the op that caused it instead of a later, unrelated call.
static bool sync_check() {
  const char* v = std::getenv("SML_SYNC_CHECK");
  return v && *v && *v != '0';
}

#define SML_CHECK_HIP(expr)                                                                           \
  do {                                                                                                \
    hipError_t _e = (expr);                                                                           \
    TORCH_CHECK(_e == hipSuccess, "HIP error: ", hipGetErrorString(_e), " @ ", #expr);                \
    if (sync_check()) {                                                                               \
      _e = hipDeviceSynchronize();                                                                    \
      if (_e == hipSuccess) _e = hipGetLastError();                                                   \
      TORCH_CHECK(_e == hipSuccess, "HIP error (SML_SYNC_CHECK): ", hipGetErrorString(_e), " after ", \
                  #expr);                                                                             \
    }                                                                                                 \
  } while (0)

void check_dev(const at::Tensor& t, const char* name, at::ScalarType st) {
  TORCH_CHECK(t.is_cuda(), name, " must be a ROCm device tensor");
  TORCH_CHECK(t.scalar_type() == st, name, " has wrong dtype ", t.scalar_type());
  TORCH_CHECK(t.is_contiguous() || t.dim() == 2, name, " must be contiguous");
}

const float* opt_ptr(const c10::optional<at::Tensor>& t) {
  return t.has_value() && t->defined() ? t->data_ptr<float>() : nullptr;
}
float* opt_mut(const c10::optional<at::Tensor>& t) {
  return t.has_value() && t->defined() ? t->data_ptr<float>() : nullptr;
}

hipStream_t cur_stream(const at::Tensor& t) {
  return c10::hip::getCurrentHIPStream(t.device().index()).stream();
}

void check_ae_dims(const std::vector<int64_t>& dims, const std::vector<int64_t>& acts) {
  TORCH_CHECK(dims.size() == 4 && acts.size() == 4, "dims/acts must have 4 entries");
  TORCH_CHECK(dims[0] >= 1 && dims[0] <= 31, "AE input dim must be in [1,31]");
  for (int i = 1; i < 4; ++i) TORCH_CHECK(dims[i] >= 1 && dims[i] <= 15, "AE hidden dims must be in [1,15]");
  for (auto a : acts) TORCH_CHECK(a >= 0 && a <= 3, "activation code must be 0..3");
}

int64_t ae_train_partials(const at::Tensor& x, const c10::optional<at::Tensor>& scale,
                          const c10::optional<at::Tensor>& shift, const at::Tensor& params, at::Tensor& partials,
                          const c10::optional<at::Tensor>& iter, std::vector<int64_t> dims, std::vector<int64_t> acts,
                          double l1, bool want_acc, int64_t max_blocks, int64_t n_rows,
                          const c10::optional<at::Tensor>& cursor, const c10::optional<at::Tensor>& xpack) {
  check_ae_dims(dims, acts);
  check_dev(x, "x", at::kFloat);
  TORCH_CHECK(x.dim() == 2 && x.stride(1) == 1, "x must be [n, ld] with unit column stride");
  TORCH_CHECK(x.size(1) >= dims[0], "x has fewer columns than the model input dim");
  check_dev(params, "params", at::kFloat);
  TORCH_CHECK(params.numel() == sml::ae_nparam(), "params must be the padded 1536-float image");
  check_dev(partials, "partials", at::kFloat);
  if (scale.has_value()) {
    TORCH_CHECK(shift.has_value(), "scale requires shift");
    check_dev(*scale, "scale", at::kFloat);
    check_dev(*shift, "shift", at::kFloat);
    TORCH_CHECK(scale->numel() >= dims[0] && shift->numel() >= dims[0], "scale/shift too short");
  }
  int64_t* iter_ptr = nullptr;
  if (iter.has_value() && iter->defined()) {
    check_dev(*iter, "iter", at::kLong);
    iter_ptr = iter->data_ptr<int64_t>();
  }
  const int64_t n = n_rows >= 0 ? n_rows : x.size(0);
  const int64_t* cur_ptr = nullptr;
  if (cursor.has_value() && cursor->defined()) {
    check_dev(*cursor, "cursor", at::kLong);
    // the ring contract (checked by the caller): cursor + n <= rows, cursor a multiple of n
    TORCH_CHECK(n > 0 && x.size(0) % n == 0, "ring rows must be a multiple of the batch");
    cur_ptr = cursor->data_ptr<int64_t>();
  } else {
    TORCH_CHECK(n <= x.size(0), "n_rows larger than x");
  }
  const uint8_t* xpack_ptr = nullptr;
  if (xpack.has_value() && xpack->defined()) {
    TORCH_CHECK(xpack->is_cuda() && xpack->scalar_type() == at::kByte && xpack->is_contiguous() &&
                    x.size(0) % 16 == 0 && xpack->numel() == x.size(0) / 16 * (64 * dims[0] + 16),
                "xpack must be the tile-packed ring of x (pack_tiles_argmax)");
    xpack_ptr = xpack->data_ptr<uint8_t>();
  }
  const int grid = sml::ae_train_grid(n, (int)max_blocks);
  TORCH_CHECK(partials.numel() >= (int64_t)grid * sml::ae_nslot(), "partials buffer too small for grid ", grid);
  int used = grid;   // the launcher may trim it (pair variants: 3 resident workgroups per CU)
  c10::hip::HIPGuard guard(x.device().index());
  int d[4] = {(int)dims[0], (int)dims[1], (int)dims[2], (int)dims[3]};
  int a[4] = {(int)acts[0], (int)acts[1], (int)acts[2], (int)acts[3]};
  SML_CHECK_HIP(sml::ae_train_launch(x.data_ptr<float>(), n, x.stride(0), opt_ptr(scale), opt_ptr(shift),
                                     params.data_ptr<float>(), partials.data_ptr<float>(), iter_ptr, cur_ptr, d, a,
                                     (float)l1,
                                     want_acc ? 1 : 0, grid, xpack_ptr, cur_stream(x), &used));
  return used;
}

// ingest-time tile-packed ring: per 16-row tile the rows then the 16 argmax bytes
// index (optional int64 [m]): pack rows x[index[0..m)] instead of x[0..n); out (optional): an
// existing byte buffer of at least the packed size (e.g. a slice of a ring being refilled)
// perm_n > 0: pack rows x[perm_row(r, perm_n, perm_key)] for r < n_rows (default perm_n): an
// epoch's shuffle as a keyed bijection evaluated in the kernel
at::Tensor pack_tiles_argmax(const at::Tensor& x, int64_t D, const c10::optional<at::Tensor>& scale,
                             const c10::optional<at::Tensor>& shift, const c10::optional<at::Tensor>& index,
                             const c10::optional<at::Tensor>& out_opt, uint64_t perm_key, int64_t perm_n,
                             int64_t n_rows) {
  check_dev(x, "x", at::kFloat);
  TORCH_CHECK(x.dim() == 2 && x.stride(1) == 1 && x.size(1) >= D && D >= 1 && D <= 64,
              "x must be [n, >=D] with D <= 64");
  TORCH_CHECK(scale.has_value() == shift.has_value(), "scale and shift go together");
  if (scale.has_value()) TORCH_CHECK(scale->numel() >= D && shift->numel() >= D, "scale/shift too short");
  int64_t n = x.size(0);
  const int64_t* idx = nullptr;
  if (index.has_value() && index->defined()) {
    TORCH_CHECK(index->is_cuda() && index->device() == x.device() && index->scalar_type() == at::kLong &&
                    index->dim() == 1 && index->is_contiguous(), "index must be a contiguous int64 device vector");
    n = index->numel();
    // the kernel trusts the indices: bounds-check on the device before launching it
    if (n > 0) {
      const auto mm = at::aminmax(*index);
      TORCH_CHECK(std::get<0>(mm).item<int64_t>() >= 0 && std::get<1>(mm).item<int64_t>() < x.size(0),
                  "index out of range for x");
    }
    idx = index->data_ptr<int64_t>();
  }
  if (perm_n > 0) {
    TORCH_CHECK(idx == nullptr, "index and perm are exclusive");
    TORCH_CHECK(perm_n <= x.size(0), "perm_n larger than x");
    n = n_rows >= 0 ? n_rows : perm_n;
    TORCH_CHECK(n <= perm_n, "more packed rows than the permuted domain");
  } else if (n_rows >= 0) {
    TORCH_CHECK(n_rows <= n, "n_rows larger than the source");
    n = n_rows;
  }
  TORCH_CHECK(n % 16 == 0, "packed rows must be a multiple of 16");
  const int64_t bytes = n / 16 * (64 * D + 16);
  c10::hip::HIPGuard guard(x.device().index());
  at::Tensor out;
  if (out_opt.has_value() && out_opt->defined()) {
    out = *out_opt;
    TORCH_CHECK(out.is_cuda() && out.device() == x.device() && out.scalar_type() == at::kByte && out.is_contiguous() &&
                    out.numel() >= bytes && (reinterpret_cast<uintptr_t>(out.data_ptr()) & 15) == 0,
                "out must be a contiguous, 16-byte aligned uint8 device buffer of >= the packed size");
  } else {
    out = at::empty({bytes}, x.options().dtype(at::kByte));
  }
  SML_CHECK_HIP(sml::pack_tiles_argmax_launch(x.data_ptr<float>(), n, x.stride(0), (int)D, opt_ptr(scale),
                                              opt_ptr(shift), out.data_ptr<uint8_t>(), cur_stream(x), idx, perm_key,
                                              perm_n));
  return out;
}

// the pack's keyed bijection, materialised: int64 [count] = perm_row(start + i, n, key)
at::Tensor perm_indices(const at::Tensor& like, int64_t n, uint64_t key, int64_t start, int64_t count) {
  TORCH_CHECK(like.is_cuda(), "like must be a device tensor");
  if (count < 0) count = n - start;
  TORCH_CHECK(n > 0 && start >= 0 && count >= 0 && start + count <= n, "need 0 <= start, start + count <= n");
  c10::hip::HIPGuard guard(like.device().index());
  auto out = at::empty({count}, like.options().dtype(at::kLong));
  SML_CHECK_HIP(sml::perm_indices_launch(out.data_ptr<int64_t>(), start, count, n, key, cur_stream(like)));
  return out;
}

// ingest-time argmax of every normalised row -> uint8 [n]
at::Tensor row_argmax_u8(const at::Tensor& x, int64_t D, const c10::optional<at::Tensor>& scale,
                         const c10::optional<at::Tensor>& shift) {
  check_dev(x, "x", at::kFloat);
  TORCH_CHECK(x.dim() == 2 && x.stride(1) == 1 && x.size(1) >= D && D >= 1 && D <= 255, "x must be [n, >=D]");
  TORCH_CHECK(scale.has_value() == shift.has_value(), "scale and shift go together");
  if (scale.has_value()) TORCH_CHECK(scale->numel() >= D && shift->numel() >= D, "scale/shift too short");
  c10::hip::HIPGuard guard(x.device().index());
  auto out = at::empty({x.size(0)}, x.options().dtype(at::kByte));
  SML_CHECK_HIP(sml::row_argmax_launch(x.data_ptr<float>(), x.size(0), x.stride(0), (int)D, opt_ptr(scale),
                                       opt_ptr(shift), out.data_ptr<uint8_t>(), cur_stream(x)));
  return out;
}

// K8: returns (out [n, D] with the kept rows first, source index [n] (or empty), total [1] int64)
std::vector<at::Tensor> normalize_filter(const at::Tensor& x, int64_t D, const c10::optional<at::Tensor>& labels,
                                         int64_t keep, const c10::optional<at::Tensor>& scale,
                                         const c10::optional<at::Tensor>& shift, bool want_index) {
  check_dev(x, "x", at::kFloat);
  TORCH_CHECK(x.dim() == 2 && x.stride(1) == 1 && x.size(1) >= D && D >= 1 && D <= 64, "x must be [n, >=D], D<=64");
  const int64_t n = x.size(0);
  const uint8_t* lab = nullptr;
  if (labels.has_value() && labels->defined()) {
    TORCH_CHECK(labels->is_cuda() && labels->scalar_type() == at::kByte && labels->numel() == n &&
                    labels->is_contiguous(), "labels must be a uint8 device tensor with one code per row");
    lab = labels->data_ptr<uint8_t>();
  }
  TORCH_CHECK(lab != nullptr || keep < 0, "filtering needs labels");
  if (scale.has_value() && scale->defined()) {
    TORCH_CHECK(shift.has_value() && shift->defined() && scale->numel() >= D && shift->numel() >= D,
                "scale/shift need D entries");
    check_dev(*scale, "scale", at::kFloat);
    check_dev(*shift, "shift", at::kFloat);
  }
  c10::hip::HIPGuard guard(x.device().index());
  auto fo = x.options();
  auto out = at::empty({n, D}, fo);
  auto idx = want_index ? at::empty({n}, fo.dtype(at::kLong)) : at::empty({0}, fo.dtype(at::kLong));
  auto total = at::empty({1}, fo.dtype(at::kLong));
  auto counts = at::empty({std::max(1, sml::filter_blocks(n))}, fo.dtype(at::kInt));
  SML_CHECK_HIP(sml::normalize_filter_launch(x.data_ptr<float>(), n, x.stride(0), (int)D, lab, (int)keep,
                                             opt_ptr(scale), opt_ptr(shift), counts.data_ptr<int>(),
                                             out.data_ptr<float>(), want_index ? idx.data_ptr<int64_t>() : nullptr,
                                             total.data_ptr<int64_t>(), cur_stream(x)));
  return {out, idx, total};
}

// SML_AE_FUSED_REDUCE=1: the wide-grid reduction in one launch (slab_adam_kernel, bit-identical
// results) instead of two (level sum, then reduce_adam); read at every call.  Default off: the
// agent-scope release fence every workgroup needs before its count writes back its XCD's whole L2
// (buffer_wbl2), which the train kernel's ~19 MB of slabs have just filled -- the one launch took
// 80 us against 5.9 + 5.9 us, 0.70 vs 0.66 ms per headline step (profiles/r06/SUMMARY.md §10).
static bool fused_reduce_enabled() {
  const char* e = std::getenv("SML_AE_FUSED_REDUCE");
  return e && e[0] == '1';
}

void reduce_adam(const at::Tensor& partials, int64_t G, int64_t S, int64_t nparam,
                 const c10::optional<at::Tensor>& grad_out, const c10::optional<at::Tensor>& params,
                 const c10::optional<at::Tensor>& m, const c10::optional<at::Tensor>& v,
                 const c10::optional<at::Tensor>& iter, double lr, double beta1, double beta2, double eps,
                 double gscale, const c10::optional<at::Tensor>& metrics, int64_t flags,
                 const c10::optional<at::Tensor>& cursor, int64_t cursor_step, int64_t cursor_ring,
                 const c10::optional<at::Tensor>& scratch, const c10::optional<at::Tensor>& counters) {
  check_dev(partials, "partials", at::kFloat);
  TORCH_CHECK(partials.numel() >= G * S, "partials smaller than G*S");
  const float* src = partials.data_ptr<float>();
  const bool wide = scratch.has_value() && scratch->defined() && G > 64;
  if (wide && counters.has_value() && counters->defined() && fused_reduce_enabled()) {
    // wide grids, one launch: the level sum and the Adam pass joined by per-column counters
    check_dev(*scratch, "scratch", at::kFloat);
    check_dev(*counters, "counters", at::kInt);
    TORCH_CHECK(counters->numel() >= sml::slab_adam_columns((int)S) && counters->is_contiguous(),
                "reduce counters too small");
    TORCH_CHECK(scratch->numel() >= ((G + 31) / 32) * S, "reduce scratch too small");
    if (flags & 2) {
      TORCH_CHECK(params.has_value() && m.has_value() && v.has_value() && iter.has_value(), "adam needs params/m/v/iter");
      TORCH_CHECK(params->numel() >= nparam && m->numel() >= nparam && v->numel() >= nparam, "adam buffers too small");
      check_dev(*iter, "iter", at::kLong);
    }
    if (flags & 1) TORCH_CHECK(grad_out.has_value() && grad_out->numel() >= S, "grad_out too small");
    if (flags & 4) TORCH_CHECK(metrics.has_value() && metrics->numel() >= S - nparam, "metrics too small");
    c10::hip::HIPGuard guard(partials.device().index());
    const int64_t* iter_ptr = (iter.has_value() && iter->defined()) ? iter->data_ptr<int64_t>() : nullptr;
    SML_CHECK_HIP(sml::slab_adam_launch(src, (int)G, (int)S, (int)nparam, scratch->data_ptr<float>(),
                                        reinterpret_cast<unsigned*>(counters->data_ptr<int>()), opt_mut(grad_out),
                                        opt_mut(params), opt_mut(m), opt_mut(v), iter_ptr, (float)lr, (float)beta1,
                                        (float)beta2, (float)eps, (float)gscale, opt_mut(metrics), (int)flags,
                                        (cursor.has_value() && cursor->defined()) ? cursor->data_ptr<int64_t>() : nullptr,
                                        cursor_step, cursor_ring, cur_stream(partials)));
    return;
  }
  if (wide) {
    // wide grids: one parallel level of the deterministic slab sum first (G -> ceil(G/32)
    // slabs over G/32 x S/256 workgroups), so the Adam kernel reads 32x fewer bytes
    check_dev(*scratch, "scratch", at::kFloat);
    const int64_t gy = (G + 31) / 32;
    TORCH_CHECK(scratch->numel() >= gy * S, "reduce scratch too small");
    c10::hip::HIPGuard guard(partials.device().index());
    const int got = sml::slab_sum_level_launch(src, (int)G, (int)S, scratch->data_ptr<float>(), cur_stream(partials));
    TORCH_CHECK(got == gy, "slab_sum_level_launch failed");
    SML_CHECK_HIP(hipGetLastError());
    src = scratch->data_ptr<float>();
    G = gy;
  }
  if (flags & 2) {
    TORCH_CHECK(params.has_value() && m.has_value() && v.has_value() && iter.has_value(), "adam needs params/m/v/iter");
    TORCH_CHECK(params->numel() >= nparam && m->numel() >= nparam && v->numel() >= nparam, "adam buffers too small");
    check_dev(*iter, "iter", at::kLong);
  }
  if (flags & 1) TORCH_CHECK(grad_out.has_value() && grad_out->numel() >= S, "grad_out too small");
  if (flags & 4) TORCH_CHECK(metrics.has_value() && metrics->numel() >= S - nparam, "metrics too small");
  c10::hip::HIPGuard guard(partials.device().index());
  const int64_t* iter_ptr = (iter.has_value() && iter->defined()) ? iter->data_ptr<int64_t>() : nullptr;
  SML_CHECK_HIP(sml::reduce_adam_launch(src, (int)G, (int)S, (int)nparam, opt_mut(grad_out),
                                        opt_mut(params), opt_mut(m), opt_mut(v), iter_ptr, (float)lr, (float)beta1,
                                        (float)beta2, (float)eps, (float)gscale, opt_mut(metrics), (int)flags,
                                        (cursor.has_value() && cursor->defined()) ? cursor->data_ptr<int64_t>() : nullptr,
                                        cursor_step, cursor_ring, cur_stream(partials)));
}

void train_minibatches_impl(const at::Tensor& x, const at::Tensor& cursor, const c10::optional<at::Tensor>& scale,
                            const c10::optional<at::Tensor>& shift, const at::Tensor& params, const at::Tensor& m,
                            const at::Tensor& v, const at::Tensor& iter, const c10::optional<at::Tensor>& metrics,
                            int64_t batch, int64_t nsteps, std::vector<int64_t> dims, std::vector<int64_t> acts,
                            double l1, double lr, double beta1, double beta2, double eps, double gscale,
                            bool want_acc, const c10::optional<at::Tensor>& prof,
                            const c10::optional<at::Tensor>& lrs, uint64_t dp_peers, int64_t dp_ranks,
                            int64_t dp_rank0, uint64_t dp_status, int64_t dp_timeout_ticks,
                            const c10::optional<at::Tensor>& ragged, const sml::MBStream* sr, hipStream_t st,
                            int64_t precision = -1) {
  // One model: params/m/v [1536], cursor/iter [1], x [ring, ld].  Fleet of M models:
  // params/m/v [M, 1536], cursor/iter [M], metrics [M, 4], x [ring, ld] (shared) or [M, ring, ld].
  check_ae_dims(dims, acts);
  check_dev(x, "x", at::kFloat);
  TORCH_CHECK(x.dim() == 2 || x.dim() == 3, "x must be [ring, ld] or [M, ring, ld]");
  TORCH_CHECK(x.stride(-1) == 1, "x must have unit column stride");
  const int64_t np = sml::ae_nparam();
  TORCH_CHECK(params.numel() % np == 0 && params.numel() > 0, "params must be [M, padded image]");
  const int64_t M = params.numel() / np;
  const int64_t ring = x.size(-2), ld = x.stride(-2);
  TORCH_CHECK(x.dim() == 2 || (x.size(0) == M && x.stride(1) * x.size(1) <= x.stride(0)),
              "per-model rings must be [M, ring, ld] with non-overlapping models");
  TORCH_CHECK(x.size(-1) >= dims[0], "x has fewer columns than the model input dim");
  TORCH_CHECK(batch >= 1 && batch <= sml::ae_minibatch_max_batch(), "batch must be in [1, ",
              sml::ae_minibatch_max_batch(), "]");
  TORCH_CHECK(nsteps >= 1 && nsteps <= (1 << 30), "nsteps out of range");
  const int64_t* ragged_ptr = nullptr;
  if (ragged.has_value() && ragged->defined()) {
    // [M][3] {first row, ring rows, steps} on the device; validated here from a host copy
    check_dev(*ragged, "ragged", at::kLong);
    TORCH_CHECK(x.dim() == 2 && ragged->numel() == 3 * M && ragged->is_contiguous(),
                "ragged needs a flat [rows, ld] x and an int64 [M, 3] table");
    auto h = ragged->cpu();
    const int64_t* r = h.data_ptr<int64_t>();
    for (int64_t i = 0; i < M; ++i) {
      TORCH_CHECK(r[3 * i] >= 0 && r[3 * i + 1] >= batch && r[3 * i + 1] % batch == 0 &&
                      r[3 * i] + r[3 * i + 1] <= x.size(0) && r[3 * i + 2] >= 0 && r[3 * i + 2] <= (1 << 30),
                  "ragged row ", i, ": needs 0 <= first, ring a positive multiple of the batch inside x, steps >= 0");
    }
    ragged_ptr = ragged->data_ptr<int64_t>();
  } else {
    TORCH_CHECK(ring >= batch && ring % batch == 0, "ring rows must be a positive multiple of the batch");
  }
  check_dev(cursor, "cursor", at::kLong);
  check_dev(iter, "iter", at::kLong);
  TORCH_CHECK(cursor.numel() == M && iter.numel() == M && cursor.is_contiguous() && iter.is_contiguous(),
              "cursor / iter must be contiguous int64 [M]");
  for (const at::Tensor* t : {&params, &m, &v}) {
    check_dev(*t, "params/m/v", at::kFloat);
    TORCH_CHECK(t->numel() == M * np && t->is_contiguous(), "params/m/v must be the padded image [M, 1536]");
  }
  if (metrics.has_value()) {
    check_dev(*metrics, "metrics", at::kFloat);
    TORCH_CHECK(metrics->is_contiguous() && metrics->numel() >= 4 * M, "metrics needs 4 slots per model");
  }
  if (scale.has_value()) TORCH_CHECK(shift.has_value() && scale->numel() >= dims[0] && shift->numel() >= dims[0],
                                     "scale requires shift, both [D]");
  const float* lrs_ptr = nullptr;
  if (lrs.has_value() && lrs->defined()) {
    check_dev(*lrs, "lrs", at::kFloat);
    TORCH_CHECK(lrs->numel() == M && lrs->is_contiguous(), "lrs must be float32 [M]");
    lrs_ptr = lrs->data_ptr<float>();
  }
  unsigned long long* prof_ptr = nullptr;
  if (prof.has_value() && prof->defined()) {
    check_dev(*prof, "prof", at::kLong);
    TORCH_CHECK(prof->numel() >= 11, "prof needs 11 int64 slots");
    prof_ptr = reinterpret_cast<unsigned long long*>(prof->data_ptr<int64_t>());
  }
  // the cursors are read on the device; their host-side validity is the caller's contract
  // (FusedAE / AEFleet keep each one a multiple of the batch below the ring size)
  c10::hip::HIPGuard guard(x.device().index());
  int d[4] = {(int)dims[0], (int)dims[1], (int)dims[2], (int)dims[3]};
  int a[4] = {(int)acts[0], (int)acts[1], (int)acts[2], (int)acts[3]};
  SML_CHECK_HIP(sml::ae_minibatch_launch(x.data_ptr<float>(), ld, ring, cursor.data_ptr<int64_t>(),
                                         opt_ptr(scale), opt_ptr(shift), params.data_ptr<float>(),
                                         m.data_ptr<float>(), v.data_ptr<float>(), iter.data_ptr<int64_t>(),
                                         opt_mut(metrics), (int)batch, (int)nsteps, d, a, (float)l1, (float)lr,
                                         (float)beta1, (float)beta2, (float)eps, (float)gscale, (int)want_acc,
                                         prof_ptr, (int)M, x.dim() == 3 ? x.stride(0) : 0, lrs_ptr, ragged_ptr,
                                         reinterpret_cast<uint64_t* const*>(dp_peers), (int)dp_ranks, (int)dp_rank0,
                                         reinterpret_cast<int*>(dp_status), (long long)dp_timeout_ticks,
                                         st, sr, (int)precision));
}

void ae_train_minibatches(const at::Tensor& x, const at::Tensor& cursor, const c10::optional<at::Tensor>& scale,
                          const c10::optional<at::Tensor>& shift, const at::Tensor& params, const at::Tensor& m,
                          const at::Tensor& v, const at::Tensor& iter, const c10::optional<at::Tensor>& metrics,
                          int64_t batch, int64_t nsteps, std::vector<int64_t> dims, std::vector<int64_t> acts,
                          double l1, double lr, double beta1, double beta2, double eps, double gscale, bool want_acc,
                          const c10::optional<at::Tensor>& prof, const c10::optional<at::Tensor>& lrs,
                          uint64_t dp_peers, int64_t dp_ranks, int64_t dp_rank0, uint64_t dp_status,
                          int64_t dp_timeout_ticks, const c10::optional<at::Tensor>& ragged, int64_t precision) {
  train_minibatches_impl(x, cursor, scale, shift, params, m, v, iter, metrics, batch, nsteps, std::move(dims),
                         std::move(acts), l1, lr, beta1, beta2, eps, gscale, want_acc, prof, lrs, dp_peers, dp_ranks,
                         dp_rank0, dp_status, dp_timeout_ticks, ragged, nullptr, cur_stream(x), precision);
}

// A streaming epoch on ONE persistent ae_minibatch launch (runtime/stream_ring.h): the
// kernel runs on the ring's own train stream and takes its batches from the device ring
// as push() lands them (doorbell = host-mapped row count written by the copy stream).
// Deadlock rule: the producer of pushed rows must not be the train stream, so train()
// never makes the caller's stream wait for the kernel -- join() does, after finish().
class StreamRingPy {
 public:
  StreamRingPy(int64_t device, int64_t rows, int64_t features)
      : dev_(device), ring_((int)device, rows, (int)features) {
    c10::hip::HIPGuard guard((int)device);
    SML_CHECK_HIP(sml::create_persistent_stream(&train_));
    SML_CHECK_HIP(hipEventCreateWithFlags(&before_, hipEventDisableTiming));
    SML_CHECK_HIP(hipEventCreateWithFlags(&after_, hipEventDisableTiming));
  }
  ~StreamRingPy() {
    if (running_) (void)hipStreamSynchronize(train_);
    (void)hipEventDestroy(before_);
    (void)hipEventDestroy(after_);
    (void)hipStreamDestroy(train_);
  }
  at::Tensor ring() const {
    auto opts = at::TensorOptions().dtype(at::kFloat).device(at::kCUDA, (int)dev_);
    return torch::from_blob(ring_.ring(), {ring_.rows(), (int64_t)ring_.features()}, opts);
  }
  void reset() {
    TORCH_CHECK(!running_, "StreamRing.reset: join() the running epoch first");
    ring_.reset();
  }
  void train(const at::Tensor& cursor, const c10::optional<at::Tensor>& scale, const c10::optional<at::Tensor>& shift,
             const at::Tensor& params, const at::Tensor& m, const at::Tensor& v, const at::Tensor& iter,
             const c10::optional<at::Tensor>& metrics, int64_t batch, int64_t max_steps, std::vector<int64_t> dims,
             std::vector<int64_t> acts, double l1, double lr, double beta1, double beta2, double eps, double gscale,
             bool want_acc, double timeout_s, int64_t precision) {
    TORCH_CHECK(!running_, "StreamRing.train: an epoch is already running");
    TORCH_CHECK(ring_.pushed() == 0 && ring_.consumed() == 0, "StreamRing.train: reset() the ring first");
    TORCH_CHECK(ring_.rows() % batch == 0, "StreamRing: ring rows must be a multiple of the batch");
    TORCH_CHECK(params.numel() == sml::ae_nparam(), "StreamRing.train: one model");
    TORCH_CHECK(params.device().index() == dev_, "StreamRing.train: parameters on another device");
    c10::hip::HIPGuard guard((int)dev_);
    // the kernel sees everything queued before it on the caller's stream (params, cursor)
    SML_CHECK_HIP(hipEventRecord(before_, cur_stream(params)));
    SML_CHECK_HIP(hipStreamWaitEvent(train_, before_, 0));
    const sml::MBStream sr = ring_.counters(timeout_s);
    train_minibatches_impl(ring(), cursor, scale, shift, params, m, v, iter, metrics, batch, max_steps,
                           std::move(dims), std::move(acts), l1, lr, beta1, beta2, eps, gscale, want_acc,
                           c10::nullopt, c10::nullopt, 0, 1, 0, 0, 0, c10::nullopt, &sr, train_, precision);
    SML_CHECK_HIP(hipEventRecord(after_, train_));
    running_ = true;
  }
  void push(const at::Tensor& x, double timeout_s) {
    check_dev(x, "rows", at::kFloat);
    TORCH_CHECK(x.dim() == 2 && x.size(1) >= ring_.features() && x.stride(1) == 1, "rows must be [n, >= features]");
    TORCH_CHECK(x.device().index() == dev_, "rows on another device");
    if (x.size(0) == 0) return;
    py::gil_scoped_release nogil;   // may block on back-pressure while the kernel trains
    ring_.push(x.data_ptr<float>(), x.size(0), x.stride(0), cur_stream(x), timeout_s);
  }
  void finish() { ring_.finish(); }
  // the caller's stream waits for the epoch's kernel; returns the kernel's status
  int join() {
    if (running_) {
      c10::hip::HIPGuard guard((int)dev_);
      SML_CHECK_HIP(hipStreamWaitEvent(c10::hip::getCurrentHIPStream((int)dev_).stream(), after_, 0));
      running_ = false;
    }
    return ring_.status();
  }
  // wait on the host for the kernel (used before reading counters)
  void synchronize() {
    py::gil_scoped_release nogil;
    SML_CHECK_HIP(hipEventSynchronize(after_));
  }
  int64_t pushed() const { return ring_.pushed(); }
  int64_t consumed() const { return ring_.consumed(); }
  int status() const { return ring_.status(); }
  int64_t rows() const { return ring_.rows(); }

 private:
  int64_t dev_;
  sml::StreamRing ring_;
  hipStream_t train_ = nullptr;
  hipEvent_t before_ = nullptr, after_ = nullptr;
  bool running_ = false;
};

void ae_forward(const at::Tensor& x, const c10::optional<at::Tensor>& scale, const c10::optional<at::Tensor>& shift,
                const at::Tensor& params, const c10::optional<at::Tensor>& recon,
                const c10::optional<at::Tensor>& score, const c10::optional<at::Tensor>& flag, double threshold,
                std::vector<int64_t> dims, std::vector<int64_t> acts, int64_t max_blocks,
                const c10::optional<at::Tensor>& metrics) {
  check_ae_dims(dims, acts);
  if (metrics.has_value() && metrics->defined())
    TORCH_CHECK(metrics->is_cuda() && metrics->scalar_type() == at::kFloat && metrics->numel() >= 4 &&
                    metrics->is_contiguous(), "metrics must be a float32 device tensor of >= 4 sums");
  check_dev(x, "x", at::kFloat);
  TORCH_CHECK(x.dim() == 2 && x.stride(1) == 1, "x must be [n, ld]");
  TORCH_CHECK(x.size(1) >= dims[0], "x has fewer columns than the model input dim");
  check_dev(params, "params", at::kFloat);
  TORCH_CHECK(params.numel() == sml::ae_nparam(), "params must be the padded image");
  const int64_t n = x.size(0);
  if (recon.has_value()) TORCH_CHECK(recon->numel() >= n * dims[0] && recon->is_contiguous(), "recon too small");
  if (score.has_value()) TORCH_CHECK(score->numel() >= n, "score too small");
  uint8_t* flag_ptr = nullptr;
  if (flag.has_value() && flag->defined()) {
    TORCH_CHECK(flag->scalar_type() == at::kByte && flag->numel() >= n, "flag must be uint8[n]");
    flag_ptr = flag->data_ptr<uint8_t>();
  }
  if (scale.has_value()) TORCH_CHECK(shift.has_value(), "scale requires shift");
  c10::hip::HIPGuard guard(x.device().index());
  int d[4] = {(int)dims[0], (int)dims[1], (int)dims[2], (int)dims[3]};
  int a[4] = {(int)acts[0], (int)acts[1], (int)acts[2], (int)acts[3]};
  SML_CHECK_HIP(sml::ae_forward_launch(x.data_ptr<float>(), n, x.stride(0), opt_ptr(scale), opt_ptr(shift),
                                       params.data_ptr<float>(), opt_mut(recon), opt_mut(score), flag_ptr,
                                       (float)threshold, d, a, (int)max_blocks, cur_stream(x), opt_mut(metrics)));
}

std::vector<at::Tensor> lstm_fwd(const at::Tensor& zx, const at::Tensor& Uw, const c10::optional<at::Tensor>& h0,
                                 const c10::optional<at::Tensor>& c0, int64_t act) {
  check_dev(zx, "zx", at::kFloat);
  check_dev(Uw, "U", at::kFloat);
  TORCH_CHECK(zx.dim() == 3 && zx.is_contiguous(), "zx must be contiguous [B, T, 4u]");
  TORCH_CHECK(Uw.dim() == 2 && Uw.is_contiguous() && Uw.size(1) == 4 * Uw.size(0), "U must be [u, 4u]");
  const int64_t B = zx.size(0), T = zx.size(1), U = Uw.size(0);
  TORCH_CHECK(zx.size(2) == 4 * U, "zx last dim must be 4u");
  TORCH_CHECK(U == 16 || U == 32 || U == 64 || U == 128,
              "LSTM units must be 16, 32, 64 or 128 (ops/lstm.py zero-pads other widths up to one of them)");
  TORCH_CHECK(act == 1 || act == 2, "LSTM activation must be relu or tanh");
  TORCH_CHECK(T >= 1 && B >= 1, "empty input");
  if (h0.has_value()) TORCH_CHECK(h0->is_contiguous() && h0->numel() == B * U, "h0 must be [B, u]");
  if (c0.has_value()) TORCH_CHECK(c0->is_contiguous() && c0->numel() == B * U, "c0 must be [B, u]");
  c10::hip::HIPGuard guard(zx.device().index());
  auto h = at::empty({B, T, U}, zx.options());
  auto c = at::empty({B, T, U}, zx.options());
  auto gt = at::empty({B, T, 4 * U}, zx.options());
  SML_CHECK_HIP(sml::lstm_fwd_launch(zx.data_ptr<float>(), Uw.data_ptr<float>(), opt_ptr(h0), opt_ptr(c0),
                                     h.data_ptr<float>(), c.data_ptr<float>(), gt.data_ptr<float>(), B, (int)T,
                                     (int)U, (int)act, cur_stream(zx)));
  return {h, c, gt};
}

std::vector<at::Tensor> lstm_bwd(const at::Tensor& dh, const at::Tensor& gates, const at::Tensor& cseq,
                                 const c10::optional<at::Tensor>& c0, const at::Tensor& Uw, int64_t act,
                                 bool want_state_grads) {
  check_dev(dh, "dh", at::kFloat);
  check_dev(gates, "gates", at::kFloat);
  check_dev(cseq, "cseq", at::kFloat);
  check_dev(Uw, "U", at::kFloat);
  const int64_t B = dh.size(0), T = dh.size(1), U = Uw.size(0);
  TORCH_CHECK(dh.is_contiguous() && gates.is_contiguous() && cseq.is_contiguous(), "inputs must be contiguous");
  TORCH_CHECK(dh.sizes() == cseq.sizes() && gates.size(2) == 4 * U && dh.size(2) == U, "shape mismatch");
  TORCH_CHECK(U == 16 || U == 32 || U == 64 || U == 128,
              "LSTM units must be 16, 32, 64 or 128 (ops/lstm.py zero-pads other widths up to one of them)");
  if (c0.has_value()) TORCH_CHECK(c0->is_contiguous() && c0->numel() == B * U, "c0 must be [B, u]");
  c10::hip::HIPGuard guard(dh.device().index());
  auto dz = at::empty({B, T, 4 * U}, dh.options());
  at::Tensor dh0, dc0;
  if (want_state_grads) {
    dh0 = at::empty({B, U}, dh.options());
    dc0 = at::empty({B, U}, dh.options());
  }
  SML_CHECK_HIP(sml::lstm_bwd_launch(dh.data_ptr<float>(), gates.data_ptr<float>(), cseq.data_ptr<float>(),
                                     opt_ptr(c0), Uw.data_ptr<float>(), dz.data_ptr<float>(),
                                     want_state_grads ? dh0.data_ptr<float>() : nullptr,
                                     want_state_grads ? dc0.data_ptr<float>() : nullptr, B, (int)T, (int)U,
                                     (int)act, cur_stream(dh)));
  if (want_state_grads) return {dz, dh0, dc0};
  return {dz};
}

// Fused softmax + sparse CE: writes dlogits (= (softmax - onehot) * gscale) and/or
// probabilities, and accumulates [loss_sum, correct] into acc.
void softmax_xent(const at::Tensor& logits, const at::Tensor& labels, double gscale,
                  const c10::optional<at::Tensor>& dlogits, const c10::optional<at::Tensor>& probs,
                  const c10::optional<at::Tensor>& acc) {
  check_dev(logits, "logits", at::kFloat);
  check_dev(labels, "labels", at::kLong);
  TORCH_CHECK(logits.dim() == 2 && logits.is_contiguous(), "logits must be contiguous [B, C]");
  const int64_t B = logits.size(0), C = logits.size(1);
  TORCH_CHECK(labels.numel() == B && labels.is_contiguous(), "labels must be [B]");
  TORCH_CHECK(C == 2 || C == 10 || C == 16 || C == 32, "softmax_xent supports C in {2, 10, 16, 32}");
  for (const auto* t : {&dlogits, &probs}) {
    if (t->has_value()) {
      check_dev(**t, "out", at::kFloat);
      TORCH_CHECK((*t)->is_contiguous() && (*t)->sizes() == logits.sizes(), "output must match logits");
    }
  }
  if (acc.has_value()) {
    check_dev(*acc, "acc", at::kFloat);
    TORCH_CHECK(acc->numel() >= 2, "acc must hold 2 floats");
  }
  c10::hip::HIPGuard guard(logits.device().index());
  SML_CHECK_HIP(sml::softmax_xent_launch(logits.data_ptr<float>(), labels.data_ptr<int64_t>(), B, (int)C,
                                         (float)gscale, opt_mut(dlogits), opt_mut(probs), opt_mut(acc),
                                         cur_stream(logits)));
}

// K1: Y = act(X . W + b) for tall-skinny X [M, K] (fp32 or bf16), W [K, N] fp32.
// w_t: W is a contiguous [N, K] weight applied transposed (dX = dY . W^T, no W^T copy).
at::Tensor dense_fwd(const at::Tensor& x, const at::Tensor& W, const c10::optional<at::Tensor>& bias, int64_t act,
                     bool out_bf16, int64_t max_blocks, bool w_t) {
  TORCH_CHECK(x.is_cuda() && W.is_cuda(), "dense_fwd needs ROCm device tensors");
  TORCH_CHECK(x.scalar_type() == at::kFloat || x.scalar_type() == at::kBFloat16, "x must be fp32 or bf16");
  TORCH_CHECK(x.dim() == 2 && x.stride(1) == 1, "x must be [M, K] with unit inner stride");
  check_dev(W, "W", at::kFloat);
  TORCH_CHECK(W.dim() == 2 && W.is_contiguous() && W.size(w_t ? 1 : 0) == x.size(1),
              w_t ? "W must be contiguous [N, K]" : "W must be contiguous [K, N]");
  const int64_t M = x.size(0), K = x.size(1), N = W.size(w_t ? 0 : 1);
  TORCH_CHECK(sml::dense_supported((int)K, (int)N), "dense_fwd: K=", K, " N=", N, " exceeds the register tile");
  if (bias.has_value()) {
    check_dev(*bias, "bias", at::kFloat);
    TORCH_CHECK(bias->numel() == N && bias->is_contiguous(), "bias must be [N]");
  }
  TORCH_CHECK(act >= 0 && act <= 3, "act must be 0..3");
  c10::hip::HIPGuard guard(x.device().index());
  auto y = at::empty({M, N}, x.options().dtype(out_bf16 ? at::kBFloat16 : at::kFloat));
  SML_CHECK_HIP(sml::rowgemm_launch(x.data_ptr(), x.scalar_type() == at::kBFloat16, M, (int)K, x.stride(0),
                                    W.data_ptr<float>(), opt_ptr(bias), (int)N, (int)act, y.data_ptr(), out_bf16, N,
                                    (int)max_blocks, cur_stream(x), w_t ? 1 : 0));
  return y;
}

// Optional (grad, map) pair of the weight-gradient bindings: the final slab reduction
// writes slab element s straight to grad[map[s]] (the parameter's place in a flat
// gradient buffer, transposes included; map[s] < 0 drops padding), so a train step
// needs no copy / transpose / accumulate kernels between the backward and Adam.
static const int* grad_map(const c10::optional<at::Tensor>& grad, const c10::optional<at::Tensor>& map, int S) {
  TORCH_CHECK(grad.has_value() == map.has_value(), "grad and map go together");
  if (!grad.has_value()) return nullptr;
  check_dev(*grad, "grad", at::kFloat);
  TORCH_CHECK(grad->is_contiguous(), "grad must be contiguous");
  TORCH_CHECK(map->is_cuda() && map->scalar_type() == at::kInt && map->is_contiguous() && map->numel() == S,
              "map must be a device int32 tensor of the slab size ", S);
  return map->data_ptr<int>();
}

// K2 (weight half): dW = X^T . dY, db = colsum(dY) over M rows (split-row MFMA + slab reduce).
// shift_T > 0: X row r is read as X[r - 1] (zero when r % shift_T == 0).
std::vector<at::Tensor> dense_wgrad(const at::Tensor& x, const at::Tensor& dy, int64_t shift_T, bool want_db,
                                    int64_t max_blocks, const c10::optional<at::Tensor>& grad,
                                    const c10::optional<at::Tensor>& map) {
  TORCH_CHECK(x.is_cuda() && dy.is_cuda(), "dense_wgrad needs ROCm device tensors");
  for (const auto* t : {&x, &dy}) {
    TORCH_CHECK(t->scalar_type() == at::kFloat || t->scalar_type() == at::kBFloat16, "inputs must be fp32 or bf16");
    TORCH_CHECK(t->dim() == 2 && t->stride(1) == 1, "inputs must be 2-D with unit inner stride");
  }
  TORCH_CHECK(x.size(0) == dy.size(0), "row count mismatch");
  const int64_t M = x.size(0), K = x.size(1), N = dy.size(1);
  TORCH_CHECK(sml::dense_supported((int)K, (int)N), "dense_wgrad: K=", K, " N=", N, " exceeds the register tile");
  c10::hip::HIPGuard guard(x.device().index());
  const int S = sml::dense_wgrad_slab((int)K, (int)N);
  const int G = sml::dense_wgrad_grid(M, (int)max_blocks);
  auto opts = x.options().dtype(at::kFloat);
  const int* mp = grad_map(grad, map, S);
  auto partials = at::empty({G, S}, opts);
  auto out = mp ? *grad : at::empty({S}, opts);
  auto scratch = at::empty({std::max(1, sml::slab_sum_scratch(G, S))}, opts);
  auto st = cur_stream(x);
  SML_CHECK_HIP(sml::wgrad_launch(x.data_ptr(), x.scalar_type() == at::kBFloat16, M, (int)K, x.stride(0),
                                  (int)shift_T, dy.data_ptr(), dy.scalar_type() == at::kBFloat16, (int)N,
                                  dy.stride(0), want_db ? 1 : 0, partials.data_ptr<float>(), G, st));
  SML_CHECK_HIP(sml::slab_sum_launch(partials.data_ptr<float>(), G, S, scratch.data_ptr<float>(),
                                     out.data_ptr<float>(), st, mp));
  if (mp) return {at::Tensor(), at::Tensor()};
  const int64_t KP = 16 * sml::dense_tiles((int)K), NP = 16 * sml::dense_tiles((int)N);
  auto dW = out.narrow(0, 0, KP * NP).view({KP, NP}).narrow(0, 0, K).narrow(1, 0, N);
  auto db = out.narrow(0, KP * NP, N);
  return {dW, db};
}

// Orientation of one GEMM operand view: kc = 1 when the contraction dim has unit stride
// (element (mn, k) at p[mn * ld + k]), kc = 0 when the mn dim has (p[k * ld + mn]); any
// other strided view is made contiguous first.
static at::Tensor gemm_operand(const at::Tensor& t, int mn_dim, int k_dim, int64_t& ld, int& kc) {
  const int64_t smn = t.stride(mn_dim), sk = t.stride(k_dim), nmn = t.size(mn_dim), nk = t.size(k_dim);
  if ((sk == 1 || nk <= 1) && (nmn <= 1 || smn >= nk)) {
    kc = 1;
    ld = nmn <= 1 ? std::max<int64_t>(nk, 1) : smn;
    return t;
  }
  if ((smn == 1 || nmn <= 1) && (nk <= 1 || sk >= nmn)) {
    kc = 0;
    ld = nk <= 1 ? std::max<int64_t>(nmn, 1) : sk;
    return t;
  }
  at::Tensor c = t.contiguous();
  return gemm_operand(c, mn_dim, k_dim, ld, kc);
}

// General MFMA GEMM (gemm.hip): act(a . b + bias) for a [M, K], b [K, N] (fp32 or bf16,
// either orientation -- transposed views need no copy).  splits: 1 = no split-K, > 1 =
// that many K slices reduced deterministically, < 0 = choose from the shape (only when
// there is no bias / activation and the output is fp32).
at::Tensor gemm(const at::Tensor& a, const at::Tensor& b, const c10::optional<at::Tensor>& bias, int64_t act,
                bool out_bf16, int64_t splits) {
  TORCH_CHECK(a.is_cuda() && b.is_cuda(), "gemm needs ROCm device tensors");
  for (const auto* t : {&a, &b})
    TORCH_CHECK(t->dim() == 2 && (t->scalar_type() == at::kFloat || t->scalar_type() == at::kBFloat16),
                "gemm operands must be 2-D fp32 or bf16");
  TORCH_CHECK(a.size(1) == b.size(0), "gemm: inner dims differ (", a.size(1), " vs ", b.size(0), ")");
  TORCH_CHECK(a.device() == b.device(), "gemm operands must be on one device");
  TORCH_CHECK(act >= 0 && act <= 3, "act must be 0..3");
  const int64_t M = a.size(0), K = a.size(1), N = b.size(1);
  if (bias.has_value()) {
    check_dev(*bias, "bias", at::kFloat);
    TORCH_CHECK(bias->numel() == N && bias->is_contiguous() && bias->device() == a.device(), "bias must be [N]");
  }
  c10::hip::HIPGuard guard(a.device().index());
  int64_t lda = 0, ldb = 0;
  int akc = 1, bkc = 1;
  const at::Tensor A = gemm_operand(a, 0, 1, lda, akc);
  // A small fp32 B (a layer's weight) is re-read and re-converted by every one of the M / 128
  // row tiles: convert it to bf16 once (one pass over <= 4 M elements) when there are many.
  // SML_GEMM_BF16_B=0 keeps the in-kernel conversion (A/B).
  static const bool pre_b = [] {
    const char* e = std::getenv("SML_GEMM_BF16_B");
    return !(e && e[0] == '0');
  }();
  const bool cast_b = pre_b && b.scalar_type() == at::kFloat && b.numel() <= (int64_t(1) << 22) && M >= 8 * 128;
  const at::Tensor B = gemm_operand(cast_b ? b.to(at::kBFloat16) : b, 1, 0, ldb, bkc);
  const int64_t Np = (N + 3) & ~int64_t(3);
  const bool plain = !bias.has_value() && act == 0 && !out_bf16;
  int s = 1;
  if (plain && M * Np < (int64_t(1) << 31)) {
    if (splits < 0) {
      static const int cus = [] {
        hipDeviceProp_t p;
        return hipGetDeviceProperties(&p, 0) == hipSuccess ? p.multiProcessorCount : 256;
      }();
      s = sml::gemm_auto_splits(M, N, K, cus);
    } else if (splits > 1) {
      s = (int)std::min<int64_t>(splits, 4096);
    }
  }
  auto st = cur_stream(a);
  auto opts = a.options().dtype(at::kFloat);
  if (s > 1) {
    auto partials = at::empty({s, M * Np}, opts);
    auto out = at::empty({M, Np}, opts);
    auto scratch = at::empty({std::max(1, sml::slab_sum_scratch(s, (int)(M * Np)))}, opts);
    SML_CHECK_HIP(sml::gemm_launch(A.data_ptr(), A.scalar_type() == at::kBFloat16, lda, akc, B.data_ptr(),
                                   B.scalar_type() == at::kBFloat16, ldb, bkc, M, N, K, nullptr, 0, nullptr, 0, Np,
                                   partials.data_ptr<float>(), s, st));
    SML_CHECK_HIP(sml::slab_sum_launch(partials.data_ptr<float>(), s, (int)(M * Np), scratch.data_ptr<float>(),
                                       out.data_ptr<float>(), st));
    return Np == N ? out : out.narrow(1, 0, N);
  }
  auto c = at::empty({M, N}, a.options().dtype(out_bf16 ? at::kBFloat16 : at::kFloat));
  SML_CHECK_HIP(sml::gemm_launch(A.data_ptr(), A.scalar_type() == at::kBFloat16, lda, akc, B.data_ptr(),
                                 B.scalar_type() == at::kBFloat16, ldb, bkc, M, N, K, opt_ptr(bias), (int)act,
                                 c.data_ptr(), out_bf16, N, nullptr, 1, st));
  return c;
}

// Fully fused LSTM layer forward: x [B, T, IN] fp32 or bf16 -> (h [B,T,U] bf16, c: bf16
// cell state for lstm_fused_bwd).
std::vector<at::Tensor> lstm_fused_fwd(const at::Tensor& x, const at::Tensor& W, const at::Tensor& Uw,
                                       const at::Tensor& b, const c10::optional<at::Tensor>& h0,
                                       const c10::optional<at::Tensor>& c0, int64_t act) {
  TORCH_CHECK(x.is_cuda() && (x.scalar_type() == at::kFloat || x.scalar_type() == at::kBFloat16),
              "x must be a float32 or bfloat16 device tensor");
  check_dev(W, "W", at::kFloat);
  check_dev(Uw, "U", at::kFloat);
  check_dev(b, "b", at::kFloat);
  // x: contiguous [B, T, IN], or a strided view whose steps are consecutive rows --
  // sliding windows base.as_strided((B, T, IN), (shift*IN, IN, 1)) read in place
  TORCH_CHECK(x.dim() == 3 && x.stride(2) == 1 && x.stride(1) == x.size(2) && x.stride(0) >= 0,
              "x must be [B, T, IN] with consecutive rows per step (contiguous or sliding windows)");
  const int64_t B = x.size(0), T = x.size(1), IN = x.size(2), U = Uw.size(0);
  const int64_t x_seq = B > 1 ? x.stride(0) : T * IN;
  TORCH_CHECK(W.is_contiguous() && W.size(0) == IN && W.size(1) == 4 * U, "W must be [IN, 4U]");
  TORCH_CHECK(Uw.is_contiguous() && Uw.size(1) == 4 * U, "U must be [U, 4U]");
  TORCH_CHECK(b.is_contiguous() && b.numel() == 4 * U, "b must be [4U]");
  TORCH_CHECK(sml::lstm_fused_supported((int)U, (int)IN), "fused LSTM: unsupported U=", U, " IN=", IN);
  TORCH_CHECK(act == 1 || act == 2, "LSTM activation must be relu or tanh");
  TORCH_CHECK(B >= 1 && T >= 1, "empty input");
  if (h0.has_value()) TORCH_CHECK(h0->is_contiguous() && h0->numel() == B * U, "h0 must be [B, U]");
  if (c0.has_value()) TORCH_CHECK(c0->is_contiguous() && c0->numel() == B * U, "c0 must be [B, U]");
  c10::hip::HIPGuard guard(x.device().index());
  // h and the cell state are padded to whole 16-sequence waves (the kernel stores
  // unmasked); c is saved for BPTT only, in the kernels' fragment-native order
  // (lstm_fused.hip header); the gates are recomputed there
  const int64_t Bp = (B + 15) / 16 * 16;
  auto bf = x.options().dtype(at::kBFloat16);
  auto h = at::empty({Bp, T, U}, bf);
  auto c = at::empty({Bp, T, U}, bf);
  SML_CHECK_HIP(sml::lstm_fused_fwd_launch(x.data_ptr(), x.scalar_type() == at::kBFloat16, W.data_ptr<float>(),
                                           Uw.data_ptr<float>(), b.data_ptr<float>(), opt_ptr(h0), opt_ptr(c0),
                                           h.data_ptr(), c.data_ptr(), B, (int)T, (int)IN, (int)U, (int)act,
                                           x_seq, cur_stream(x)));
  return {h.narrow(0, 0, B), c};
}

// Two stacked fused LSTM layers in one forward launch -> [h1 [B,T,U1] bf16, c1 (padded, fragment
// order), h2 [B,T,U2] bf16, c2] -- the same four tensors two lstm_fused_fwd calls return.
std::vector<at::Tensor> lstm_fused_fwd2(const at::Tensor& x, const at::Tensor& W1, const at::Tensor& U1,
                                        const at::Tensor& b1, const at::Tensor& W2, const at::Tensor& U2,
                                        const at::Tensor& b2, int64_t act1, int64_t act2, bool hfrag) {
  TORCH_CHECK(x.is_cuda() && x.scalar_type() == at::kFloat, "x must be a float32 device tensor");
  for (const auto* t : {&W1, &U1, &b1, &W2, &U2, &b2}) check_dev(*t, "weights", at::kFloat);
  TORCH_CHECK(x.dim() == 3 && x.stride(2) == 1 && x.stride(1) == x.size(2) && x.stride(0) >= 0,
              "x must be [B, T, IN] with consecutive rows per step (contiguous or sliding windows)");
  const int64_t B = x.size(0), T = x.size(1), IN = x.size(2), Ua = U1.size(0), Ub = U2.size(0);
  const int64_t x_seq = B > 1 ? x.stride(0) : T * IN;
  TORCH_CHECK(W1.is_contiguous() && W1.size(0) == IN && W1.size(1) == 4 * Ua, "W1 must be [IN, 4U1]");
  TORCH_CHECK(U1.is_contiguous() && U1.size(1) == 4 * Ua, "U1 must be [U1, 4U1]");
  TORCH_CHECK(b1.is_contiguous() && b1.numel() == 4 * Ua, "b1 must be [4U1]");
  TORCH_CHECK(W2.is_contiguous() && W2.size(0) == Ua && W2.size(1) == 4 * Ub, "W2 must be [U1, 4U2]");
  TORCH_CHECK(U2.is_contiguous() && U2.size(1) == 4 * Ub, "U2 must be [U2, 4U2]");
  TORCH_CHECK(b2.is_contiguous() && b2.numel() == 4 * Ub, "b2 must be [4U2]");
  TORCH_CHECK(sml::lstm_fused_fwd2_supported((int)IN, (int)Ua, (int)Ub, (int)act1, (int)act2),
              "fused two-layer LSTM forward: unsupported IN=", IN, " U1=", Ua, " U2=", Ub);
  TORCH_CHECK(B >= 1 && T >= 1, "empty input");
  c10::hip::HIPGuard guard(x.device().index());
  const int64_t Bp = (B + 15) / 16 * 16;
  const int64_t Bw = std::max<int64_t>(Bp, sml::lstm_fused_fwd2_rows(B));   // whole waves of the kernel's tiles
  auto bf = x.options().dtype(at::kBFloat16);
  auto h1 = at::empty({Bw, T, Ua}, bf), c1 = at::empty({Bw, T, Ua}, bf);
  auto h2 = at::empty({Bw, T, Ub}, bf), c2 = at::empty({Bw, T, Ub}, bf);
  at::Tensor hl = hfrag ? at::empty({Bp, Ub}, bf) : at::Tensor();
  SML_CHECK_HIP(sml::lstm_fused_fwd2_launch(x.data_ptr<float>(), W1.data_ptr<float>(), U1.data_ptr<float>(),
                                            b1.data_ptr<float>(), W2.data_ptr<float>(), U2.data_ptr<float>(),
                                            b2.data_ptr<float>(), h1.data_ptr(), c1.data_ptr(), h2.data_ptr(),
                                            c2.data_ptr(), hfrag ? hl.data_ptr() : nullptr, B, (int)T, (int)IN,
                                            (int)act1, (int)act2, x_seq, cur_stream(x)));
  // c: the 16-sequence-padded prefix the backward expects (contiguous).  hfrag: h1 / h2 hold the
  // fragment-native sequences (views of B rows over the padded buffers, for lstm_fused_bwd frag=True)
  // and the fifth tensor is layer 2's h_T [B, U2]
  return {h1.narrow(0, 0, B), c1.narrow(0, 0, Bp), h2.narrow(0, 0, B), c2.narrow(0, 0, Bp),
          hfrag ? hl.narrow(0, 0, B) : at::Tensor()};
}

// Fully fused LSTM layer backward -> [dx (x's dtype, or undefined), dW [IN,4U], dU [U,4U],
// db [4U], dh0, dc0].  dh: bf16 [B, T, U], or [B, U] (h_T only) when dh_last_only.
std::vector<at::Tensor> lstm_fused_bwd(const at::Tensor& dh, const at::Tensor& cseq, const at::Tensor& hseq,
                                       const at::Tensor& x, const c10::optional<at::Tensor>& h0,
                                       const c10::optional<at::Tensor>& c0, const at::Tensor& W, const at::Tensor& Uw,
                                       const at::Tensor& b, int64_t act, bool want_dx, bool want_state_grads,
                                       bool dh_last_only, const c10::optional<at::Tensor>& grad,
                                       const c10::optional<at::Tensor>& map, bool frag, bool defer_sum) {
  check_dev(dh, "dh", at::kBFloat16);
  check_dev(cseq, "c", at::kBFloat16);
  check_dev(hseq, "h", at::kBFloat16);
  TORCH_CHECK(x.is_cuda() && (x.scalar_type() == at::kFloat || x.scalar_type() == at::kBFloat16),
              "x must be a float32 or bfloat16 device tensor");
  check_dev(W, "W", at::kFloat);
  check_dev(Uw, "U", at::kFloat);
  check_dev(b, "b", at::kFloat);
  const int64_t B = x.size(0), T = x.size(1), IN = x.size(2), U = Uw.size(0);
  TORCH_CHECK(dh.is_contiguous() && cseq.is_contiguous() && hseq.is_contiguous(), "inputs must be contiguous");
  TORCH_CHECK(x.dim() == 3 && x.stride(2) == 1 && x.stride(1) == IN && x.stride(0) >= 0,
              "x must be [B, T, IN] with consecutive rows per step (contiguous or sliding windows)");
  const int64_t x_seq = B > 1 ? x.stride(0) : T * IN;
  const int64_t Bp = (B + 15) / 16 * 16;
  TORCH_CHECK(hseq.size(0) == B && hseq.size(1) == T && hseq.size(2) == U, "h shape mismatch");
  TORCH_CHECK(cseq.dim() == 3 && cseq.size(0) == Bp && cseq.size(1) == T && cseq.size(2) == U,
              "c must be the padded buffer lstm_fused_fwd returned");
  TORCH_CHECK(W.is_contiguous() && W.size(0) == IN && W.size(1) == 4 * U && Uw.is_contiguous() &&
              Uw.size(1) == 4 * U && b.is_contiguous() && b.numel() == 4 * U, "weight shape mismatch");
  if (dh_last_only) {
    TORCH_CHECK(dh.dim() == 2 && dh.size(0) == B && dh.size(1) == U, "dh must be [B, U] (h_T only)");
  } else {
    TORCH_CHECK(dh.sizes() == hseq.sizes(), "dh must be [B, T, U]");
  }
  TORCH_CHECK(sml::lstm_fused_supported((int)U, (int)IN), "fused LSTM: unsupported U=", U, " IN=", IN);
  // frag: h (and a bf16 x, and dh unless dh_last_only) are fragment-native sequences as
  // lstm_fused_fwd2(hfrag=True) / this function's frag dx produce them (B-row views over buffers
  // padded to whole 16-sequence tiles); dx comes back fragment-native too
  TORCH_CHECK(!frag || sml::lstm_fused_frag_supported((int)U, (int)IN, x.scalar_type() == at::kBFloat16, want_dx),
              "fused LSTM: no fragment-mode instance for U=", U, " IN=", IN);
  c10::hip::HIPGuard guard(x.device().index());
  auto opts = x.options().dtype(at::kFloat);
  at::Tensor dx, dh0, dc0;
  at::Tensor dx_pad;
  if (want_dx) dx_pad = at::empty({Bp, T, (int64_t)sml::lstm_fused_dx_ld((int)IN)}, x.options());
  if (want_state_grads) {
    dh0 = at::empty({B, U}, opts);
    dc0 = at::empty({B, U}, opts);
  }
  const int S = sml::lstm_fused_slab((int)U, (int)IN);
  const int G = sml::lstm_fused_bwd_slabs(B, (int)U, (int)IN, want_dx, x.scalar_type() == at::kBFloat16, dh_last_only);
  const int* mp = grad_map(grad, map, S);
  auto partials = at::empty({G, S}, opts);   // every workgroup writes its slab (idle waves add nothing)
  auto out = mp ? *grad : at::empty({S}, opts);
  auto scratch = at::empty({std::max(1, sml::slab_sum_scratch(G, S))}, opts);
  const int64_t dzb = sml::lstm_fused_dz_bytes(B, (int)T, (int)U);   // U >= 64: dz for the gate-group wgrad
  at::Tensor dzs = dzb > 0 ? at::empty({dzb / 2}, x.options().dtype(at::kBFloat16)) : at::Tensor();
  auto st = cur_stream(x);
  SML_CHECK_HIP(sml::lstm_fused_bwd_launch(
      dh.data_ptr(), cseq.data_ptr(), hseq.data_ptr(), x.data_ptr(), x.scalar_type() == at::kBFloat16, opt_ptr(h0),
      opt_ptr(c0), W.data_ptr<float>(), Uw.data_ptr<float>(), b.data_ptr<float>(),
      want_dx ? dx_pad.data_ptr() : nullptr, want_state_grads ? dh0.data_ptr<float>() : nullptr,
      want_state_grads ? dc0.data_ptr<float>() : nullptr, partials.data_ptr<float>(), B, (int)T, (int)IN, (int)U,
      (int)act, dh_last_only ? 1 : 0, x_seq, dzb > 0 ? dzs.data_ptr() : nullptr, frag ? 1 : 0, st));
  // defer_sum (with grad + map): the weight-gradient slabs come back unreduced as the second output, for
  // slab_sum2 to reduce together with another layer's in one launch
  TORCH_CHECK(!defer_sum || mp, "defer_sum needs grad and map");
  if (defer_sum) {
    at::Tensor dxo;
    if (want_dx) {
      dxo = dx_pad.narrow(0, 0, B);
      if (dx_pad.size(2) != IN && !frag) dxo = dxo.narrow(2, 0, IN).contiguous();
    }
    return {dxo, partials, at::Tensor(), at::Tensor(), dh0, dc0};
  }
  SML_CHECK_HIP(sml::slab_sum_launch(partials.data_ptr<float>(), G, S, scratch.data_ptr<float>(),
                                     out.data_ptr<float>(), st, mp));
  const int64_t G4 = 4 * U, LDW = (S / G4) - U - 1;
  at::Tensor dW, dU, db;
  if (!mp) {
    dW = out.narrow(0, 0, G4 * LDW).view({G4, LDW}).narrow(1, 0, IN).t().contiguous();
    dU = out.narrow(0, G4 * LDW, G4 * U).view({G4, U}).t().contiguous();
    db = out.narrow(0, G4 * LDW + G4 * U, G4);
  }
  if (want_dx) {
    dx = dx_pad.narrow(0, 0, B);
    if (dx_pad.size(2) != IN && !frag) dx = dx.narrow(2, 0, IN).contiguous();
  }
  return {dx, dW, dU, db, dh0, dc0};
}

// Backward of two stacked fused LSTM layers (U 32 -> 16) in one launch.  Layer 1's x (fp32
// model input), its saved h / c, layer 2's saved h / c and layer 2's incoming dh (bf16, [B, 16]
// when dh2_last_only).  With grad + map1 + map2 the two weight-gradient slabs are reduced
// straight into the flat gradient; otherwise returns [dW1, dU1, db1, dW2, dU2, db2].
std::vector<at::Tensor> lstm_fused_bwd2(const at::Tensor& x, const at::Tensor& h1, const at::Tensor& c1,
                                        const at::Tensor& h2, const at::Tensor& c2, const at::Tensor& dh2,
                                        const at::Tensor& W1, const at::Tensor& U1, const at::Tensor& b1,
                                        const at::Tensor& W2, const at::Tensor& U2, const at::Tensor& b2, int64_t act,
                                        bool dh2_last_only, const c10::optional<at::Tensor>& grad,
                                        const c10::optional<at::Tensor>& map1, const c10::optional<at::Tensor>& map2) {
  TORCH_CHECK(x.is_cuda() && x.scalar_type() == at::kFloat, "x must be a float32 device tensor");
  for (const auto* t : {&h1, &c1, &h2, &c2, &dh2}) check_dev(*t, "saved state", at::kBFloat16);
  for (const auto* t : {&W1, &U1, &b1, &W2, &U2, &b2}) check_dev(*t, "weights", at::kFloat);
  TORCH_CHECK(x.dim() == 3 && x.stride(2) == 1 && x.stride(1) == x.size(2) && x.stride(0) >= 0,
              "x must be [B, T, IN] with consecutive rows per step (contiguous or sliding windows)");
  const int64_t B = x.size(0), T = x.size(1), IN = x.size(2);
  const int64_t x_seq = B > 1 ? x.stride(0) : T * IN, Bp = (B + 15) / 16 * 16;
  TORCH_CHECK(h1.is_contiguous() && h1.size(0) == B && h1.size(1) == T && h1.size(2) == 32, "h1 must be [B, T, 32]");
  TORCH_CHECK(h2.is_contiguous() && h2.size(0) == B && h2.size(1) == T && h2.size(2) == 16, "h2 must be [B, T, 16]");
  TORCH_CHECK(c1.is_contiguous() && c1.size(0) == Bp && c1.size(2) == 32 && c2.is_contiguous() && c2.size(0) == Bp &&
                  c2.size(2) == 16, "c1 / c2 must be the padded buffers the forward returned");
  TORCH_CHECK(dh2.is_contiguous() && (dh2_last_only ? (dh2.dim() == 2 && dh2.size(0) == B && dh2.size(1) == 16)
                                                    : dh2.sizes() == h2.sizes()), "dh2 shape mismatch");
  TORCH_CHECK(W1.size(0) == IN && W1.size(1) == 128 && U1.size(0) == 32 && W2.size(0) == 32 && W2.size(1) == 64 &&
                  U2.size(0) == 16 && b1.numel() == 128 && b2.numel() == 64, "weight shape mismatch");
  TORCH_CHECK(sml::lstm_fused_bwd2_supported((int)IN, 32, 16, (int)act, (int)act), "stacked LSTM backward: unsupported");
  c10::hip::HIPGuard guard(x.device().index());
  auto opts = x.options().dtype(at::kFloat);
  const int S1 = sml::lstm_fused_slab(32, (int)IN), S2 = sml::lstm_fused_slab(16, 32);
  const int G = sml::lstm_fused_bwd2_grid(B);
  TORCH_CHECK(map1.has_value() == map2.has_value(), "map1 and map2 go together");
  const int* mp1 = grad_map(grad, map1, S1);
  const int* mp2 = grad.has_value() ? grad_map(grad, map2, S2) : nullptr;
  auto p1 = at::empty({G, S1}, opts), p2 = at::empty({G, S2}, opts);
  auto o1 = mp1 ? *grad : at::empty({S1}, opts);
  auto o2 = mp2 ? *grad : at::empty({S2}, opts);
  auto scratch = at::empty({std::max(1, std::max(sml::slab_sum_scratch(G, S1), sml::slab_sum_scratch(G, S2)))}, opts);
  auto st = cur_stream(x);
  SML_CHECK_HIP(sml::lstm_fused_bwd2_launch(x.data_ptr<float>(), x_seq, (int)IN, h1.data_ptr(), c1.data_ptr(),
                                            h2.data_ptr(), c2.data_ptr(), dh2.data_ptr(), dh2_last_only ? 1 : 0,
                                            W1.data_ptr<float>(), U1.data_ptr<float>(), b1.data_ptr<float>(),
                                            W2.data_ptr<float>(), U2.data_ptr<float>(), b2.data_ptr<float>(),
                                            p1.data_ptr<float>(), p2.data_ptr<float>(), B, (int)T, (int)act, st));
  SML_CHECK_HIP(sml::slab_sum_launch(p1.data_ptr<float>(), G, S1, scratch.data_ptr<float>(), o1.data_ptr<float>(), st,
                                     mp1));
  SML_CHECK_HIP(sml::slab_sum_launch(p2.data_ptr<float>(), G, S2, scratch.data_ptr<float>(), o2.data_ptr<float>(), st,
                                     mp2));
  if (mp1) return {};
  auto unpack = [&](const at::Tensor& o, int64_t U, int64_t in, int S) {
    const int64_t G4 = 4 * U, LDW = (S / G4) - U - 1;
    return std::vector<at::Tensor>{o.narrow(0, 0, G4 * LDW).view({G4, LDW}).narrow(1, 0, in).t().contiguous(),
                                   o.narrow(0, G4 * LDW, G4 * U).view({G4, U}).t().contiguous(),
                                   o.narrow(0, G4 * LDW + G4 * U, G4)};
  };
  auto a1 = unpack(o1, 32, IN, S1), a2 = unpack(o2, 16, 32, S2);
  return {a1[0], a1[1], a1[2], a2[0], a2[1], a2[2]};
}

// ---- MNIST MLP layers (mlp.hip) ----
static void check_x_mlp(const at::Tensor& x) {
  TORCH_CHECK(x.is_cuda() && x.dim() == 2 && x.stride(1) == 1 &&
                  (x.scalar_type() == at::kFloat || x.scalar_type() == at::kByte),
              "x must be a device [B, K] float32 or uint8 tensor with unit column stride");
}

at::Tensor mlp_fwd(const at::Tensor& x, const at::Tensor& W, const c10::optional<at::Tensor>& b, bool relu,
                   double keep, int64_t seed, int64_t step) {
  check_x_mlp(x);
  check_dev(W, "W", at::kFloat);
  TORCH_CHECK(W.is_contiguous() && W.dim() == 2 && W.size(0) == x.size(1), "W must be [K, N] contiguous");
  if (b.has_value()) {
    check_dev(*b, "b", at::kFloat);
    TORCH_CHECK(b->is_contiguous() && b->numel() == W.size(1), "b must be [N]");
  }
  TORCH_CHECK(keep > 0.0 && keep <= 1.0, "keep must be in (0, 1]");
  c10::hip::HIPGuard guard(x.device().index());
  auto y = at::empty({x.size(0), W.size(1)}, x.options().dtype(at::kFloat));
  if (x.size(0) == 0) return y;
  SML_CHECK_HIP(sml::mlp_fwd_launch(x.data_ptr(), x.scalar_type() == at::kByte, x.stride(0), W.data_ptr<float>(),
                                    opt_ptr(b), y.data_ptr<float>(), (int)x.size(0), (int)x.size(1),
                                    (int)W.size(1), relu ? 1 : 0, (float)keep, (uint32_t)seed, (uint32_t)step,
                                    cur_stream(x)));
  return y;
}

at::Tensor mlp_bwd_data(const at::Tensor& dz, const at::Tensor& W, const at::Tensor& h, double keep) {
  check_dev(dz, "dz", at::kFloat);
  check_dev(W, "W", at::kFloat);
  check_dev(h, "h", at::kFloat);
  TORCH_CHECK(dz.is_contiguous() && W.is_contiguous() && h.is_contiguous(), "inputs must be contiguous");
  TORCH_CHECK(W.dim() == 2 && dz.dim() == 2 && h.dim() == 2 && dz.size(1) == W.size(1) && h.size(1) == W.size(0) &&
                  h.size(0) == dz.size(0), "shapes: dz [B, N2], W [N1, N2], h [B, N1]");
  c10::hip::HIPGuard guard(dz.device().index());
  auto dh = at::empty_like(h);
  if (dz.size(0) == 0) return dh;
  SML_CHECK_HIP(sml::mlp_bwd_data_launch(dz.data_ptr<float>(), W.data_ptr<float>(), h.data_ptr<float>(),
                                         dh.data_ptr<float>(), (int)dz.size(0), (int)W.size(0), (int)W.size(1),
                                         (float)(1.0 / keep), cur_stream(dz)));
  return dh;
}

void mlp_wgrad(const at::Tensor& x, const at::Tensor& dy, at::Tensor& out) {
  check_x_mlp(x);
  check_dev(dy, "dy", at::kFloat);
  check_dev(out, "out", at::kFloat);
  TORCH_CHECK(dy.is_contiguous() && out.is_contiguous() && dy.dim() == 2 && dy.size(0) == x.size(0),
              "dy must be [B, N] contiguous");
  TORCH_CHECK(out.numel() == (x.size(1) + 1) * dy.size(1), "out must hold [K + 1, N] (dW then db)");
  c10::hip::HIPGuard guard(x.device().index());
  SML_CHECK_HIP(sml::mlp_wgrad_launch(x.data_ptr(), x.scalar_type() == at::kByte, x.stride(0), dy.data_ptr<float>(),
                                      out.data_ptr<float>(), (int)x.size(0), (int)x.size(1), (int)dy.size(1),
                                      cur_stream(x)));
}

at::Tensor mlp_dropout_mask(const at::Tensor& like, int64_t M, int64_t N, double keep, int64_t seed, int64_t step) {
  TORCH_CHECK(like.is_cuda(), "needs a device tensor for placement");
  c10::hip::HIPGuard guard(like.device().index());
  auto out = at::empty({M, N}, like.options().dtype(at::kFloat));
  SML_CHECK_HIP(sml::mlp_dropout_mask_launch(out.data_ptr<float>(), (int)M, (int)N, (float)keep, (uint32_t)seed,
                                             (uint32_t)step, cur_stream(like)));
  return out;
}

// N consecutive Keras steps of the reference LSTM stack (look_back 1) in one launch.
at::Tensor lstm_ref_train(const at::Tensor& flat, const at::Tensor& m, const at::Tensor& v, const at::Tensor& iter,
                          const at::Tensor& x, const at::Tensor& y, const c10::optional<at::Tensor>& order,
                          int64_t row0, int64_t B, int64_t nsteps, int64_t act, double lr, double beta1, double beta2,
                          double eps) {
  check_dev(flat, "flat", at::kFloat);
  check_dev(m, "m", at::kFloat);
  check_dev(v, "v", at::kFloat);
  check_dev(x, "x", at::kFloat);
  check_dev(y, "y", at::kFloat);
  TORCH_CHECK(iter.is_cuda() && iter.scalar_type() == at::kLong && iter.numel() == 1, "iter must be a device int64[1]");
  const int64_t P = sml::lstm_ref_train_params();
  TORCH_CHECK(flat.is_contiguous() && m.is_contiguous() && v.is_contiguous() && flat.numel() >= P &&
                  m.numel() >= P && v.numel() >= P, "flat / m / v must hold the reference stack's ", P, " parameters");
  TORCH_CHECK(x.dim() == 2 && y.dim() == 2 && x.size(1) == 18 && y.size(1) == 18 && x.stride(1) == 1 &&
                  y.stride(1) == 1 && x.size(0) == y.size(0), "x / y must be [n, 18] row views");
  const int64_t n = x.size(0);
  if (order.has_value()) {
    TORCH_CHECK(order->is_cuda() && order->scalar_type() == at::kInt && order->is_contiguous() && order->numel() == n,
                "order must be a device int32 permutation of the n samples");
  }
  TORCH_CHECK(B >= 1 && B <= 32 && nsteps >= 1 && row0 >= 0 && row0 < n, "bad B / nsteps / row0");
  c10::hip::HIPGuard guard(x.device().index());
  auto out = at::zeros({nsteps, 2}, flat.options());
  SML_CHECK_HIP(sml::lstm_ref_train_launch(flat.data_ptr<float>(), m.data_ptr<float>(), v.data_ptr<float>(),
                                           iter.data_ptr<int64_t>(), x.data_ptr<float>(), x.stride(0),
                                           y.data_ptr<float>(), y.stride(0),
                                           order.has_value() ? order->data_ptr<int32_t>() : nullptr, n, row0, (int)B,
                                           (int)nsteps, (int)act, (float)lr, (float)beta1, (float)beta2, (float)eps,
                                           out.data_ptr<float>(), cur_stream(x)));
  return out;
}

// Fused LSTM Dense head (lstm_head.hip): returns dh = dy . W^T as bf16 [n, 16]; dW / db into grad
// through map (the dense_wgrad slab layout), this step's [sum sq err, #correct] into acc, out =
// acc / div, counter + 1.
at::Tensor lstm_head(const at::Tensor& h, const at::Tensor& W, const at::Tensor& b, const at::Tensor& y,
                     double gscale, const at::Tensor& grad, const at::Tensor& map, const at::Tensor& acc,
                     const c10::optional<at::Tensor>& out, double div0, double div1,
                     const c10::optional<at::Tensor>& counter) {
  check_dev(h, "h", at::kBFloat16);
  check_dev(W, "W", at::kFloat);
  check_dev(b, "b", at::kFloat);
  check_dev(y, "y", at::kFloat);
  check_dev(acc, "acc", at::kFloat);
  TORCH_CHECK(h.dim() == 2 && h.size(1) == 16 && h.stride(1) == 1, "h must be [n, 16] bf16 rows");
  const int64_t n = h.size(0), N = W.size(1);
  TORCH_CHECK(W.is_contiguous() && W.size(0) == 16 && N >= 1 && N <= 32, "W must be [16, N <= 32]");
  TORCH_CHECK(b.is_contiguous() && b.numel() == N, "b must be [N]");
  TORCH_CHECK(y.dim() == 2 && y.size(0) == n && y.size(1) == N && y.stride(1) == 1, "y must be [n, N] rows");
  TORCH_CHECK(acc.numel() >= 2, "acc needs 2 floats");
  const int S = sml::dense_wgrad_slab(16, (int)N);
  const int* mp = grad_map(grad, map, S);
  if (out.has_value()) {
    check_dev(*out, "out", at::kFloat);
    TORCH_CHECK(out->numel() >= 2 && out->is_contiguous(), "out needs 2 contiguous floats");
  }
  if (counter.has_value()) check_dev(*counter, "counter", at::kLong);
  c10::hip::HIPGuard guard(h.device().index());
  auto dh = at::empty({n, 16}, h.options());
  auto part = at::empty({sml::lstm_head_partials(n, (int)N)}, h.options().dtype(at::kFloat));
  SML_CHECK_HIP(sml::lstm_head_launch(h.data_ptr(), h.stride(0), W.data_ptr<float>(), b.data_ptr<float>(),
                                      y.data_ptr<float>(), y.stride(0), dh.data_ptr(), n, (int)N, (float)gscale,
                                      part.data_ptr<float>(), grad.data_ptr<float>(), mp, acc.data_ptr<float>(),
                                      opt_mut(out), (float)div0, (float)div1,
                                      counter.has_value() ? counter->data_ptr<int64_t>() : nullptr, cur_stream(h)));
  return dh;
}

// Two layers' deferred weight-gradient slabs (lstm_fused_bwd defer_sum) reduced into grad in ONE launch.
// With params (+ m, v, iter, rest): Adam fused in (the step's last launch; iter already advanced).
void slab_sum2(const at::Tensor& p0, const at::Tensor& map0, const at::Tensor& p1, const at::Tensor& map1,
               const at::Tensor& grad, const c10::optional<at::Tensor>& params, const c10::optional<at::Tensor>& m,
               const c10::optional<at::Tensor>& v, const c10::optional<at::Tensor>& iter, double lr, double beta1,
               double beta2, double eps, double gscale, const c10::optional<at::Tensor>& rest) {
  for (const auto* t : {&p0, &p1}) {
    check_dev(*t, "partials", at::kFloat);
    TORCH_CHECK(t->dim() == 2 && t->is_contiguous() && t->size(0) <= 4096, "partials must be [G <= 4096, S]");
  }
  const int* m0 = grad_map(grad, map0, (int)p0.size(1));
  const int* m1 = grad_map(grad, map1, (int)p1.size(1));
  sml::SlabAdam ad;
  const bool adam = params.has_value() && params->defined();
  if (adam) {
    TORCH_CHECK(m.has_value() && v.has_value() && iter.has_value() && rest.has_value(), "Adam needs m, v, iter, rest");
    for (const auto* t : {&*params, &*m, &*v}) {
      check_dev(*t, "adam buffer", at::kFloat);
      TORCH_CHECK(t->is_contiguous() && t->numel() == grad.numel(), "Adam buffers must match grad");
    }
    check_dev(*iter, "iter", at::kLong);
    check_dev(*rest, "rest", at::kInt);
    // the kernel scatters through rest unchecked, as through the slab maps: the caller builds it in
    // range (LSTMPredictor._fused_plan asserts it once; no device read here, so a step stays capturable)
    TORCH_CHECK(rest->dim() == 1 && rest->is_contiguous() && rest->numel() <= grad.numel(),
                "rest must be a flat int32 index list");
    ad.params = params->data_ptr<float>();
    ad.m = m->data_ptr<float>();
    ad.v = v->data_ptr<float>();
    ad.iter = iter->data_ptr<int64_t>();
    ad.lr = (float)lr; ad.b1 = (float)beta1; ad.b2 = (float)beta2; ad.eps = (float)eps; ad.gscale = (float)gscale;
    ad.rest = rest->numel() ? rest->data_ptr<int>() : nullptr;
    ad.nrest = (int)rest->numel();
  }
  c10::hip::HIPGuard guard(p0.device().index());
  SML_CHECK_HIP(sml::slab_sum2_launch(p0.data_ptr<float>(), (int)p0.size(0), (int)p0.size(1), m0, p1.data_ptr<float>(),
                                      (int)p1.size(0), (int)p1.size(1), m1, grad.data_ptr<float>(), cur_stream(p0),
                                      adam ? &ad : nullptr));
}

// K3 + K6: (y_pred - y) * gscale -> grad, [sum sq err, #correct rows] += into acc.
void mse_acc(const at::Tensor& yp, const at::Tensor& y, int64_t bcast, double gscale,
             const c10::optional<at::Tensor>& grad, const c10::optional<at::Tensor>& acc, bool reset,
             const c10::optional<at::Tensor>& out, double div0, double div1,
             const c10::optional<at::Tensor>& counter) {
  check_dev(yp, "y_pred", at::kFloat);
  check_dev(y, "y", at::kFloat);
  TORCH_CHECK(yp.is_contiguous() && y.is_contiguous(), "inputs must be contiguous");
  const int64_t F = yp.size(-1);
  const int64_t rows = yp.numel() / F;
  TORCH_CHECK(y.size(-1) == F && bcast >= 1 && y.numel() / F * bcast == rows, "target rows * bcast != prediction rows");
  TORCH_CHECK(sml::mse_acc_supported((int)F), "mse_acc: unsupported feature count ", F);
  if (grad.has_value()) {
    check_dev(*grad, "grad", at::kFloat);
    TORCH_CHECK(grad->is_contiguous() && grad->numel() == yp.numel(), "grad must match y_pred");
  }
  if (acc.has_value()) {
    check_dev(*acc, "acc", at::kFloat);
    TORCH_CHECK(acc->numel() >= 2, "acc needs 2 floats");
  }
  if (out.has_value()) {
    TORCH_CHECK(acc.has_value(), "out needs acc");
    check_dev(*out, "out", at::kFloat);
    TORCH_CHECK(out->numel() >= 2 && out->is_contiguous(), "out needs 2 contiguous floats");
  }
  if (counter.has_value()) {
    TORCH_CHECK(acc.has_value(), "counter needs acc");
    check_dev(*counter, "counter", at::kLong);
  }
  c10::hip::HIPGuard guard(yp.device().index());
  at::Tensor part;
  if (acc.has_value()) part = at::empty({2 * (int64_t)sml::mse_acc_blocks(rows, (int)F)}, yp.options());
  SML_CHECK_HIP(sml::mse_acc_launch(yp.data_ptr<float>(), y.data_ptr<float>(), rows, (int)F, (int)bcast,
                                    (float)gscale, opt_mut(grad), opt_mut(acc),
                                    part.defined() ? part.data_ptr<float>() : nullptr, reset ? 1 : 0, cur_stream(yp),
                                    opt_mut(out), (float)div0, (float)div1,
                                    counter.has_value() ? counter->data_ptr<int64_t>() : nullptr));
}

at::Tensor lane_xor_probe(const at::Tensor& like) {
  TORCH_CHECK(like.is_cuda(), "needs a device tensor for placement");
  c10::hip::HIPGuard guard(like.device().index());
  auto out = at::empty({128}, like.options().dtype(at::kFloat));
  SML_CHECK_HIP(sml::lane_xor_probe_launch(out.data_ptr<float>(), cur_stream(like)));
  return out;
}

// Python face of the pinned staging ring: fill (host memcpy, GIL released),
// submit (hipMemcpyAsync on the ring's copy stream), wait / release against the
// caller's current HIP stream.
// P2P gradient-exchange buffers (runtime/p2p.h)
struct P2PPy {
  std::unique_ptr<sml::P2PExchange> x;
  P2PPy(int device, int rank, int world, int64_t slots) {
    c10::hip::HIPGuard guard(device);
    x = std::make_unique<sml::P2PExchange>(device, rank, world, slots);
  }
  explicit P2PPy(sml::P2PExchange* p) : x(p) {}
  static P2PPy* local(int device, int world, int64_t slots) {
    c10::hip::HIPGuard guard(device);
    return new P2PPy(sml::P2PExchange::local(device, world, slots));
  }
  py::bytes handle() const { return py::bytes(x->handle()); }
  void open(const std::vector<std::string>& h) {
    py::gil_scoped_release rel;
    x->open(h);
  }
};

void p2p_allreduce(at::Tensor& t, P2PPy& ex, double timeout_s) {
  check_dev(t, "x", at::kFloat);
  TORCH_CHECK(t.is_contiguous(), "x must be contiguous");
  TORCH_CHECK(ex.x->ready(), "exchange not opened");
  TORCH_CHECK(t.numel() <= ex.x->slots(), "x larger than the exchange buffers (", ex.x->slots(), " slots)");
  const uint64_t e = ex.x->next_epoch();
  c10::hip::HIPGuard guard(t.device().index());
  SML_CHECK_HIP(sml::p2p_allreduce_launch(t.data_ptr<float>(), t.numel(), ex.x->peers_dev(), ex.x->world(),
                                          ex.x->rank(), ex.x->slots(), sml::p2p_call_tag((int64_t)e),
                                          (int)(e & 1), ex.x->status_dev(), (long long)(timeout_s * 1e8),
                                          cur_stream(t)));
}

struct RingPy {
  std::unique_ptr<sml::PinnedRing> r;
  int device;
  RingPy(int slots, int64_t slot_bytes, int dev) : device(dev) {
    c10::hip::HIPGuard guard(dev);
    r = std::make_unique<sml::PinnedRing>(slots, (size_t)slot_bytes, dev);
  }
  int64_t fill(int slot, py::array arr, int64_t offset) {
    py::buffer_info bi = arr.request();
    if (!(arr.flags() & py::array::c_style)) throw std::invalid_argument("fill: array must be C-contiguous");
    const size_t bytes = (size_t)bi.size * (size_t)bi.itemsize;
    if (offset < 0 || (size_t)offset + bytes > r->slot_bytes())
      throw std::invalid_argument("fill: array does not fit the ring slot at that offset");
    const void* src = bi.ptr;
    {
      py::gil_scoped_release rel;
      char* dst = static_cast<char*>(r->host(slot));   // waits for the slot's previous H2D
      std::memcpy(dst + offset, src, bytes);
    }
    return (int64_t)bytes;
  }
  // Host address of a slot once its previous H2D has landed: native producers (the
  // C++ ingest feed) write decoded rows straight into the page-locked buffer.
  uint64_t host_ptr(int slot) {
    py::gil_scoped_release rel;
    return reinterpret_cast<uint64_t>(r->host(slot));
  }
  void submit(int slot, const at::Tensor& dst, int64_t bytes) {
    TORCH_CHECK(dst.is_cuda() && dst.is_contiguous(), "submit: dst must be a contiguous device tensor");
    TORCH_CHECK(bytes <= (int64_t)(dst.numel() * dst.element_size()), "submit: dst too small");
    c10::hip::HIPGuard guard(device);
    py::gil_scoped_release rel;
    r->submit(slot, dst.data_ptr(), (size_t)bytes);
  }
  void wait(int slot) {
    c10::hip::HIPGuard guard(device);
    r->wait(slot, c10::hip::getCurrentHIPStream(device).stream());
  }
  void release(int slot) {
    c10::hip::HIPGuard guard(device);
    r->release(slot, c10::hip::getCurrentHIPStream(device).stream());
  }
};

// Python face of the persistent scorer: numpy in / numpy out, GIL released while
// the host thread spins on the completion counter.
struct ServePy {
  std::unique_ptr<sml::ServeRing> s;
  ServePy() = default;
  // C ABI for the host-only streaming loop in _io (sml_scorer_api.h)
  SmlScorerApi api{};
  std::string err;
  static int api_infer(void* ctx, const float* rows, int k, float* scores, uint32_t* flags, float* recon,
                       double timeout_s) {
    auto* self = static_cast<ServePy*>(ctx);
    if (self->nkeys() > 0) {   // the C loop carries no car keys
      self->err = "a keyed (LSTM) scorer cannot serve the key-less C scoring loop";
      return 1;
    }
    try {
      self->s->infer(rows, k, scores, flags, recon, timeout_s);
      return 0;
    } catch (const std::exception& e) {
      self->err = e.what();
      return 1;
    }
  }
  static int api_infer_keyed(void* ctx, const float* rows, const uint32_t* keys, int k, float* scores,
                             uint32_t* flags, float* recon, double timeout_s) {
    auto* self = static_cast<ServePy*>(ctx);
    const int64_t nk = self->nkeys();
    if (nk <= 0) {
      self->err = "infer_keyed on a key-less scorer";
      return 1;
    }
    for (int i = 0; i < k; ++i)
      if ((int64_t)keys[i] >= nk) {
        self->err = "key outside [0, nkeys)";
        return 1;
      }
    try {
      self->s->infer(rows, k, scores, flags, recon, timeout_s, keys);
      return 0;
    } catch (const std::exception& e) {
      self->err = e.what();
      return 1;
    }
  }
  static const char* api_error(void* ctx) { return static_cast<ServePy*>(ctx)->err.c_str(); }
  uintptr_t c_api() {
    api.version = SML_SCORER_API_VERSION;
    api.dim = s->D();
    api.ctx = this;
    api.infer = &ServePy::api_infer;
    api.last_error = &ServePy::api_error;
    api.nkeys = nkeys();
    api.infer_keyed = nkeys() > 0 ? &ServePy::api_infer_keyed : nullptr;
    return reinterpret_cast<uintptr_t>(&api);
  }
  ServePy(int device, int nslots, py::array_t<float, py::array::c_style | py::array::forcecast> weights,
          std::vector<int> dims, std::vector<int> acts, py::object scale, py::object shift, double threshold,
          double idle_seconds) {
    if (dims.size() != 3 || acts.size() != 4) throw std::invalid_argument("dims = [D, n1, n2], acts = 4 codes");
    std::vector<float> w(weights.data(), weights.data() + weights.size());
    std::vector<float> sc, sh;
    if (!scale.is_none()) {
      auto a = scale.cast<py::array_t<float, py::array::c_style | py::array::forcecast>>();
      auto b = shift.cast<py::array_t<float, py::array::c_style | py::array::forcecast>>();
      sc.assign(a.data(), a.data() + a.size());
      sh.assign(b.data(), b.data() + b.size());
    }
    c10::hip::HIPGuard guard(device);
    s = std::make_unique<sml::AEServe>(device, nslots, w, dims.data(), acts.data(), sc, sh, (float)threshold,
                                       idle_seconds);
  }
  // optional per-row uint32 keys (the LSTM scorer's car keys), validated against nkeys
  static std::vector<uint32_t> keys_of(const py::object& keys, ssize_t n, int64_t nkeys) {
    std::vector<uint32_t> out;
    if (keys.is_none()) {
      if (nkeys > 0) throw std::invalid_argument("this scorer needs one key per row");
      return out;
    }
    auto k = keys.cast<py::array_t<int64_t, py::array::c_style | py::array::forcecast>>();
    if (k.ndim() != 1 || k.shape(0) != n) throw std::invalid_argument("keys must be [k] integers, one per row");
    out.resize((size_t)n);
    for (ssize_t i = 0; i < n; ++i) {
      const int64_t v = k.data()[i];
      if (v < 0 || (nkeys > 0 && v >= nkeys) || v > 0xffffffffLL) throw std::out_of_range("key outside [0, nkeys)");
      out[(size_t)i] = (uint32_t)v;
    }
    return out;
  }
  virtual int64_t nkeys() const { return 0; }
  virtual ~ServePy() = default;
  py::tuple infer(py::array_t<float, py::array::c_style | py::array::forcecast> rows, bool want_recon,
                  double timeout_s, py::object keys) {
    if (rows.ndim() != 2 || rows.shape(1) != s->D()) throw std::invalid_argument("rows must be [k, D]");
    const int k = (int)rows.shape(0);
    const std::vector<uint32_t> kv = keys_of(keys, k, nkeys());
    py::array_t<float> scores(k);
    py::array_t<uint32_t> flags(k);
    py::array_t<float> recon(want_recon ? std::vector<ssize_t>{k, s->D()} : std::vector<ssize_t>{0});
    const float* src = rows.data();
    float* ps = scores.mutable_data();
    uint32_t* pf = flags.mutable_data();
    float* pr = want_recon ? recon.mutable_data() : nullptr;
    {
      py::gil_scoped_release rel;
      s->infer(src, k, ps, pf, pr, timeout_s, kv.empty() ? nullptr : kv.data());
    }
    return py::make_tuple(scores, flags, recon);
  }
  // -> int64 [n, 2]: host round-trip ns, device processing ns
  py::array_t<int64_t> latency_run(py::array_t<float, py::array::c_style | py::array::forcecast> rows,
                                   int64_t gap_ns, py::object keys) {
    if (rows.ndim() != 2 || rows.shape(1) != s->D()) throw std::invalid_argument("rows must be [n, D]");
    const std::vector<uint32_t> kv = keys_of(keys, rows.shape(0), nkeys());
    std::vector<int64_t> lat, dev;
    {
      py::gil_scoped_release rel;
      lat = s->latency_run(rows.data(), (int)rows.shape(0), gap_ns, &dev, kv.empty() ? nullptr : kv.data());
    }
    // columns: host round trip, device total, device load, device compute (ns)
    py::array_t<int64_t> out(std::vector<ssize_t>{(ssize_t)lat.size(), 4});
    int64_t* o = out.mutable_data();
    for (size_t i = 0; i < lat.size(); ++i) {
      o[4 * i] = lat[i];
      o[4 * i + 1] = ((dev[i] >> 42) & 0x1fffff) * 10;
      o[4 * i + 2] = ((dev[i] >> 21) & 0x1fffff) * 10;
      o[4 * i + 3] = (dev[i] & 0x1fffff) * 10;
    }
    return out;
  }
};

// layers: list of (kind, in, u, act, ret, n, woff, uoff, boff) tuples (sml::LstmServeLayer)
struct LSTMServePy : ServePy {
  int64_t nk = 0;
  LSTMServePy(int device, int nslots, py::array_t<float, py::array::c_style | py::array::forcecast> weights,
              std::vector<std::vector<int>> layers, int D, int T, int nkeys, py::object scale, py::object shift,
              double threshold, double idle_seconds) {
    std::vector<float> w(weights.data(), weights.data() + weights.size());
    std::vector<sml::LstmServeLayer> L;
    for (const auto& t : layers) {
      if (t.size() != 9) throw std::invalid_argument("layer descriptor: (kind, in, u, act, ret, n, woff, uoff, boff)");
      L.push_back(sml::LstmServeLayer{t[0], t[1], t[2], t[3], t[4], t[5], t[6], t[7], t[8]});
    }
    std::vector<float> sc, sh;
    if (!scale.is_none()) {
      auto a = scale.cast<py::array_t<float, py::array::c_style | py::array::forcecast>>();
      auto b = shift.cast<py::array_t<float, py::array::c_style | py::array::forcecast>>();
      sc.assign(a.data(), a.data() + a.size());
      sh.assign(b.data(), b.data() + b.size());
    }
    c10::hip::HIPGuard guard(device);
    s = std::make_unique<sml::LSTMServe>(device, nslots, w, L, D, T, nkeys, sc, sh, (float)threshold, idle_seconds);
    nk = nkeys;
  }
  int64_t nkeys() const override { return nk; }
};

}  // namespace

PYBIND11_MODULE(TORCH_EXTENSION_NAME, m) {
  m.doc() = "streamml gfx950 HIP kernels";
  m.attr("AE_NSLOT") = sml::ae_nslot();
  m.attr("AE_NPARAM") = sml::ae_nparam();
  m.def("ae_train_partials", &ae_train_partials, "fused AE fwd+bwd -> per-workgroup gradient slabs",
        py::arg("x"), py::arg("scale"), py::arg("shift"), py::arg("params"), py::arg("partials"), py::arg("iter"),
        py::arg("dims"), py::arg("acts"), py::arg("l1"), py::arg("want_acc"), py::arg("max_blocks"),
        py::arg("n_rows") = -1, py::arg("cursor") = py::none(), py::arg("xpack") = py::none());
  m.def("pack_tiles_argmax", &pack_tiles_argmax, "tile-packed training ring (rows + ingest-time argmax per tile)",
        py::arg("x"), py::arg("D"), py::arg("scale") = py::none(), py::arg("shift") = py::none(),
        py::arg("index") = py::none(), py::arg("out") = py::none(), py::arg("perm_key") = 0,
        py::arg("perm_n") = 0, py::arg("n_rows") = -1);
  m.def("perm_indices", &perm_indices, "the pack's keyed row bijection of [0, n), materialised", py::arg("like"),
        py::arg("n"), py::arg("key"), py::arg("start") = 0, py::arg("count") = -1);
  m.def("row_argmax_u8", &row_argmax_u8, "ingest-time argmax of each normalised row (uint8)", py::arg("x"),
        py::arg("D"), py::arg("scale") = py::none(), py::arg("shift") = py::none());
  m.def("ae_minibatch_max_batch", &sml::ae_minibatch_max_batch, "largest batch the persistent small-batch trainer takes");
  m.def("ae_train_minibatches", &ae_train_minibatches,
        "persistent small-batch AE trainer: nsteps sequential Keras steps (fwd+bwd+Adam) in one launch",
        py::arg("x"), py::arg("cursor"), py::arg("scale"), py::arg("shift"), py::arg("params"), py::arg("m"),
        py::arg("v"), py::arg("iter"), py::arg("metrics"), py::arg("batch"), py::arg("nsteps"), py::arg("dims"),
        py::arg("acts"), py::arg("l1"), py::arg("lr"), py::arg("beta1"), py::arg("beta2"), py::arg("eps"),
        py::arg("gscale"), py::arg("want_acc"), py::arg("prof") = py::none(), py::arg("lrs") = py::none(),
        py::arg("dp_peers") = 0, py::arg("dp_ranks") = 1, py::arg("dp_rank0") = 0, py::arg("dp_status") = 0,
        py::arg("dp_timeout_ticks") = 0, py::arg("ragged") = py::none(), py::arg("precision") = -1);
  m.def("normalize_filter", &normalize_filter, "K8: normalise + keep rows with label == keep, order-preserving",
        py::arg("x"), py::arg("D"), py::arg("labels"), py::arg("keep"), py::arg("scale"), py::arg("shift"),
        py::arg("want_index") = false);
  m.def("ae_train_blocks_per_cu", &sml::ae_train_blocks_per_cu,
        "workgroups per CU the selected AE train-kernel variant keeps resident (SML_AE_OCC)");
  m.def("ae_train_grid", &sml::ae_train_grid, "grid size the AE train kernel uses", py::arg("n"),
        py::arg("max_blocks"));
  m.def("reduce_adam", &reduce_adam, "slab reduction + optional Adam", py::arg("partials"), py::arg("G"),
        py::arg("S"), py::arg("nparam"), py::arg("grad_out"), py::arg("params"), py::arg("m"), py::arg("v"),
        py::arg("iter"), py::arg("lr"), py::arg("beta1"), py::arg("beta2"), py::arg("eps"), py::arg("gscale"),
        py::arg("metrics"), py::arg("flags"), py::arg("cursor") = py::none(), py::arg("cursor_step") = 0,
        py::arg("cursor_ring") = 0, py::arg("scratch") = py::none(), py::arg("counters") = py::none());
  py::class_<P2PPy>(m, "P2PExchange")
      .def(py::init<int, int, int, int64_t>(), py::arg("device"), py::arg("rank"), py::arg("world"),
           py::arg("slots"))
      .def_static("local", &P2PPy::local, py::arg("device"), py::arg("world"), py::arg("slots"),
                  py::return_value_policy::take_ownership)
      .def("handle", &P2PPy::handle)
      .def("open", &P2PPy::open, py::arg("handles"))
      .def("status", [](const P2PPy& p) { return p.x->status(); })
      .def("reset_status", [](P2PPy& p) { p.x->reset_status(); })
      .def("clear", [](P2PPy& p) { p.x->clear(); })
      .def_property_readonly("ready", [](const P2PPy& p) { return p.x->ready(); })
      .def_property_readonly("rank", [](const P2PPy& p) { return p.x->rank(); })
      .def_property_readonly("world", [](const P2PPy& p) { return p.x->world(); })
      .def_property_readonly("slots", [](const P2PPy& p) { return p.x->slots(); })
      .def_property_readonly("peers_ptr", [](const P2PPy& p) { return reinterpret_cast<uint64_t>(p.x->peers_dev()); })
      .def_property_readonly("status_ptr", [](const P2PPy& p) { return reinterpret_cast<uint64_t>(p.x->status_dev()); });
  m.def("p2p_allreduce", &p2p_allreduce, "in-place sum over the P2P exchange's ranks (one launch, one xGMI hop)",
        py::arg("x"), py::arg("exchange"), py::arg("timeout_s") = 10.0);
  py::class_<StreamRingPy>(m, "StreamRing")
      .def(py::init<int64_t, int64_t, int64_t>(), py::arg("device"), py::arg("rows"), py::arg("features"))
      .def("ring", &StreamRingPy::ring)
      .def("reset", &StreamRingPy::reset)
      .def("train", &StreamRingPy::train, py::arg("cursor"), py::arg("scale"), py::arg("shift"), py::arg("params"),
           py::arg("m"), py::arg("v"), py::arg("iter"), py::arg("metrics"), py::arg("batch"), py::arg("max_steps"),
           py::arg("dims"), py::arg("acts"), py::arg("l1"), py::arg("lr"), py::arg("beta1"), py::arg("beta2"),
           py::arg("eps"), py::arg("gscale"), py::arg("want_acc"), py::arg("timeout_s") = 30.0,
           py::arg("precision") = -1)
      .def("push", &StreamRingPy::push, py::arg("rows"), py::arg("timeout_s") = 30.0)
      .def("finish", &StreamRingPy::finish)
      .def("join", &StreamRingPy::join)
      .def("synchronize", &StreamRingPy::synchronize)
      .def_property_readonly("pushed", &StreamRingPy::pushed)
      .def_property_readonly("consumed", &StreamRingPy::consumed)
      .def_property_readonly("status", &StreamRingPy::status)
      .def_property_readonly("rows", &StreamRingPy::rows);
  py::class_<RingPy>(m, "PinnedRing")
      .def(py::init<int, int64_t, int>(), py::arg("slots"), py::arg("slot_bytes"), py::arg("device"))
      .def("fill", &RingPy::fill, py::arg("slot"), py::arg("array"), py::arg("offset") = 0)
      .def("host_ptr", &RingPy::host_ptr, py::arg("slot"))
      .def("submit", &RingPy::submit, py::arg("slot"), py::arg("dst"), py::arg("bytes"))
      .def("wait", &RingPy::wait, py::arg("slot"))
      .def("release", &RingPy::release, py::arg("slot"))
      .def("reset", [](RingPy& r) {
        py::gil_scoped_release rel;
        r.r->reset();
      })
      .def_property_readonly("slots", [](const RingPy& r) { return r.r->slots(); })
      .def_property_readonly("slot_bytes", [](const RingPy& r) { return (int64_t)r.r->slot_bytes(); })
      .def_property_readonly("bytes_copied", [](const RingPy& r) { return (uint64_t)r.r->bytes_copied(); });
  m.def("lstm_fwd", &lstm_fwd, "fused LSTM recurrence forward (h, c, gates)", py::arg("zx"), py::arg("U"),
        py::arg("h0") = py::none(), py::arg("c0") = py::none(), py::arg("act") = 1);
  m.def("lstm_bwd", &lstm_bwd, "fused LSTM BPTT -> pre-activation gate grads", py::arg("dh"), py::arg("gates"),
        py::arg("cseq"), py::arg("c0"), py::arg("U"), py::arg("act") = 1, py::arg("want_state_grads") = false);
  m.def("softmax_xent", &softmax_xent, "fused softmax + sparse categorical CE fwd/bwd", py::arg("logits"),
        py::arg("labels"), py::arg("gscale"), py::arg("dlogits") = py::none(), py::arg("probs") = py::none(),
        py::arg("acc") = py::none());
  m.def("dense_fwd", &dense_fwd, "K1 tall-skinny dense forward act(X.W + b) on MFMA", py::arg("x"), py::arg("W"),
        py::arg("bias") = py::none(), py::arg("act") = 0, py::arg("out_bf16") = false, py::arg("max_blocks") = 1024,
        py::arg("w_t") = false);
  m.def("dense_wgrad", &dense_wgrad, "K2 weight gradient X^T.dY (+ colsum dY) over rows", py::arg("x"),
        py::arg("dy"), py::arg("shift_T") = 0, py::arg("want_db") = true, py::arg("max_blocks") = 1024,
        py::arg("grad") = py::none(), py::arg("map") = py::none());
  m.def("gemm", &gemm, "general LDS-tiled MFMA GEMM act(a . b + bias), any shape / orientation", py::arg("a"),
        py::arg("b"), py::arg("bias") = py::none(), py::arg("act") = 0, py::arg("out_bf16") = false,
        py::arg("splits") = -1);
  m.def("dense_wgrad_slab", &sml::dense_wgrad_slab, "floats per dense_wgrad slab", py::arg("K"), py::arg("N"));
  m.def("dense_tiles", &sml::dense_tiles, "16-wide tiles a dense dimension is padded to", py::arg("d"));
  m.def("lstm_fused_slab", &sml::lstm_fused_slab, "floats per fused-LSTM weight-gradient slab", py::arg("U"),
        py::arg("IN"));
  m.def("lstm_fused_dx_ld", &sml::lstm_fused_dx_ld, "padded feature stride of the fused-LSTM slab / dx",
        py::arg("IN"));
  m.def("dense_supported", &sml::dense_supported, "whether (K, N) fits the register-resident tile", py::arg("K"),
        py::arg("N"));
  m.def("lstm_fused_fwd2", &lstm_fused_fwd2, "two stacked fused LSTM layers (U 32 -> 16) in one forward launch",
        py::arg("x"), py::arg("W1"), py::arg("U1"), py::arg("b1"), py::arg("W2"), py::arg("U2"), py::arg("b2"),
        py::arg("act1"), py::arg("act2"), py::arg("hfrag") = false);
  m.def("lstm_fused_fwd2_supported", &sml::lstm_fused_fwd2_supported);
  m.def("lstm_fused_frag_supported", &sml::lstm_fused_frag_supported,
        "whether lstm_fused_bwd(frag=True) has an instance for this layer", py::arg("U"), py::arg("IN"),
        py::arg("x_bf16"), py::arg("want_dx"));
  m.def("lstm_split_applies", &sml::lstm_split_applies,
        "whether lstm_fused_bwd runs this layer on the unit-block split kernel (two waves per tile)", py::arg("U"),
        py::arg("IN"), py::arg("dx"), py::arg("x_bf16") = false, py::arg("dh_last_only") = false);
  m.def("lstm_split_grid", &sml::lstm_split_grid, "workgroups (= weight-gradient slabs) of the split backward",
        py::arg("B"));
  m.def("lstm_fused_bwd2", &lstm_fused_bwd2, "two stacked fused LSTM layers' backward (U 32 -> 16) in one launch",
        py::arg("x"), py::arg("h1"), py::arg("c1"), py::arg("h2"), py::arg("c2"), py::arg("dh2"), py::arg("W1"),
        py::arg("U1"), py::arg("b1"), py::arg("W2"), py::arg("U2"), py::arg("b2"), py::arg("act"),
        py::arg("dh2_last_only"), py::arg("grad") = py::none(), py::arg("map1") = py::none(),
        py::arg("map2") = py::none());
  m.def("lstm_fused_bwd2_supported", &sml::lstm_fused_bwd2_supported);
  m.def("lstm_fused_fwd", &lstm_fused_fwd, "fully fused LSTM layer forward (x.W + recurrence in one kernel)",
        py::arg("x"), py::arg("W"), py::arg("U"), py::arg("b"), py::arg("h0") = py::none(),
        py::arg("c0") = py::none(), py::arg("act") = 1);
  m.def("lstm_fused_bwd", &lstm_fused_bwd,
        "fully fused LSTM layer backward (gate recompute + BPTT + dW/dU/db + dX in one kernel)", py::arg("dh"),
        py::arg("c"), py::arg("h"), py::arg("x"), py::arg("h0") = py::none(), py::arg("c0") = py::none(),
        py::arg("W"), py::arg("U"), py::arg("b"), py::arg("act") = 1, py::arg("want_dx") = true,
        py::arg("want_state_grads") = false, py::arg("dh_last_only") = false, py::arg("grad") = py::none(),
        py::arg("map") = py::none(), py::arg("frag") = false, py::arg("defer_sum") = false);
  m.def("slab_sum2", &slab_sum2, "two deferred weight-gradient slab sets reduced into grad in one launch",
        py::arg("p0"), py::arg("map0"), py::arg("p1"), py::arg("map1"), py::arg("grad"), py::arg("params") = py::none(),
        py::arg("m") = py::none(), py::arg("v") = py::none(), py::arg("iter") = py::none(), py::arg("lr") = 0.0,
        py::arg("beta1") = 0.0, py::arg("beta2") = 0.0, py::arg("eps") = 0.0, py::arg("gscale") = 1.0,
        py::arg("rest") = py::none());
  m.def("lstm_ref_train", &lstm_ref_train,
        "persistent trainer: nsteps Keras Adam steps of the reference LSTM stack (look_back 1) in one launch",
        py::arg("flat"), py::arg("m"), py::arg("v"), py::arg("iter"), py::arg("x"), py::arg("y"),
        py::arg("order") = py::none(), py::arg("row0") = 0, py::arg("B") = 1, py::arg("nsteps") = 1,
        py::arg("act") = 1, py::arg("lr") = 1e-3, py::arg("beta1") = 0.9, py::arg("beta2") = 0.999,
        py::arg("eps") = 1e-7);
  m.def("lstm_ref_train_params", &sml::lstm_ref_train_params);
  m.def("mlp_fwd", &mlp_fwd, "dropout(act(x . W + b)) on fp32 MFMA (x float32 or uint8 scaled by 1/255)",
        py::arg("x"), py::arg("W"), py::arg("b") = py::none(), py::arg("relu") = false, py::arg("keep") = 1.0,
        py::arg("seed") = 0, py::arg("step") = 0);
  m.def("mlp_bwd_data", &mlp_bwd_data, "(dz . W^T) * [h > 0] / keep", py::arg("dz"), py::arg("W"), py::arg("h"),
        py::arg("keep") = 1.0);
  m.def("mlp_wgrad", &mlp_wgrad, "[x ; 1]^T . dy -> out [K + 1, N] (dW then db)", py::arg("x"), py::arg("dy"),
        py::arg("out"));
  m.def("mlp_dropout_mask", &mlp_dropout_mask, "the in-kernel dropout multipliers (0 or 1/keep)", py::arg("like"),
        py::arg("M"), py::arg("N"), py::arg("keep"), py::arg("seed"), py::arg("step"));
  m.def("lstm_fused_supported", &sml::lstm_fused_supported, "whether (U, IN) has a fused LSTM kernel", py::arg("U"),
        py::arg("IN"));
  py::class_<ServePy>(m, "AEServe", "persistent per-event autoencoder scorer over host-mapped rings")
      .def("debug_state", [](ServePy& p, uint64_t seq) { return p.s->debug_state(seq); }, py::arg("seq"))
      .def(py::init<int, int, py::array_t<float, py::array::c_style | py::array::forcecast>, std::vector<int>,
                    std::vector<int>, py::object, py::object, double, double>(),
           py::arg("device"), py::arg("nslots"), py::arg("weights"), py::arg("dims"), py::arg("acts"),
           py::arg("scale") = py::none(), py::arg("shift") = py::none(), py::arg("threshold") = 5.0,
           py::arg("idle_seconds") = 2.0)
      .def("infer", &ServePy::infer, py::arg("rows"), py::arg("want_recon") = false, py::arg("timeout_s") = 10.0,
           py::arg("keys") = py::none())
      .def("latency_run", &ServePy::latency_run, py::arg("rows"), py::arg("gap_ns") = 0, py::arg("keys") = py::none())
      .def("stop", [](ServePy& p) { p.s->stop(); })
      .def("c_api", &ServePy::c_api, "address of the SmlScorerApi table (for _io.ScoreLoop)")
      .def_property_readonly("launches", [](ServePy& p) { return p.s->launches(); });
  py::class_<LSTMServePy, ServePy>(m, "LSTMServe",
                                   "persistent per-event LSTM forecaster: per-key windows on the device")
      .def(py::init<int, int, py::array_t<float, py::array::c_style | py::array::forcecast>,
                    std::vector<std::vector<int>>, int, int, int, py::object, py::object, double, double>(),
           py::arg("device"), py::arg("nslots"), py::arg("weights"), py::arg("layers"), py::arg("D"), py::arg("T"),
           py::arg("nkeys"), py::arg("scale") = py::none(), py::arg("shift") = py::none(),
           py::arg("threshold") = 5.0, py::arg("idle_seconds") = 2.0)
      .def("reset_keys", [](LSTMServePy& p) {
        p.s->stop();   // the kernel must not run while its state is cleared
        static_cast<sml::LSTMServe*>(p.s.get())->reset_keys();
      })
      .def_property_readonly("nkeys", [](LSTMServePy& p) { return p.nk; });
  m.def("lstm_head", &lstm_head, "fused LSTM Dense head: forward, MSE + accuracy, dW / db, dh (one pass + fold)",
        py::arg("h"), py::arg("W"), py::arg("b"), py::arg("y"), py::arg("gscale"), py::arg("grad"), py::arg("map"),
        py::arg("acc"), py::arg("out") = py::none(), py::arg("div0") = 1.0, py::arg("div1") = 1.0,
        py::arg("counter") = py::none());
  m.def("mse_acc", &mse_acc, "fused MSE fwd/bwd + categorical accuracy (K3 + K6)", py::arg("y_pred"), py::arg("y"),
        py::arg("bcast") = 1, py::arg("gscale") = 1.0, py::arg("grad") = py::none(), py::arg("acc") = py::none(),
        py::arg("reset") = false, py::arg("out") = py::none(), py::arg("div0") = 1.0, py::arg("div1") = 1.0,
        py::arg("counter") = py::none());
  m.def("mse_acc_supported", &sml::mse_acc_supported, "feature counts with a fused MSE kernel", py::arg("F"));
  m.def("lane_xor_probe", &lane_xor_probe, "self-test of the permlane lane-exchange helpers", py::arg("like"));
  m.def("ae_forward", &ae_forward, "fused AE inference: reconstruction + per-row MSE score", py::arg("x"),
        py::arg("scale"), py::arg("shift"), py::arg("params"), py::arg("recon"), py::arg("score"), py::arg("flag"),
        py::arg("threshold"), py::arg("dims"), py::arg("acts"), py::arg("max_blocks"), py::arg("metrics") = py::none());
}
