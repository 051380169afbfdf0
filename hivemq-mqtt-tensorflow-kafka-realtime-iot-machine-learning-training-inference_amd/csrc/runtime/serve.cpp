#include "serve.h"

#include <chrono>
#include <cstring>
#include <stdexcept>
#include <string>
#include <thread>
#include <algorithm>

namespace sml {
namespace {

void ck(hipError_t e, const char* what) {
  if (e != hipSuccess) throw std::runtime_error(std::string("AEServe: ") + what + ": " + hipGetErrorString(e));
}

inline uint64_t load_acq(const uint64_t* p) { return __atomic_load_n(p, __ATOMIC_ACQUIRE); }
inline void store_rel(uint64_t* p, uint64_t v) { __atomic_store_n(p, v, __ATOMIC_RELEASE); }

inline void cpu_relax() {
#if defined(__x86_64__)
  __builtin_ia32_pause();
#endif
}

}  // namespace

AEServe::AEServe(int device, int nslots, const std::vector<float>& weights, const int dims[3], const int acts[4],
                 const std::vector<float>& scale, const std::vector<float>& shift, float threshold,
                 double idle_seconds)
    : device_(device), nslots_(nslots), D_(dims[0]), threshold_(threshold), idle_s_(idle_seconds) {
  if (nslots < 64) throw std::invalid_argument("AEServe: nslots must be >= 64");
  for (int i = 0; i < 3; ++i) dims_[i] = dims[i];
  for (int i = 0; i < 4; ++i) acts_[i] = acts[i];
  const int D = dims[0], n1 = dims[1], n2 = dims[2];
  if (D < 1 || D > 32 || n1 < 1 || n1 > 16 || n2 < 1 || n2 > 16)
    throw std::invalid_argument("AEServe: dims exceed the serving kernel (D <= 32, hidden <= 16)");
  const size_t nw = (size_t)D * n1 + n1 + (size_t)n1 * n2 + n2 + (size_t)n2 * n2 + n2 + (size_t)n2 * D + D;
  if (weights.size() != nw) throw std::invalid_argument("AEServe: weight vector has the wrong length");
  ck(hipSetDevice(device), "hipSetDevice");
  const unsigned fl = hipHostMallocMapped | hipHostMallocCoherent;
  ck(hipHostMalloc((void**)&ctl_, sizeof(ServeCtl), fl), "hipHostMalloc ctl");
  ck(hipHostMalloc((void**)&req_, sizeof(float) * 32 * (size_t)nslots, fl), "hipHostMalloc req");
  ck(hipHostMalloc((void**)&res_, sizeof(ServeResult) * (size_t)nslots, fl), "hipHostMalloc res");
  std::memset(ctl_, 0, sizeof(ServeCtl));
  std::memset(req_, 0, sizeof(float) * 32 * (size_t)nslots);
  std::memset(res_, 0, sizeof(ServeResult) * (size_t)nslots);
  ck(hipHostGetDevicePointer((void**)&ctl_d_, ctl_, 0), "device ptr ctl");
  ck(hipHostGetDevicePointer((void**)&req_d_, req_, 0), "device ptr req");
  ck(hipHostGetDevicePointer((void**)&res_d_, res_, 0), "device ptr res");
  ck(hipMalloc((void**)&wts_d_, nw * sizeof(float)), "hipMalloc weights");
  ck(hipMemcpy(wts_d_, weights.data(), nw * sizeof(float), hipMemcpyHostToDevice), "copy weights");
  if (!scale.empty()) {
    if ((int)scale.size() != D || (int)shift.size() != D) throw std::invalid_argument("AEServe: scale/shift size");
    ck(hipMalloc((void**)&scale_d_, D * sizeof(float)), "hipMalloc scale");
    ck(hipMalloc((void**)&shift_d_, D * sizeof(float)), "hipMalloc shift");
    ck(hipMemcpy(scale_d_, scale.data(), D * sizeof(float), hipMemcpyHostToDevice), "copy scale");
    ck(hipMemcpy(shift_d_, shift.data(), D * sizeof(float), hipMemcpyHostToDevice), "copy shift");
  }
  ck(hipStreamCreateWithFlags(&stream_, hipStreamNonBlocking), "stream");
  launch();
}

AEServe::~AEServe() {
  try {
    stop();
  } catch (...) {
  }
  if (stream_) (void)hipStreamDestroy(stream_);
  if (wts_d_) (void)hipFree(wts_d_);
  if (scale_d_) (void)hipFree(scale_d_);
  if (shift_d_) (void)hipFree(shift_d_);
  if (ctl_) (void)hipHostFree(ctl_);
  if (req_) (void)hipHostFree(req_);
  if (res_) (void)hipHostFree(res_);
}

void AEServe::launch() {
  ck(hipSetDevice(device_), "hipSetDevice");
  __atomic_store_n(&ctl_->stop, 0u, __ATOMIC_RELEASE);
  ck(ae_serve_launch(ctl_d_, req_d_, res_d_, nslots_, wts_d_, scale_d_, shift_d_, dims_, acts_, threshold_, idle_s_,
                     stream_),
     "launch");
  ++launches_;
}

uint64_t AEServe::submit(const float* rows, int k) {
  if (k <= 0) return head_;
  if (k > nslots_) throw std::invalid_argument("AEServe: more rows than slots");
  // back-pressure: never overwrite a slot whose event is not done
  while (head_ + (uint64_t)k - load_acq(&ctl_->done) > (uint64_t)nslots_) wait(head_ + k - nslots_, 10.0);
  const uint64_t first = head_;
  for (int i = 0; i < k; ++i) {
    float* dst = req_ + (size_t)((first + i) % (uint64_t)nslots_) * 32;
    std::memcpy(dst, rows + (size_t)i * D_, sizeof(float) * D_);
  }
  head_ += k;
  store_rel(&ctl_->head, head_);
  return first;
}

void AEServe::wait(uint64_t seq_end, double timeout_s) {
  const auto t0 = std::chrono::steady_clock::now();
  uint32_t spins = 0;
  while (load_acq(&ctl_->done) < seq_end) {
    cpu_relax();
    if ((++spins & 0x3ff) == 0) {
      // the kernel exits after idle_seconds without work, or may have raced its
      // exit with our publish: relaunch it once it has really finished
      if (hipStreamQuery(stream_) == hipSuccess && load_acq(&ctl_->done) < seq_end) launch();
      const double el = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
      if (el > timeout_s) throw std::runtime_error("AEServe: timed out waiting for results");
    }
  }
}

void AEServe::infer(const float* rows, int k, float* scores, uint32_t* flags, float* recon, double timeout_s) {
  int off = 0;
  while (off < k) {
    const int n = std::min(k - off, nslots_);
    const uint64_t first = submit(rows + (size_t)off * D_, n);
    wait(first + n, timeout_s);
    for (int i = 0; i < n; ++i) {
      const ServeResult& r = result(first + i);
      if (scores) scores[off + i] = r.score;
      if (flags) flags[off + i] = r.flag;
      if (recon) std::memcpy(recon + (size_t)(off + i) * D_, r.recon, sizeof(float) * D_);
    }
    off += n;
  }
}

std::vector<int64_t> AEServe::latency_run(const float* rows, int n, int64_t gap_ns, std::vector<int64_t>* dev_ns) {
  std::vector<int64_t> lat(n);
  if (dev_ns) dev_ns->assign(n, 0);
  auto next = std::chrono::steady_clock::now();
  for (int i = 0; i < n; ++i) {
    while (std::chrono::steady_clock::now() < next) cpu_relax();
    const auto t0 = std::chrono::steady_clock::now();
    const uint64_t s = submit(rows + (size_t)i * D_, 1);
    wait(s + 1, 10.0);
    const auto t1 = std::chrono::steady_clock::now();
    lat[i] = std::chrono::duration_cast<std::chrono::nanoseconds>(t1 - t0).count();
    if (dev_ns) {
      const ServeResult& r = result(s);
      // 100 MHz ticks -> ns, packed: [total | load | compute] in three 21-bit fields (ns / 10)
      const int64_t tot = (int64_t)(r.t_done - r.t_seen), ld = (int64_t)(r.t_loaded - r.t_seen),
                    cp = (int64_t)(r.t_comp - r.t_loaded);
      (*dev_ns)[i] = (std::min<int64_t>(tot, 0x1fffff) << 42) | (std::min<int64_t>(ld, 0x1fffff) << 21) |
                     std::min<int64_t>(cp, 0x1fffff);
    }
    next = t0 + std::chrono::nanoseconds(gap_ns);
  }
  return lat;
}

void AEServe::stop() {
  if (!ctl_) return;
  __atomic_store_n(&ctl_->stop, 1u, __ATOMIC_RELEASE);
  if (stream_) (void)hipStreamSynchronize(stream_);
}

}  // namespace sml
