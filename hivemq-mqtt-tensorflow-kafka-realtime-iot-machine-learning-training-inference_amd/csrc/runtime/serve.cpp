#include "serve.h"
#include "queues.h"

#include <chrono>
#include <cstring>
#include <stdexcept>
#include <string>
#include <thread>
#include <algorithm>

namespace sml {
namespace {

void ck(hipError_t e, const char* what) {
  if (e != hipSuccess) throw std::runtime_error(std::string("serve: ") + what + ": " + hipGetErrorString(e));
}

inline uint64_t load_acq(const uint64_t* p) { return __atomic_load_n(p, __ATOMIC_ACQUIRE); }
inline void store_rel(uint64_t* p, uint64_t v) { __atomic_store_n(p, v, __ATOMIC_RELEASE); }

inline void cpu_relax() {
#if defined(__x86_64__)
  __builtin_ia32_pause();
#endif
}

}  // namespace

ServeRing::ServeRing(int device, int nslots, int D, double idle_seconds, int max_D)
    : device_(device), nslots_(nslots), D_(D), idle_s_(idle_seconds) {
  if (nslots < 64) throw std::invalid_argument("serve: nslots must be >= 64");
  if (max_D > 32) max_D = 32;   // a request slot holds 32 words
  if (D < 1 || D > max_D)
    throw std::invalid_argument(std::string("serve: rows must have 1..") + std::to_string(max_D) + " features");
  ck(hipSetDevice(device), "hipSetDevice");
  const unsigned fl = hipHostMallocMapped | hipHostMallocCoherent;
  ck(hipHostMalloc((void**)&ctl_, sizeof(ServeCtl), fl), "hipHostMalloc ctl");
  ck(hipHostMalloc((void**)&req_, sizeof(ServeReq) * (size_t)nslots, fl), "hipHostMalloc req");
  ck(hipHostMalloc((void**)&res_, sizeof(ServeResult) * (size_t)nslots, fl), "hipHostMalloc res");
  std::memset(ctl_, 0, sizeof(ServeCtl));
  std::memset(req_, 0, sizeof(ServeReq) * (size_t)nslots);   // tag 0 = empty (tags start at 1)
  std::memset(res_, 0, sizeof(ServeResult) * (size_t)nslots);
  ck(hipHostGetDevicePointer((void**)&ctl_d_, ctl_, 0), "device ptr ctl");
  ck(hipHostGetDevicePointer((void**)&req_d_, req_, 0), "device ptr req");
  ck(hipHostGetDevicePointer((void**)&res_d_, res_, 0), "device ptr res");
  ck(create_persistent_stream(&stream_), "stream");
}

ServeRing::~ServeRing() {
  if (stream_) (void)hipStreamDestroy(stream_);
  if (ctl_) (void)hipHostFree(ctl_);
  if (req_) (void)hipHostFree(req_);
  if (res_) (void)hipHostFree(res_);
}

void ServeRing::launch() {
  ck(hipSetDevice(device_), "hipSetDevice");
  __atomic_store_n(&ctl_->stop, 0u, __ATOMIC_RELEASE);
  ck(launch_kernel(), "launch");
  ++launches_;
}

AEServe::AEServe(int device, int nslots, const std::vector<float>& weights, const int dims[3], const int acts[4],
                 const std::vector<float>& scale, const std::vector<float>& shift, float threshold,
                 double idle_seconds)
    : ServeRing(device, nslots, dims[0], idle_seconds, 32), threshold_(threshold) {   // no key word: all 32
  name_ = "AEServe";
  for (int i = 0; i < 3; ++i) dims_[i] = dims[i];
  for (int i = 0; i < 4; ++i) acts_[i] = acts[i];
  const int D = dims[0], n1 = dims[1], n2 = dims[2];
  if (D < 1 || D > 32 || n1 < 1 || n1 > 16 || n2 < 1 || n2 > 16)
    throw std::invalid_argument("AEServe: dims exceed the serving kernel (D <= 32, hidden <= 16)");
  const size_t nw = (size_t)D * n1 + n1 + (size_t)n1 * n2 + n2 + (size_t)n2 * n2 + n2 + (size_t)n2 * D + D;
  if (weights.size() != nw) throw std::invalid_argument("AEServe: weight vector has the wrong length");
  ck(hipMalloc((void**)&wts_d_, nw * sizeof(float)), "hipMalloc weights");
  ck(hipMemcpy(wts_d_, weights.data(), nw * sizeof(float), hipMemcpyHostToDevice), "copy weights");
  if (!scale.empty()) {
    if ((int)scale.size() != D || (int)shift.size() != D) throw std::invalid_argument("AEServe: scale/shift size");
    ck(hipMalloc((void**)&scale_d_, D * sizeof(float)), "hipMalloc scale");
    ck(hipMalloc((void**)&shift_d_, D * sizeof(float)), "hipMalloc shift");
    ck(hipMemcpy(scale_d_, scale.data(), D * sizeof(float), hipMemcpyHostToDevice), "copy scale");
    ck(hipMemcpy(shift_d_, shift.data(), D * sizeof(float), hipMemcpyHostToDevice), "copy shift");
  }
  launch();
}

AEServe::~AEServe() {
  try {
    stop();
  } catch (...) {
  }
  if (wts_d_) (void)hipFree(wts_d_);
  if (scale_d_) (void)hipFree(scale_d_);
  if (shift_d_) (void)hipFree(shift_d_);
}

hipError_t AEServe::launch_kernel() {
  return ae_serve_launch(ctl_d_, req_d_, res_d_, nslots_, wts_d_, scale_d_, shift_d_, dims_, acts_, threshold_,
                         idle_s_, stream_);
}

LSTMServe::LSTMServe(int device, int nslots, const std::vector<float>& weights,
                     const std::vector<LstmServeLayer>& layers, int D, int T, int nkeys,
                     const std::vector<float>& scale, const std::vector<float>& shift, float threshold,
                     double idle_seconds)
    : ServeRing(device, nslots, D, idle_seconds, 31) {   // request word 31 carries the car key
  name_ = "LSTMServe";
  if (layers.empty() || layers.size() > (size_t)LS_MAXLAYERS) throw std::invalid_argument("LSTMServe: 1..8 layers");
  if (T < 1 || T > 64) throw std::invalid_argument("LSTMServe: look_back must be 1..64");
  if (nkeys < 1) throw std::invalid_argument("LSTMServe: nkeys must be >= 1");
  for (const auto& L : layers) {   // every offset inside the weight vector
    const int64_t G = L.kind == LS_LSTM ? 4 * (int64_t)L.u : L.u;
    if (L.kind == LS_REPEAT) continue;
    if (L.woff < 0 || (int64_t)L.woff + (int64_t)L.in * G > (int64_t)weights.size() || L.boff < 0 ||
        (int64_t)L.boff + G > (int64_t)weights.size() ||
        (L.kind == LS_LSTM && (L.uoff < 0 || (int64_t)L.uoff + (int64_t)L.u * G > (int64_t)weights.size())))
      throw std::invalid_argument("LSTMServe: a layer's weights lie outside the weight vector");
  }
  if (lstm_serve_lds_bytes((int)weights.size()) > 160 * 1024)
    throw std::invalid_argument("LSTMServe: the weights do not fit the scorer's LDS");
  ck(hipMalloc((void**)&wts_d_, weights.size() * sizeof(float)), "hipMalloc weights");
  ck(hipMemcpy(wts_d_, weights.data(), weights.size() * sizeof(float), hipMemcpyHostToDevice), "copy weights");
  if (!scale.empty()) {
    if ((int)scale.size() != D || (int)shift.size() != D) throw std::invalid_argument("LSTMServe: scale/shift size");
    ck(hipMalloc((void**)&scale_d_, D * sizeof(float)), "hipMalloc scale");
    ck(hipMalloc((void**)&shift_d_, D * sizeof(float)), "hipMalloc shift");
    ck(hipMemcpy(scale_d_, scale.data(), D * sizeof(float), hipMemcpyHostToDevice), "copy scale");
    ck(hipMemcpy(shift_d_, shift.data(), D * sizeof(float), hipMemcpyHostToDevice), "copy shift");
  }
  LstmServeArgs& a = args_;
  a.ctl = ctl_d_;
  a.req = req_d_;
  a.res = res_d_;
  a.nslots = nslots_;
  a.wts = wts_d_;
  a.nw = (int)weights.size();
  a.nl = (int)layers.size();
  for (size_t i = 0; i < layers.size(); ++i) a.L[i] = layers[i];
  a.scale = scale_d_;
  a.shift = shift_d_;
  a.D = D;
  a.T = T;
  a.nkeys = nkeys;
  a.threshold = threshold;
  a.idle_ticks = (uint64_t)(idle_seconds * 100e6);   // s_memrealtime runs at 100 MHz
  ck(hipMalloc((void**)&a.hist, (size_t)nkeys * T * D * sizeof(float)), "hipMalloc windows");
  ck(hipMalloc((void**)&a.hcount, (size_t)nkeys * sizeof(int)), "hipMalloc counts");
  ck(hipMalloc((void**)&a.lastpred, (size_t)nkeys * D * sizeof(float)), "hipMalloc forecasts");
  reset_keys();   // zeroes the key state and launches the resident kernel
}

void LSTMServe::reset_keys() {
  // the resident kernel reads and writes the key state: stop it first (flag + drain the
  // stream), so the memsets never queue behind a kernel that only leaves at its idle timeout
  stop();
  ck(hipMemsetAsync(args_.hcount, 0, (size_t)args_.nkeys * sizeof(int), stream_), "memset counts");
  ck(hipMemsetAsync(args_.lastpred, 0, (size_t)args_.nkeys * args_.D * sizeof(float), stream_), "memset forecasts");
  ck(hipStreamSynchronize(stream_), "sync");
  launch();
}

LSTMServe::~LSTMServe() {
  try {
    stop();
  } catch (...) {
  }
  if (args_.hist) (void)hipFree(args_.hist);
  if (args_.hcount) (void)hipFree(args_.hcount);
  if (args_.lastpred) (void)hipFree(args_.lastpred);
  if (wts_d_) (void)hipFree(wts_d_);
  if (scale_d_) (void)hipFree(scale_d_);
  if (shift_d_) (void)hipFree(shift_d_);
}

hipError_t LSTMServe::launch_kernel() { return lstm_serve_launch(args_, stream_); }

uint64_t ServeRing::submit(const float* rows, int k, const uint32_t* keys) {
  if (k <= 0) return head_;
  if (k > nslots_) throw std::invalid_argument("serve: more rows than slots");
  // back-pressure: never overwrite a slot whose event is not done
  if (head_ + (uint64_t)k > (uint64_t)nslots_) wait_done(head_ + (uint64_t)k - (uint64_t)nslots_, 10.0);
  const uint64_t first = head_;
  for (int i = 0; i < k; ++i) {
    const uint64_t ev = first + (uint64_t)i;
    ServeReq& dst = req_[ev % (uint64_t)nslots_];
    const uint64_t tag = (uint64_t)(uint32_t)(ev + 1) << 32;
    const float* row = rows + (size_t)i * D_;
    for (int j = 0; j < D_; ++j) {   // 8-byte atomic stores: a word is never seen half-written
      uint32_t bits;
      std::memcpy(&bits, &row[j], 4);
      __atomic_store_n(&dst.w[j], tag | bits, __ATOMIC_RELAXED);
    }
    if (keys) __atomic_store_n(&dst.w[31], tag | keys[i], __ATOMIC_RELAXED);
  }
  head_ += k;
  store_rel(&ctl_->head, head_);   // after the rows: the backlog path trusts rows below head
  return first;
}

bool ServeRing::complete(uint64_t seq) const {
  const ServeResult& r = res_[seq % (uint64_t)nslots_];
  const uint32_t tag = (uint32_t)(seq + 1);
  for (int i = kServeScore; i < kServeWords; ++i)
    if ((uint32_t)(__atomic_load_n(&r.w[i], __ATOMIC_RELAXED) >> 32) != tag) return false;
  for (int i = 0; i < D_; ++i)
    if ((uint32_t)(__atomic_load_n(&r.w[i], __ATOMIC_RELAXED) >> 32) != tag) return false;
  __atomic_thread_fence(__ATOMIC_ACQUIRE);
  return true;
}

uint32_t ServeRing::word(uint64_t seq, int i) const {
  return (uint32_t)__atomic_load_n(&res_[seq % (uint64_t)nslots_].w[i], __ATOMIC_RELAXED);
}

float ServeRing::score(uint64_t seq) const {
  const uint32_t b = word(seq, kServeScore);
  float f;
  std::memcpy(&f, &b, 4);
  return f;
}

void ServeRing::wait_done(uint64_t n, double timeout_s) {
  const auto t0 = std::chrono::steady_clock::now();
  uint32_t spins = 0;
  while (load_acq(&ctl_->done) < n) {
    cpu_relax();
    if ((++spins & 0x3ff) == 0) {
      if (hipStreamQuery(stream_) == hipSuccess && load_acq(&ctl_->done) < n) launch();
      const double el = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
      if (el > timeout_s) throw std::runtime_error(std::string(name_) + ": timed out waiting for free slots");
    }
  }
}

void ServeRing::wait(uint64_t seq_end, double timeout_s) {
  const auto t0 = std::chrono::steady_clock::now();
  uint32_t spins = 0;
  uint64_t ev = complete_ < seq_end ? std::max<uint64_t>(complete_, seq_end > (uint64_t)nslots_ ?
                                                                       seq_end - (uint64_t)nslots_ : 0)
                                    : seq_end;
  while (ev < seq_end) {
    if (complete(ev)) {
      ++ev;
      continue;
    }
    cpu_relax();
    if ((++spins & 0x3ff) == 0) {
      // the kernel exits after idle_seconds without work, or may have raced its
      // exit with our publish: relaunch it once it has really finished (it resumes
      // at `done`, written after each event's result stores were issued)
      if (hipStreamQuery(stream_) == hipSuccess && !complete(ev)) launch();
      const double el = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
      if (el > timeout_s) throw std::runtime_error(std::string(name_) + ": timed out waiting for results");
    }
  }
  complete_ = std::max(complete_, seq_end);
}

void ServeRing::infer(const float* rows, int k, float* scores, uint32_t* flags, float* recon, double timeout_s,
                      const uint32_t* keys) {
  int off = 0;
  while (off < k) {
    const int n = std::min(k - off, nslots_);
    const uint64_t first = submit(rows + (size_t)off * D_, n, keys ? keys + off : nullptr);
    wait(first + n, timeout_s);
    for (int i = 0; i < n; ++i) {
      const uint64_t ev = first + (uint64_t)i;
      if (scores) scores[off + i] = score(ev);
      if (flags) flags[off + i] = word(ev, kServeFlag);
      if (recon)
        for (int j = 0; j < D_; ++j) {
          const uint32_t b = word(ev, j);
          std::memcpy(&recon[(size_t)(off + i) * D_ + j], &b, 4);
        }
    }
    off += n;
  }
}

std::vector<int64_t> ServeRing::latency_run(const float* rows, int n, int64_t gap_ns, std::vector<int64_t>* dev_ns,
                                            const uint32_t* keys) {
  std::vector<int64_t> lat(n);
  if (dev_ns) dev_ns->assign(n, 0);
  auto next = std::chrono::steady_clock::now();
  for (int i = 0; i < n; ++i) {
    while (std::chrono::steady_clock::now() < next) cpu_relax();
    const auto t0 = std::chrono::steady_clock::now();
    const uint64_t s = submit(rows + (size_t)i * D_, 1, keys ? keys + i : nullptr);
    wait(s + 1, 10.0);
    const auto t1 = std::chrono::steady_clock::now();
    lat[i] = std::chrono::duration_cast<std::chrono::nanoseconds>(t1 - t0).count();
    if (dev_ns) {
      // 100 MHz ticks -> ns, packed: [total | load | compute] in three 21-bit fields (ns / 10)
      const int64_t tot = word(s, kServeTDone), ld = word(s, kServeTLoad),
                    cp = (int64_t)word(s, kServeTComp) - (int64_t)word(s, kServeTLoad);
      (*dev_ns)[i] = (std::min<int64_t>(tot, 0x1fffff) << 42) | (std::min<int64_t>(ld, 0x1fffff) << 21) |
                     std::min<int64_t>(cp, 0x1fffff);
    }
    next = t0 + std::chrono::nanoseconds(gap_ns);
  }
  return lat;
}

std::vector<uint64_t> ServeRing::debug_state(uint64_t seq) const {
  std::vector<uint64_t> v = {__atomic_load_n(&ctl_->head, __ATOMIC_ACQUIRE), __atomic_load_n(&ctl_->done, __ATOMIC_ACQUIRE),
                             __atomic_load_n(&ctl_->stop, __ATOMIC_ACQUIRE), __atomic_load_n(&ctl_->alive, __ATOMIC_ACQUIRE),
                             launches_, hipStreamQuery(stream_) == hipSuccess ? 1u : 0u};
  const ServeResult& r = res_[seq % (uint64_t)nslots_];
  for (size_t i = 0; i < sizeof(ServeResult) / 8; ++i) v.push_back(__atomic_load_n(&r.w[i], __ATOMIC_ACQUIRE));
  const ServeReq& q = req_[seq % (uint64_t)nslots_];
  for (int i = 0; i < 32; ++i) v.push_back(__atomic_load_n(&q.w[i], __ATOMIC_ACQUIRE));
  return v;
}

void ServeRing::stop() {
  if (!ctl_) return;
  __atomic_store_n(&ctl_->stop, 1u, __ATOMIC_RELEASE);
  if (stream_) (void)hipStreamSynchronize(stream_);
}

}  // namespace sml
