#include "stream_ring.h"


#include <algorithm>
#include <chrono>
#include <cstring>
#include <stdexcept>
#include <string>

namespace sml {
namespace {

void ck(hipError_t e, const char* what) {
  if (e != hipSuccess) throw std::runtime_error(std::string("StreamRing: ") + what + ": " + hipGetErrorString(e));
}

inline void cpu_relax() {
#if defined(__x86_64__)
  __builtin_ia32_pause();
#endif
}

}  // namespace

StreamRing::StreamRing(int device, int64_t rows, int features) : device_(device), rows_(rows), features_(features) {
  if (rows < 1 || features < 1 || features > 31) throw std::invalid_argument("StreamRing: rows >= 1, 1..31 features");
  ck(hipSetDevice(device), "hipSetDevice");
  ck(hipExtMallocWithFlags(reinterpret_cast<void**>(&ring_), (size_t)rows * features * sizeof(float),
                           hipDeviceMallocUncached),
     "uncached ring allocation");
  ck(hipHostMalloc(reinterpret_cast<void**>(&host_), 4 * sizeof(int64_t), hipHostMallocMapped | hipHostMallocCoherent),
     "counters");
  ck(hipHostGetDevicePointer(reinterpret_cast<void**>(&dev_), host_, 0), "counters device pointer");
  ck(hipStreamCreateWithFlags(&copy_, hipStreamNonBlocking), "copy stream");
  ck(hipEventCreateWithFlags(&produced_, hipEventDisableTiming), "event");
  ck(hipEventCreateWithFlags(&copied_, hipEventDisableTiming), "event");
  reset();
}

StreamRing::~StreamRing() {
  if (copy_) (void)hipStreamSynchronize(copy_);
  if (produced_) (void)hipEventDestroy(produced_);
  if (copied_) (void)hipEventDestroy(copied_);
  if (copy_) (void)hipStreamDestroy(copy_);
  if (ring_) (void)hipFree(ring_);
  if (host_) (void)hipHostFree(host_);
}

void StreamRing::reset() {
  ck(hipStreamSynchronize(copy_), "sync");
  __atomic_store_n(&host_[0], (int64_t)0, __ATOMIC_RELEASE);
  __atomic_store_n(&host_[1], (int64_t)-1, __ATOMIC_RELEASE);
  __atomic_store_n(&host_[2], (int64_t)0, __ATOMIC_RELEASE);
  __atomic_store_n(&host_[3], (int64_t)0, __ATOMIC_RELEASE);
  pushed_ = 0;
  finished_ = false;
}

int64_t StreamRing::consumed() const { return __atomic_load_n(&host_[2], __ATOMIC_ACQUIRE); }
int StreamRing::status() const { return (int)__atomic_load_n(&host_[3], __ATOMIC_ACQUIRE); }

MBStream StreamRing::counters(double timeout_s) const {
  MBStream s;
  s.avail = dev_;
  s.total = dev_ + 1;
  s.consumed = dev_ + 2;
  s.status = reinterpret_cast<int*>(dev_ + 3);
  s.timeout_ticks = (long long)(timeout_s * 100e6);   // s_memrealtime: 100 MHz
  return s;
}

void StreamRing::push(const float* src, int64_t n, int64_t ld, hipStream_t producer, double timeout_s) {
  if (finished_) throw std::logic_error("StreamRing: push after finish");
  if (n <= 0) return;
  if (ld < features_) throw std::invalid_argument("StreamRing: row stride smaller than the features");
  ck(hipSetDevice(device_), "hipSetDevice");
  ck(hipEventRecord(produced_, producer), "record");
  ck(hipStreamWaitEvent(copy_, produced_, 0), "wait");
  const auto t0 = std::chrono::steady_clock::now();
  int64_t done = 0;
  while (done < n) {
    // back-pressure: at most `rows_` rows between the kernel's consumed mark and pushed
    int64_t room = rows_ - (pushed_ - consumed());
    uint32_t spins = 0;
    while (room <= 0) {
      cpu_relax();
      if ((++spins & 0x3ff) == 0) {
        if (status()) throw std::runtime_error("StreamRing: the training kernel timed out waiting for rows");
        const double el = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        if (el > timeout_s) throw std::runtime_error("StreamRing: timed out waiting for ring space");
      }
      room = rows_ - (pushed_ - consumed());
    }
    const int64_t pos = pushed_ % rows_;
    const int64_t k = std::min({n - done, room, rows_ - pos});   // never across the wrap
    float* dst = ring_ + pos * features_;
    const float* s = src + done * ld;
    if (ld == features_)
      ck(hipMemcpyAsync(dst, s, (size_t)k * features_ * sizeof(float), hipMemcpyDeviceToDevice, copy_), "copy");
    else
      ck(hipMemcpy2DAsync(dst, (size_t)features_ * sizeof(float), s, (size_t)ld * sizeof(float),
                          (size_t)features_ * sizeof(float), (size_t)k, hipMemcpyDeviceToDevice, copy_),
         "strided copy");
    pushed_ += k;
    done += k;
    // publish after the copy, in copy-stream order: the kernel never reads a row early
    ck(hipStreamWriteValue64(copy_, dev_ + 0, (uint64_t)pushed_, 0), "publish");
  }
  ck(hipEventRecord(copied_, copy_), "record");
  ck(hipStreamWaitEvent(producer, copied_, 0), "producer waits for the copy");
}

void StreamRing::finish() {
  if (finished_) return;
  ck(hipSetDevice(device_), "hipSetDevice");
  ck(hipStreamWriteValue64(copy_, dev_ + 1, (uint64_t)pushed_, 0), "publish total");
  finished_ = true;
}

}  // namespace sml
