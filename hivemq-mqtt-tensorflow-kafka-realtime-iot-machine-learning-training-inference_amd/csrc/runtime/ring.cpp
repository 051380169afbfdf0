// Pinned-host staging ring (see ring.h).
#include "ring.h"

#include <string>

namespace sml {

#define RING_CHECK(expr)                                                                         \
  do {                                                                                           \
    hipError_t _e = (expr);                                                                      \
    if (_e != hipSuccess) throw std::runtime_error(std::string("PinnedRing: ") + #expr + ": " + \
                                                   hipGetErrorString(_e));                       \
  } while (0)

PinnedRing::PinnedRing(int slots, size_t slot_bytes, int device) : device_(device), slot_bytes_(slot_bytes) {
  if (slots < 1 || slot_bytes == 0) throw std::invalid_argument("PinnedRing: need >= 1 slot of > 0 bytes");
  RING_CHECK(hipSetDevice(device_));
  RING_CHECK(hipStreamCreateWithFlags(&copy_, hipStreamNonBlocking));
  host_.assign((size_t)slots, nullptr);
  copied_.assign((size_t)slots, nullptr);
  released_.assign((size_t)slots, nullptr);
  pending_copy_.assign((size_t)slots, 0);
  pending_release_.assign((size_t)slots, 0);
  state_.assign((size_t)slots, SlotState::kIdle);
  for (int i = 0; i < slots; ++i) {
    RING_CHECK(hipHostMalloc(&host_[(size_t)i], slot_bytes_, hipHostMallocDefault));
    RING_CHECK(hipEventCreateWithFlags(&copied_[(size_t)i], hipEventDisableTiming));
    RING_CHECK(hipEventCreateWithFlags(&released_[(size_t)i], hipEventDisableTiming));
  }
}

PinnedRing::~PinnedRing() {
  if (copy_) hipStreamSynchronize(copy_);
  for (size_t i = 0; i < host_.size(); ++i) {
    if (host_[i]) hipHostFree(host_[i]);
    if (copied_[i]) hipEventDestroy(copied_[i]);
    if (released_[i]) hipEventDestroy(released_[i]);
  }
  if (copy_) hipStreamDestroy(copy_);
}

void* PinnedRing::host(int slot) {
  check(slot);
  bool pending;
  {
    std::lock_guard<std::mutex> g(mu_);
    pending = pending_copy_[(size_t)slot] != 0;
  }
  if (pending) {  // host buffer still being read by the DMA engine (wait outside the lock)
    RING_CHECK(hipEventSynchronize(copied_[(size_t)slot]));
    std::lock_guard<std::mutex> g(mu_);
    pending_copy_[(size_t)slot] = 0;
  }
  return host_[(size_t)slot];
}

void PinnedRing::submit(int slot, void* dst, size_t bytes) {
  check(slot);
  if (bytes > slot_bytes_) throw std::invalid_argument("PinnedRing: copy larger than a slot");
  std::lock_guard<std::mutex> g(mu_);
  if (state_[(size_t)slot] != SlotState::kIdle)
    throw std::logic_error("PinnedRing: submit on slot " + std::to_string(slot) +
                           (state_[(size_t)slot] == SlotState::kCopying ? " whose previous copy was never consumed"
                                                                        : " still held by the consumer (release it first)"));
  RING_CHECK(hipSetDevice(device_));
  if (pending_release_[(size_t)slot]) {  // device buffer still in use by the consumer
    RING_CHECK(hipStreamWaitEvent(copy_, released_[(size_t)slot], 0));
    pending_release_[(size_t)slot] = 0;
  }
  RING_CHECK(hipMemcpyAsync(dst, host_[(size_t)slot], bytes, hipMemcpyHostToDevice, copy_));
  RING_CHECK(hipEventRecord(copied_[(size_t)slot], copy_));
  pending_copy_[(size_t)slot] = 1;
  state_[(size_t)slot] = SlotState::kCopying;
  bytes_ += bytes;
}

void PinnedRing::wait(int slot, hipStream_t stream) {
  check(slot);
  std::lock_guard<std::mutex> g(mu_);
  if (state_[(size_t)slot] == SlotState::kIdle)
    throw std::logic_error("PinnedRing: wait on slot " + std::to_string(slot) + " with no copy submitted");
  RING_CHECK(hipStreamWaitEvent(stream, copied_[(size_t)slot], 0));
  state_[(size_t)slot] = SlotState::kConsuming;
}

void PinnedRing::release(int slot, hipStream_t stream) {
  check(slot);
  std::lock_guard<std::mutex> g(mu_);
  if (state_[(size_t)slot] != SlotState::kConsuming)
    throw std::logic_error("PinnedRing: release of slot " + std::to_string(slot) +
                           " whose copy the consumer never waited for");
  RING_CHECK(hipEventRecord(released_[(size_t)slot], stream));
  pending_release_[(size_t)slot] = 1;
  state_[(size_t)slot] = SlotState::kIdle;
}

void PinnedRing::reset() {
  for (size_t i = 0; i < host_.size(); ++i) {
    bool pending;
    {
      std::lock_guard<std::mutex> g(mu_);
      pending = pending_copy_[i] != 0;
    }
    if (pending) RING_CHECK(hipEventSynchronize(copied_[i]));
    std::lock_guard<std::mutex> g(mu_);
    pending_copy_[i] = 0;
    state_[i] = SlotState::kIdle;
  }
}

}  // namespace sml
