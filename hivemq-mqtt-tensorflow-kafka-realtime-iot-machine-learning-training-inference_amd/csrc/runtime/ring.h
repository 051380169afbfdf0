// Pinned-host staging ring -> device, with copy/compute overlap.
//
// The reference's input pipeline is tf.data on CPU (KafkaDataset -> decode ->
// normalize -> batch, cardata-v3.py:197-218) feeding a CPU model.  Here decoded
// micro-batches are written into page-locked (hipHostMalloc) slots and copied
// to device buffers with hipMemcpyAsync on a dedicated copy stream; the compute
// stream waits on the slot's copy event (hipStreamWaitEvent), and a slot is only
// rewritten after the consumer recorded its release event, so decode (host
// threads), H2D (copy engine) and training kernels (compute queue) overlap.
#pragma once
#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdint>
#include <mutex>
#include <stdexcept>
#include <vector>

namespace sml {

class PinnedRing {
 public:
  PinnedRing(int slots, size_t slot_bytes, int device);
  ~PinnedRing();
  PinnedRing(const PinnedRing&) = delete;
  PinnedRing& operator=(const PinnedRing&) = delete;

  int slots() const { return (int)host_.size(); }
  size_t slot_bytes() const { return slot_bytes_; }
  // Block until `slot` may be refilled (its last H2D finished) and return its host buffer.
  void* host(int slot);
  // Copy `bytes` from the host slot to `dst` (device) on the copy stream once the
  // consumer has released the previous use of that destination.
  void submit(int slot, void* dst, size_t bytes);
  // Make `stream` wait until slot's copy has landed.
  void wait(int slot, hipStream_t stream);
  // Consumer is done with the device buffer of `slot` once `stream` reaches here.
  void release(int slot, hipStream_t stream);
  // Back to all-IDLE for a new owner (a pooled ring, data/loader.py): copies submitted but
  // never consumed are waited for on the host; pending releases stay pending (the next
  // submit of that slot still waits for the old consumer's release event).
  void reset();
  //
  // Ordering contract, asserted on every call (every H2D copy records an
  // event that the compute stream waits on), per slot:
  //     IDLE --submit--> COPYING --wait--> CONSUMING --release--> IDLE
  // submit on a slot the consumer still holds (the copy would race its kernels),
  // release of a slot whose copy the consumer never waited for (its kernels may
  // have read stale data), or wait on a slot with no copy in flight throw
  // std::logic_error instead of silently corrupting a batch.
  //
  // Thread safety: one producer thread may host()/submit() slots while one consumer
  // thread wait()s / release()s OTHER slots (per-slot state is byte-sized and guarded
  // by a mutex; the blocking copy-event wait in host() runs outside it).  The caller
  // still orders release(slot) before the next submit(slot) (DeviceLoader: a
  // free-slot semaphore), so the copy stream never waits on an unrecorded event.
  hipStream_t copy_stream() const { return copy_; }
  uint64_t bytes_copied() const { return bytes_; }

 private:
  int device_;
  size_t slot_bytes_;
  std::vector<void*> host_;
  std::vector<hipEvent_t> copied_, released_;
  std::vector<uint8_t> pending_copy_, pending_release_;   // not vector<bool>: slots change from two threads
  enum class SlotState : uint8_t { kIdle, kCopying, kConsuming };
  std::vector<SlotState> state_;
  hipStream_t copy_ = nullptr;
  uint64_t bytes_ = 0;
  std::mutex mu_;
  void check(int slot) const {
    if (slot < 0 || slot >= (int)host_.size()) throw std::out_of_range("PinnedRing: bad slot");
  }
};

}  // namespace sml
