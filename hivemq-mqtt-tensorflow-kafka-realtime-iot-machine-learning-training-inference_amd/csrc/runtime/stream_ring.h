// Device-side row ring for a streaming epoch trained by ONE persistent kernel launch.
//
// The reference's streaming job re-batches a Kafka stream on the CPU and runs a graph
// step per batch (cardata-v3.py:44-75, 212-222).  The persistent Keras-step kernel
// (ae_minibatch.hip) can instead stay resident for the whole epoch and take its batches
// from a device ring while the stream is still arriving:
//
//   producer stream (slabs landing from the pinned H2D ring / K8)
//        | event
//   copy stream:  D2D copy of the chunk into the ring (split at the wrap)
//                 hipStreamWriteValue64(avail)   <- ordered after the copy
//   train stream: the kernel polls `avail` (host-mapped, once per batch it does not
//                 already know is present), trains, reports `consumed`
//   host:         push() blocks while the ring is full (consumed + capacity)
//
// No launch per chunk, no carry copy between chunks (batches straddle chunk boundaries
// in the ring), no host synchronisation per batch.  The ring memory is uncached device
// memory: rows are written by another engine while the kernel runs, so a cached line
// from the previous lap must never shadow them.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

#include "sml_ops.h"

namespace sml {

class StreamRing {
 public:
  StreamRing(int device, int64_t rows, int features);
  ~StreamRing();
  StreamRing(const StreamRing&) = delete;
  StreamRing& operator=(const StreamRing&) = delete;

  // New epoch: counters back to zero (the kernel of the previous epoch must have finished).
  void reset();
  // Append n rows (device memory, row stride ld floats) once `producer` has produced them;
  // the producer stream is made to wait for the copy, so it may reuse `src` afterwards.
  // Blocks while the ring holds `rows` unconsumed rows; throws after timeout_s.
  void push(const float* src, int64_t n, int64_t ld, hipStream_t producer, double timeout_s);
  // The stream ended: publish the total (after every copy) so the kernel finishes.
  void finish();
  int64_t pushed() const { return pushed_; }
  int64_t consumed() const;
  int status() const;
  float* ring() const { return ring_; }
  int64_t rows() const { return rows_; }
  int features() const { return features_; }
  MBStream counters(double timeout_s) const;

 private:
  int device_;
  int64_t rows_;
  int features_;
  float* ring_ = nullptr;
  hipStream_t copy_ = nullptr;
  hipEvent_t produced_ = nullptr, copied_ = nullptr;
  int64_t* host_ = nullptr;   // [0] avail, [1] total, [2] consumed, [3] status (int)
  int64_t* dev_ = nullptr;    // device view of host_
  int64_t pushed_ = 0;
  bool finished_ = false;
};

}  // namespace sml
