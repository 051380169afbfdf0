// Host side of the persistent per-event scorer (kernels/ae_serve.hip).
//
// Request slots, result slots and the control block are fine-grained pinned host
// memory mapped into the GPU's address space, so an event travels host -> GPU ->
// host with no hipMemcpy and no kernel launch: submit() writes the rows and
// publishes the new head with a release store; the resident wave picks them up,
// and wait() spins on the completion counter.  If the kernel exited (idle timeout
// or a race with its exit), wait() relaunches it; it resumes at `done`.
#pragma once
#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdint>
#include <vector>

#include "sml_ops.h"

namespace sml {

class AEServe {
 public:
  AEServe(int device, int nslots, const std::vector<float>& weights, const int dims[3], const int acts[4],
          const std::vector<float>& scale, const std::vector<float>& shift, float threshold, double idle_seconds);
  ~AEServe();
  AEServe(const AEServe&) = delete;
  AEServe& operator=(const AEServe&) = delete;

  // Publish k rows of D floats; returns the sequence number of the first one.
  uint64_t submit(const float* rows, int k);
  // Block until every event < seq_end is done (throws after timeout_s).
  void wait(uint64_t seq_end, double timeout_s);
  const ServeResult& result(uint64_t seq) const { return res_[seq % (uint64_t)nslots_]; }
  // submit + wait + copy scores / flags (/ recon) for k rows.
  void infer(const float* rows, int k, float* scores, uint32_t* flags, float* recon, double timeout_s);
  // Per-event latency (ns) of n events submitted one at a time, spaced by gap_ns.
  // Also fills dev_ns[i] (device pick-up -> stores issued, if non-null) and counts relaunches.
  std::vector<int64_t> latency_run(const float* rows, int n, int64_t gap_ns, std::vector<int64_t>* dev_ns = nullptr);
  void stop();
  int D() const { return D_; }
  uint64_t launches() const { return launches_; }

 private:
  void launch();
  int device_, nslots_, D_;
  int dims_[3], acts_[4];
  float threshold_;
  double idle_s_;
  ServeCtl* ctl_ = nullptr;
  float* req_ = nullptr;
  ServeResult* res_ = nullptr;
  ServeCtl* ctl_d_ = nullptr;
  float* req_d_ = nullptr;
  ServeResult* res_d_ = nullptr;
  float* wts_d_ = nullptr;
  float* scale_d_ = nullptr;
  float* shift_d_ = nullptr;
  hipStream_t stream_ = nullptr;
  uint64_t head_ = 0;
  uint64_t launches_ = 0;
};

}  // namespace sml
