// Host side of the persistent per-event scorer (kernels/ae_serve.hip).
//
// Request slots, result slots and the control block are fine-grained pinned host
// memory mapped into the GPU's address space, so an event travels host -> GPU ->
// host with no hipMemcpy and no kernel launch.  Slots are LL-framed (sml_ops.h):
// submit() writes each row as tagged 8-byte words and then publishes the new head;
// the resident wave polls the next slot's words directly; wait() polls the tagged
// result words in host memory.  `done` is only a back-pressure / restart hint.  If
// the kernel exited (idle timeout or a race with its exit), wait() relaunches it; it
// resumes at `done`.
#pragma once
#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdint>
#include <vector>

#include "sml_ops.h"

namespace sml {

// The host-mapped request / result rings and the relaunch-on-demand protocol shared by the
// persistent scorers; a subclass supplies the kernel launch.
class ServeRing {
 public:
  // max_D: widest row the subclass's kernel takes (<= 32 request words; 31 when word 31
  // carries a key)
  ServeRing(int device, int nslots, int D, double idle_seconds, int max_D);
  virtual ~ServeRing();
  ServeRing(const ServeRing&) = delete;
  ServeRing& operator=(const ServeRing&) = delete;

  // Publish k rows of D floats (keys: optional per-row uint32 in request word 31);
  // returns the sequence number of the first one.
  uint64_t submit(const float* rows, int k, const uint32_t* keys = nullptr);
  // Block until the results of the events in [seq_end - nslots, seq_end) have landed
  // (throws after timeout_s).
  void wait(uint64_t seq_end, double timeout_s);
  const ServeResult& result(uint64_t seq) const { return res_[seq % (uint64_t)nslots_]; }
  // all tagged words of event seq's result have landed
  bool complete(uint64_t seq) const;
  // payload of result word i of event seq (call after complete())
  uint32_t word(uint64_t seq, int i) const;
  float score(uint64_t seq) const;
  // submit + wait + copy scores / flags (/ recon) for k rows.
  void infer(const float* rows, int k, float* scores, uint32_t* flags, float* recon, double timeout_s,
             const uint32_t* keys = nullptr);
  // Per-event latency (ns) of n events submitted one at a time, spaced by gap_ns.
  // Also fills dev_ns[i] (device pick-up -> stores issued, if non-null) and counts relaunches.
  std::vector<int64_t> latency_run(const float* rows, int n, int64_t gap_ns, std::vector<int64_t>* dev_ns = nullptr,
                                   const uint32_t* keys = nullptr);
  void stop();
  int D() const { return D_; }
  // debugging: {head, done, stop, alive, launches, stream idle (1) / busy (0)} then the raw
  // result words and request words of event `seq`'s slot
  std::vector<uint64_t> debug_state(uint64_t seq) const;
  uint64_t launches() const { return launches_; }

 protected:
  virtual hipError_t launch_kernel() = 0;
  void launch();
  // back-pressure: block until the device consumed every event < n (its request slot is free)
  void wait_done(uint64_t n, double timeout_s);
  int device_, nslots_, D_;
  double idle_s_;
  ServeCtl* ctl_ = nullptr;
  ServeReq* req_ = nullptr;
  ServeResult* res_ = nullptr;
  ServeCtl* ctl_d_ = nullptr;
  ServeReq* req_d_ = nullptr;
  ServeResult* res_d_ = nullptr;
  hipStream_t stream_ = nullptr;
  uint64_t head_ = 0;
  uint64_t launches_ = 0;
  uint64_t complete_ = 0;   // events known complete (prefix)
  const char* name_ = "serve";
};

// Dense autoencoder scorer (ae_serve.hip): reconstruction + MSE anomaly score per event.
class AEServe : public ServeRing {
 public:
  AEServe(int device, int nslots, const std::vector<float>& weights, const int dims[3], const int acts[4],
          const std::vector<float>& scale, const std::vector<float>& shift, float threshold, double idle_seconds);
  ~AEServe() override;

 protected:
  hipError_t launch_kernel() override;

 private:
  int dims_[3], acts_[4];
  float threshold_;
  float* wts_d_ = nullptr;
  float* scale_d_ = nullptr;
  float* shift_d_ = nullptr;
};

// LSTM forecaster (lstm_serve.hip): per car key, the last T events stay on the device; each
// event is scored against the key's previous forecast and a new forecast is emitted.
class LSTMServe : public ServeRing {
 public:
  // layers: LstmServeLayer descriptors (offsets into weights); keys in [0, nkeys)
  LSTMServe(int device, int nslots, const std::vector<float>& weights, const std::vector<LstmServeLayer>& layers,
            int D, int T, int nkeys, const std::vector<float>& scale, const std::vector<float>& shift, float threshold,
            double idle_seconds);
  ~LSTMServe() override;
  int nkeys() const { return args_.nkeys; }
  // forget every key's window and forecast: stops the resident kernel, zeroes the key state
  // on the device, relaunches (returns without waiting for the kernel's idle timeout)
  void reset_keys();

 protected:
  hipError_t launch_kernel() override;

 private:
  LstmServeArgs args_{};
  float* wts_d_ = nullptr;
  float* scale_d_ = nullptr;
  float* shift_d_ = nullptr;
};

}  // namespace sml
