// Peer-to-peer exchange buffers for small-message data parallelism over xGMI.
//
// The reference trains one model in one process (no tf.distribute); the
// BASELINE asks for DP on 8 MI355X.  Its gradient bucket is tiny (571 floats for the
// 18-14-7-7-18 autoencoder), and at Keras granularity (one Adam step per 32 or 100 rows,
// ~2-4 us of compute) an RCCL all-reduce per step (~10-30 us, plus a launch) would cost
// several times the step.  So the gradient exchange is a direct one-hop push over the
// fully connected xGMI links: every rank owns ONE receive buffer
//     [2 parities][world source ranks][slots] 8-byte granules {tag, float value}
// allocated uncached (fine-grained: remote writes are seen by local polls without any
// cache maintenance) and exported with a HIP IPC handle.  Each rank maps its peers'
// buffers; a kernel publishes its values into slot [parity][my rank] of EVERY peer's
// buffer with system-scope 8-byte stores (one posted xGMI write per granule, all 7 links
// busy at once), then polls its own buffer until every peer's granules carry the current
// tag, and sums in rank order -- the same order on every rank, so replicas stay
// bit-identical.  A granule is its own flag (tag and value in one 8-byte store), so no
// fence or separate flag write is needed; the parity double-buffer lets a rank publish
// step s+1 while a slower peer still reads step s.
//
// `local` mode allocates every rank's buffer in one process (ranks = workgroups of one
// launch, or the unit tests), with no IPC.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <string>
#include <vector>

namespace sml {

class P2PExchange {
 public:
  // One rank of a multi-process group (call handle(), exchange, then open()).
  P2PExchange(int device, int rank, int world, int64_t slots);
  // Every rank's buffer in this process ("in-launch" ranks).
  static P2PExchange* local(int device, int world, int64_t slots);
  ~P2PExchange();
  P2PExchange(const P2PExchange&) = delete;
  P2PExchange& operator=(const P2PExchange&) = delete;

  std::string handle() const;                             // hipIpcMemHandle_t bytes
  void open(const std::vector<std::string>& handles);     // peers' handles, index = rank
  bool ready() const { return peers_dev_ != nullptr; }

  int rank() const { return rank_; }
  int world() const { return world_; }
  int64_t slots() const { return slots_; }
  uint64_t** peers_dev() const { return peers_dev_; }     // device array [world] of receive buffers
  int* status_dev() const { return status_; }              // device int: 1 = a poll timed out
  int status() const;
  void reset_status();
  void clear();   // re-zero this process's receive buffer(s) (caller brackets it with barriers)
  uint64_t next_epoch() { return ++epoch_; }               // host-side call counter (allreduce tags)

  // bytes of one receive buffer: granules + a validation word
  size_t buffer_bytes() const { return (size_t)2 * world_ * slots_ * 8 + 64; }

 private:
  P2PExchange() = default;
  int device_ = 0, rank_ = 0, world_ = 1;
  int64_t slots_ = 0;
  std::vector<void*> own_;        // buffers this process allocated (1, or world in local mode)
  std::vector<void*> opened_;     // IPC-mapped peer buffers (to close)
  std::vector<void*> peers_;      // receive buffer of every rank, as seen from this device
  uint64_t** peers_dev_ = nullptr;
  int* status_ = nullptr;
  uint64_t epoch_ = 0;
  void alloc_buffer(int rank_id);
  void publish_peers();
};

// Host-callable small all-reduce (sum) over the exchange: x[n] (fp32, device) is summed
// across ranks in rank order, in place.  One launch per call, n <= slots.
hipError_t p2p_allreduce_launch(float* x, int64_t n, uint64_t** peers, int world, int rank, int64_t slots,
                                uint32_t tag, int parity, int* status, long long timeout_ticks, hipStream_t stream);

}  // namespace sml
