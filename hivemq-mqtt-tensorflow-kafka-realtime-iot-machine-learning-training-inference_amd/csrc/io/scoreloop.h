// Low-latency streaming scorer: Kafka -> Avro decode -> GPU score -> result records ->
// Kafka, all in one C++ thread (`serve --low-latency`).
//
// The reference's inference job (AUTOENCODER-TensorFlow-IO-Kafka/cardata-v3.py:235-279)
// is a bounded Keras predict over a KafkaDataset with a per-batch output callback:
// events wait for a whole batch, every output is formatted in Python
// (np.array2string) and produced through KafkaOutputSequence.  Here each fetch is
// scored as soon as it arrives:
//
//   * long-poll fetch (fetch.min.bytes = 1, fetch.max.wait.ms): the broker answers the
//     moment a record is appended, no polling interval;
//   * records are walked in place (RecordSetCursor) and decoded straight into a row
//     buffer (feed::Feed's compiled Avro plan);
//   * the rows go to the persistent GPU scorer through the SmlScorerApi table
//     (host-mapped request ring, no launch, no hipMemcpy -- runtime/serve.h);
//   * result records ({car, partition, offset, score, anomaly[, reconstruction]}, byte
//     for byte what cli/serve.py writes with json.dumps / np.array2string) are
//     formatted here (format.h) and produced as ONE record batch per fetch (acks = 1);
//   * offsets are committed to the consumer group after the produce (at-least-once).
//
// With `record_latency`, the steady-clock time at which each event's result became
// visible (produce acknowledged) is kept per input offset, for the append -> visible
// latency bench (bench/bench_infer.py).
#pragma once
#include <atomic>
#include <cstdint>
#include <memory>
#include <string>
#include <unordered_map>
#include <utility>
#include <vector>

#include "avro.h"
#include "feed.h"
#include "jsonrow.h"
#include "kafka.h"
#include "sml_scorer_api.h"

namespace sml {
namespace serve {

struct LoopConfig {
  std::string topic, result_topic, group;   // group "" = no offset commits
  std::vector<int> partitions;              // owned source partitions
  std::vector<int64_t> starts;              // start offset per owned partition
  std::vector<int> result_partitions;       // result partition per owned partition
  std::vector<int> feature_fields;          // schema field of each model feature
  bool framing = true;
  bool emit_recon = false;                  // add "reconstruction": np.array2string(recon)
  int max_batch = 4096;                     // rows per scorer call
  int32_t max_bytes = 1 << 20;
  int32_t max_wait_ms = 100;                // long-poll bound
  int offset_reset = 0;                     // auto.offset.reset: 0 earliest, 1 latest, 2 none (raise)
  double commit_interval_s = 0.0;           // 0: commit after every produced batch
  bool record_latency = false;
  // JSON source records (the MQTT bridge's `sensor-data`, KSQL SENSOR_DATA_S) instead of
  // Avro: (key, model column) per feature, decoded by jsonrow::Plan; json_stamp names a
  // numeric field copied into the latency records (the device simulator's send time)
  std::vector<std::pair<std::string, int>> json_columns;
  std::string json_stamp;
  // key-hash share per owned partition (kafka/assign.py "keys"): a record is scored only if
  // the top 32 bits of fmix64(FNV-1a 64) of its key lie in [lo, hi); empty = every key of every
  // owned partition.  Replicas sharing a partition split its cars this way, each car on
  // exactly one replica, in order.
  std::vector<std::pair<uint64_t, uint64_t>> hash_ranges;
};

struct LoopStats {
  uint64_t events = 0, anomalies = 0, skipped = 0, batches = 0, fetches = 0, empty_fetches = 0, commits = 0;
  uint64_t keys = 0;   // keyed (LSTM) scorer: distinct record keys given a device slot
  uint64_t foreign = 0;        // records of a shared partition whose key another replica owns
  uint64_t reset_skipped = 0;  // records jumped over after OFFSET_OUT_OF_RANGE (retention)
  uint64_t keys_dropped = 0;   // keyed scorer: records not scored (key table full, or a null key)
  double fetch_s = 0, decode_s = 0, score_s = 0, format_s = 0, produce_s = 0, commit_s = 0, wall_s = 0;
};

class ScoreLoop {
 public:
  ScoreLoop(std::string bootstrap, kafka::ClientConfig ccfg, std::vector<avro::Field> fields, LoopConfig cfg,
            const SmlScorerApi* api);
  // Blocking: runs until stop(), `max_events` scored events (0 = unbounded) or
  // `idle_timeout_s` without records (< 0 = unbounded).
  LoopStats run(int64_t max_events, double idle_timeout_s);
  void stop() { stop_ = true; }
  std::vector<int64_t> positions() const;   // next offset per owned partition
  // kLatCols int64 per scored event when record_latency: partition, offset, steady-clock ns
  // of the produce ack (result visible), of the fetch response, of the scores, of the
  // formatted records, and the record's json_stamp field (0 without one)
  static constexpr int kLatCols = 7;
  const std::vector<int64_t>& latency_records() const { return lat_; }
  // bytes of latency records written so far: readable while the loop runs, so a soak can
  // tell the measurement's own memory from the scorer's
  size_t latency_bytes() const { return lat_bytes_.load(std::memory_order_relaxed); }

 private:
  std::string bootstrap_;
  kafka::ClientConfig ccfg_;
  LoopConfig cfg_;
  const SmlScorerApi* api_;
  feed::Feed decoder_;   // only its compiled decode plan is used (never started)
  std::unique_ptr<jsonrow::Plan> json_;   // JSON source records
  // keyed scorers: record key -> device slot, first come first served (the device keeps
  // each slot's window); records of keys past the scorer's nkeys slots, and null-keyed
  // records, are skipped and counted (LoopStats::keys_dropped), never scored into a shared slot
  std::unordered_map<std::string, uint32_t> key_ids_;
  std::vector<int64_t> pos_;
  std::vector<int64_t> lat_;
  std::atomic<size_t> lat_bytes_{0};
  size_t rot_ = 0;   // first partition of the next multi-partition fetch (rotated, KIP-74)
  std::atomic<bool> stop_{false};
};

// Producer side of the latency bench: append records (value i = values[offs[i],
// offs[i+1]), key i) one produce request per record, paced at `qps`; returns the
// steady-clock ns just before each request was sent.
std::vector<int64_t> paced_produce(const std::string& bootstrap, kafka::ClientConfig ccfg, const std::string& topic,
                                   int partition, const std::string& values, const std::vector<int64_t>& offs,
                                   const std::vector<std::string>& keys, double qps);

int64_t steady_ns();
uint32_t key_share_hash(const uint8_t* key, int64_t len);   // fmix64(FNV-1a 64) >> 32 (kafka/assign.py key_hash)

}  // namespace serve
}  // namespace sml
