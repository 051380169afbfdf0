// Kafka wire protocol: client + in-process broker.
//
// The reference consumes Kafka through tensorflow-io's KafkaDataset (C++ over
// librdkafka, `KafkaDataset(["topic:0:offset"], servers, group, eof, config_global)`,
// AUTOENCODER-TensorFlow-IO-Kafka/cardata-v3.py:44-47) and produces results with
// KafkaOutputSequence (cardata-v3.py:238-252).  librdkafka is not available here,
// so this is a from-scratch implementation of the protocol subset those paths use:
//
//   ApiVersions v0, Metadata v1, ListOffsets v1, Fetch v4, Produce v3,
//   SaslHandshake v1 + SaslAuthenticate v0 (SASL/PLAIN, as in the reference's
//   `security.protocol=sasl_plaintext, sasl.mechanisms=PLAIN`),
//   FindCoordinator v1, OffsetCommit v2, OffsetFetch v1 (consumer-group offsets),
//   record batches v2 (magic 2, CRC-32C, uncompressed).
//
// `Broker` is an in-process partitioned append-only log that serves the same
// protocol on 127.0.0.1 so the client is always exercised over real sockets.  It
// has fault-injection knobs (failed / delayed fetches) for the recovery tests
// (SURVEY.md 5.3).
#pragma once
#include <atomic>
#include <condition_variable>
#include <cstdint>
#include <deque>
#include <map>
#include <memory>
#include <mutex>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

namespace sml {
namespace kafka {

struct Error : std::runtime_error {
  int code;
  Error(const std::string& m, int c = -1) : std::runtime_error(m), code(c) {}
};

uint32_t crc32c(const uint8_t* p, size_t n, uint32_t crc = 0);

struct Record {
  int64_t offset = 0;
  int64_t timestamp = 0;
  std::string key;
  std::string value;
  bool key_null = true;
};

// Flat batch of fetched records: values back to back (value i spans
// [value_offsets[i], value_offsets[i+1])), plus per-record metadata.
struct FetchResult {
  std::string values;
  std::vector<int64_t> value_offsets{0};
  std::vector<int64_t> offsets;
  std::vector<int64_t> timestamps;
  std::vector<std::string> keys;
  int64_t high_watermark = -1;
  int error_code = 0;
  size_t size() const { return offsets.size(); }
};

// record batch v2 codec
std::string encode_record_batch(int64_t base_offset, const std::vector<Record>& recs);
std::string encode_record_batch(int64_t base_offset, const Record* recs, size_t n);
// Record set of consecutive batches, each at most ~max_batch_bytes (a broker refuses a batch
// over message.max.bytes: 1 048 588 by default)
constexpr size_t kMaxBatchBytes = 900u * 1024u;
std::string encode_record_set(const std::vector<Record>& recs, size_t max_batch_bytes = kMaxBatchBytes);
void decode_record_batches(const uint8_t* p, size_t n, int64_t min_offset, FetchResult& out);

// Zero-copy iteration over the records of a fetched record set (v2 batches, CRC
// checked once per batch): values and keys are pointers into the caller's buffer.
struct RecordView {
  int64_t offset = 0, timestamp = 0;
  const uint8_t* key = nullptr;
  int64_t key_len = -1;   // -1 = null key
  const uint8_t* value = nullptr;
  int64_t value_len = 0;
};
class RecordSetCursor {
 public:
  RecordSetCursor() = default;
  // verify_crc: check each record batch's CRC-32C (consumers that trust the transport may
  // skip it, as librdkafka does by default: check.crcs=false)
  RecordSetCursor(const uint8_t* p, size_t n, bool verify_crc = true) : p_(p), n_(n), crc_(verify_crc) {}
  // next data record (control batches / records skipped); false at the end of the set
  bool next(RecordView& out);
 private:
  const uint8_t* p_ = nullptr;
  size_t n_ = 0, pos_ = 0;      // next batch header
  const uint8_t* bp_ = nullptr;  // current batch records area
  size_t bn_ = 0, bi_ = 0;
  int32_t left_ = 0;
  int64_t base_ = 0, first_ts_ = 0;
  bool control_ = false;
  bool crc_ = true;
};

struct ClientConfig {
  std::string client_id = "streamml";
  std::string sasl_mechanism;  // "" or "PLAIN"
  std::string sasl_username, sasl_password;
  int timeout_ms = 30000;
  int max_retries = 5;
  // > 0: busy-poll (non-blocking recv) a response this many microseconds before blocking --
  // the low-latency serving loop's socket policy (a blocked recv costs a thread wake-up)
  int spin_us = 0;
};

class Connection;

class Client {
 public:
  Client(const std::string& bootstrap, ClientConfig cfg);
  ~Client();

  std::map<std::string, int> partitions();                      // topic -> #partitions
  int64_t list_offset(const std::string& topic, int partition, int64_t time);  // -2 earliest, -1 latest
  FetchResult fetch(const std::string& topic, int partition, int64_t offset, int32_t max_bytes = 1 << 20,
                    int32_t max_wait_ms = 100);
  // Fetch without materialising records: `resp` keeps the whole response; the record set
  // is resp[rec_off, rec_off + rec_len) (iterate it with RecordSetCursor).  Returns the
  // partition's high watermark.
  int64_t fetch_raw(const std::string& topic, int partition, int64_t offset, int32_t max_bytes,
                    int32_t max_wait_ms, std::string& resp, size_t& rec_off, size_t& rec_len);
  int64_t produce(const std::string& topic, int partition, const std::vector<Record>& recs, int16_t acks = 1);
  // Fetch several partitions of one topic in ONE request (they must share a leader:
  // same_leader()); a long poll returns as soon as ANY of them has records.  On return
  // `parts[i]` holds (record-set offset, record-set length, high watermark) inside `resp`
  // for the i-th requested (partition, offset).
  struct PartSlice {
    size_t rec_off = 0, rec_len = 0;
    int64_t hwm = -1;
  };
  void fetch_multi_raw(const std::string& topic, const std::vector<std::pair<int, int64_t>>& want, int32_t max_bytes,
                       int32_t max_wait_ms, std::string& resp, std::vector<PartSlice>& parts);
  bool same_leader(const std::string& topic, const std::vector<int>& partitions);
  // commit several partitions' offsets in one OffsetCommit request
  void commit_multi(const std::string& group, const std::string& topic,
                    const std::vector<std::pair<int, int64_t>>& offsets);
  // Several partitions of one topic: ONE Produce request per partition leader carrying all
  // of that leader's partitions (one round trip instead of one per partition).
  void produce_multi(const std::string& topic, const std::vector<std::pair<int, std::vector<Record>>>& parts,
                     int16_t acks = 1);
  void commit(const std::string& group, const std::string& topic, int partition, int64_t offset);
  int64_t committed(const std::string& group, const std::string& topic, int partition);
  // topic empty: all topics (replaces the cache); else that topic only (merged; on
  // brokers with auto.create.topics.enable this creates it, as librdkafka does).
  void refresh_metadata(const std::string& topic = std::string());
  uint64_t bytes_received() const { return bytes_rx_; }

 private:
  struct BrokerAddr {
    std::string host;
    int port;
  };
  ClientConfig cfg_;
  std::vector<BrokerAddr> bootstrap_;
  std::map<int32_t, BrokerAddr> brokers_;
  std::map<std::string, std::vector<int32_t>> leaders_;  // topic -> leader per partition
  std::map<int32_t, std::unique_ptr<Connection>> conns_;
  std::unique_ptr<Connection> any_;
  int32_t corr_ = 1;
  uint64_t bytes_rx_ = 0;
  std::mutex mu_;

  Connection& conn_for(const std::string& topic, int partition);
  Connection& any_conn();
  std::unique_ptr<Connection> open(const BrokerAddr& a);
  std::string call(Connection& c, int16_t api, int16_t ver, const std::string& body);
  // same, into a caller buffer that is only ever grown (no per-call allocation / zero-fill);
  // returns the response length
  size_t call_into(Connection& c, int16_t api, int16_t ver, const std::string& body, std::string& resp);
};

struct BrokerConfig {
  int port = 0;  // 0 = ephemeral
  std::string sasl_username, sasl_password;  // empty = no auth
  int64_t retention_records = -1;           // -1 = unbounded
  // Kafka's retention.ms / retention.bytes topic defaults (log.retention.*): -1 = unbounded.  The
  // reference creates sensor-data and model-predictions with retention.ms=100000
  // (infrastructure/confluent/01_installConfluentPlatform.sh:180, 183).  A background check every
  // retention_check_ms (log.retention.check.interval.ms) deletes whole segments, oldest first.
  int64_t retention_ms = -1;
  int64_t retention_bytes = -1;
  int retention_check_ms = 1000;
  bool auto_create_topics = true;            // Kafka's auto.create.topics.enable default
  int spin_us = 0;                           // > 0: connection threads / long polls busy-wait this long first
  int64_t message_max_bytes = 1048588;        // Kafka's message.max.bytes default (per record batch); <= 0 = no cap
};

class Broker {
 public:
  explicit Broker(BrokerConfig cfg);
  ~Broker();
  int port() const { return port_; }
  // retention_ms / retention_bytes: the topic's retention.ms / retention.bytes (-2 = the broker
  // default, -1 = unbounded)
  void create_topic(const std::string& name, int partitions, int64_t retention_ms = -2, int64_t retention_bytes = -2);
  // One retention pass now (the background check runs the same): returns segments deleted.
  size_t enforce_retention();
  uint64_t deleted_segments() const { return deleted_segs_; }
  uint64_t deleted_records() const { return deleted_recs_; }
  // bytes / segments held by the log (all topics)
  int64_t log_bytes();
  size_t log_segments();
  int64_t append(const std::string& topic, int partition, const std::vector<Record>& recs);
  int64_t end_offset(const std::string& topic, int partition);
  int64_t start_offset(const std::string& topic, int partition);
  std::vector<Record> read(const std::string& topic, int partition, int64_t offset, size_t max_records);
  // fault injection: every `fail_every`-th fetch returns NOT_LEADER_OR_FOLLOWER;
  // every fetch is delayed by `delay_ms`.
  void set_faults(int fail_every, int delay_ms) {
    fail_every_ = fail_every;
    delay_ms_ = delay_ms;
  }
  uint64_t fetch_count() const { return fetches_; }
  // Low-latency mode: each connection thread busy-polls its socket, and an empty long-poll
  // fetch watches the append counter, for `us` microseconds before blocking (0 = off).
  void set_spin_us(int us) { spin_us_ = us; }
  // CPUs for the connection threads accepted from now on (empty: unpinned).  The latency
  // bench keeps every spinning thread of the append -> result path on one L3 domain: a hop
  // between core complexes costs microseconds on the loopback path.
  void set_thread_cpus(const std::vector<int>& cpus);
  // Record the steady-clock time (ns, the process's std::chrono::steady_clock) at which
  // every record is appended from now on -- Kafka's LogAppendTime, for latency accounting.
  void record_append_times(bool on);
  // Append times of offsets [start, start + count) of a partition (-1 where not recorded).
  std::vector<int64_t> append_times(const std::string& topic, int partition, int64_t start, int64_t count);
  uint64_t injected_failures() const { return failures_; }
  void stop();

 private:
  // The log is kept the way Kafka keeps it: as encoded record batches, served to
  // fetches verbatim (a fetch copies whole batches; the consumer skips the records
  // below its offset).  Segments are immutable and shared, so a fetch assembles its
  // response outside the broker lock.
  static constexpr size_t kSegmentRecords = 1024;
  struct Segment {
    int64_t base = 0;
    int32_t count = 0;
    int64_t append_ms = 0;   // steady-clock ms of the append (the segment's newest record)
    std::shared_ptr<const std::string> bytes;
  };
  struct Partition {
    std::deque<Segment> segs;   // retention pops from the front: O(deleted), not O(retained)
    int64_t start = 0;  // offset of the first retained record
    int64_t end = 0;    // next offset to assign
    int64_t bytes = 0;  // encoded bytes of segs
    int64_t tbase = -1;              // first offset with a recorded append time
    std::deque<int64_t> tappend;     // append times (ns) of offsets tbase, tbase + 1, ...
  };
  int64_t append_locked(Partition& p, const Record* recs, size_t n);
  // A fetch reply: the response framing in `meta`, with the (shared, immutable) segment
  // bytes of each partition spliced in at byte offset `at` of `meta` -- sent with
  // sendmsg() straight from the log segments, never concatenated.
  struct FetchReply {
    std::string meta;
    std::vector<std::pair<size_t, std::shared_ptr<const std::string>>> splice;
    size_t total() const;
  };
  FetchReply handle_fetch(const uint8_t* body, size_t n);
  BrokerConfig cfg_;
  std::vector<int> thread_cpus_;   // guarded by mu_
  int listen_fd_ = -1;
  int port_ = 0;
  std::atomic<bool> running_{false};
  std::thread accept_thread_;
  std::vector<std::thread> workers_;
  std::vector<int> client_fds_;
  std::mutex mu_;
  std::map<std::string, std::vector<Partition>> topics_;
  struct TopicRetention {
    int64_t ms = -2, bytes = -2;   // -2: the broker default
  };
  std::map<std::string, TopicRetention> retention_;   // guarded by mu_
  std::thread retention_thread_;
  std::condition_variable retention_cv_;
  std::atomic<uint64_t> deleted_segs_{0}, deleted_recs_{0};
  void retention_loop();
  // Deleted segment bytes are moved into `dead` so the caller frees them after unlocking.
  size_t enforce_locked(int64_t now_ms, std::vector<std::shared_ptr<const std::string>>& dead);
  // finished connection threads, joined by the accept loop (a long soak opens many connections)
  std::vector<std::shared_ptr<std::atomic<bool>>> worker_done_;
  std::condition_variable data_cv_;   // appends -> long-polling fetches
  std::map<std::string, int64_t> group_offsets_;  // "group/topic/partition" -> offset
  std::atomic<int> fail_every_{0}, delay_ms_{0}, spin_us_{0};
  std::atomic<bool> record_times_{false};
  std::atomic<uint64_t> append_seq_{0};   // bumped by every append: lock-free wake-up check for spinning polls
  std::atomic<uint64_t> fetches_{0}, failures_{0};

  void accept_loop();
  void serve(int fd);
  std::string handle(int16_t api, int16_t ver, const uint8_t* body, size_t n, bool& authed, bool& handshaken);
};

}  // namespace kafka
}  // namespace sml
