// Native Kafka ingest feed: partition-parallel fetch + Avro decode straight into
// caller-owned (page-locked) slabs.
//
// The reference reads its training data through tensorflow-io's KafkaDataset ->
// substr(e, 5) -> decode_avro -> normalize_fn, one tf.string per message
// (AUTOENCODER-TensorFlow-IO-Kafka/cardata-v3.py:44-75).  Here `workers` C++ threads, each
// with its own broker connection, own disjoint partitions; every fetched record set is
// walked in place (RecordSetCursor: no per-record copies or allocations), the
// Confluent-framed Avro value is decoded field by field and only the projected features
// (float32, in the model's column order) and the failure_occurred label code are written,
// row by row, into a slab the Python side allocated with hipHostMalloc (the pinned ring
// the H2D copy engine reads).  An optional label filter (the reference's
// filter(y == "false"), cardata-v3.py:212) drops rows at decode time.  No Python object is
// created per record and the GIL is never taken by the workers.
//
// Slab protocol: start() hands over S slabs of `cap` rows; a worker takes a free slab,
// fills it (rows [n][F] float32 followed by n label bytes), and publishes it; pop()
// returns published slabs (per-partition order is kept: a partition belongs to one
// worker, whose slabs are published in order); recycle() returns a slab once its H2D copy
// has completed.
#pragma once
#include <atomic>
#include <condition_variable>
#include <cstdint>
#include <deque>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "avro.h"
#include "kafka.h"

namespace sml {
namespace feed {

struct PartSpec {
  std::string topic;
  int partition = 0;
  int64_t start = 0;
  int64_t end = -1;   // exclusive; < 0: unbounded (follow the log)
};

struct FeedConfig {
  std::vector<int> feature_fields;   // schema field index of each output feature
  int label_field = -1;              // schema field index of the label string (-1: label 0)
  int keep_label = -1;               // >= 0: keep only rows with this label code
  bool framing = true;               // Confluent 5-byte header
  int32_t max_bytes = 4 << 20;
  int32_t max_wait_ms = 100;
  int workers = 1;
  double idle_timeout_s = -1.0;      // unbounded streams: a worker stops after this long without data
  // librdkafka's check.crcs (default false there too): verify every record batch's CRC-32C.
  // The checksum is one dependent crc32 chain over every byte (~16 ns of a ~45 ns row decode)
  bool check_crcs = false;
  // auto.offset.reset after OFFSET_OUT_OF_RANGE (the position was deleted by retention):
  // 0 earliest, 1 latest, 2 none (the worker fails)
  int offset_reset = 0;
};

struct Stats {
  uint64_t records = 0, rows = 0, dropped = 0, errors = 0, bytes = 0, fetches = 0, slabs = 0;
  uint64_t reset_skipped = 0;   // records jumped over by auto.offset.reset
  double fetch_s = 0, decode_s = 0, wait_slab_s = 0;
};

// label codes (streamml.data.stream): 0 "false", 1 "true", 2 missing / other
uint8_t label_code(const uint8_t* p, size_t n);

class Feed {
 public:
  Feed(std::string bootstrap, kafka::ClientConfig ccfg, std::vector<avro::Field> fields, FeedConfig cfg,
       std::vector<PartSpec> parts);
  ~Feed();
  Feed(const Feed&) = delete;
  Feed& operator=(const Feed&) = delete;

  void start(const std::vector<uintptr_t>& slabs, int64_t cap_rows);
  // Pre-staged source: the n record values of buf (value i = buf[offs[i], offs[i+1]), as fetched
  // responses hold them) split into `workers` contiguous shares, each decoded by its own thread into
  // the slabs and published like fetched rows -- the decode + ring + H2D path without the broker
  // (buf / offs must outlive the stream).  No partitions, no commit marks.
  void start_staged(const std::vector<uintptr_t>& slabs, int64_t cap_rows, const uint8_t* buf, const int64_t* offs,
                    int64_t n, int workers);
  // 1 = got a slab, 0 = timed out, -1 = end of stream.  Rethrows a worker's error.
  int pop(int& slab, int64_t& rows, int timeout_ms);
  void recycle(int slab);
  void stop();
  Stats stats() const;
  std::vector<int64_t> positions() const;   // next offset to read, per PartSpec
  // commit marks of a popped slab: (PartSpec index, next offset) of the publishing worker's
  // partitions at publish time -- every record before them is in this slab, an earlier slab
  // of the same worker, or was dropped by the label filter (at-least-once commit points)
  std::vector<std::pair<int, int64_t>> slab_marks(int slab) const;
  int features() const { return (int)cfg_.feature_fields.size(); }
  // decode one (framed) Avro value into a projected row + label code; false = malformed
  bool decode_row(const uint8_t* p, size_t n, float* out_row, uint8_t* label) const;
  // Decode-only rate: the n values of a pre-staged buffer (value i = buf[offs[i], offs[i+1]),
  // as fetched record values sit in a response) split into `workers` contiguous shares,
  // each decoded by its own thread into a private slab -- no broker, no socket, no ring.
  // Best rows/s over `repeats`; `rows_out` = rows decoded per pass.
  double decode_throughput(const uint8_t* buf, const int64_t* offs, int64_t n, int workers, int repeats,
                           int64_t* rows_out) const;
  // runs of the fast plan (0: the schema takes the generic interpreted plan)
  int fast_plan() const { return fast_ ? (int)runs_.size() : 0; }

 private:
  struct Part {
    PartSpec spec;
    std::atomic<int64_t> pos{0};
    bool done = false;
  };
  struct Worker {
    std::thread th;
    std::vector<int> parts;
  };
  void run_staged(int w, const uint8_t* buf, const int64_t* offs, int64_t a, int64_t b);
  std::string bootstrap_;
  kafka::ClientConfig ccfg_;
  std::vector<avro::Field> fields_;
  std::vector<int> col_of_;   // schema field -> output feature column (-1 = not projected)
  struct Op {                 // compiled decode plan, one entry per schema field
    uint8_t kind;
    int8_t null_branch;
    int8_t col;               // output column, -1 = skip
    uint8_t label;            // 1 = the label string
    int32_t fixed;
  };
  std::vector<Op> plan_;
  // Fast plan (schemas of float / int / long / double / string fields, plain or as KSQL's
  // ["null", T] unions -- the car schemas): runs of same-kind fields landing in consecutive
  // output columns, decoded assuming every union takes its value branch: one bounds check
  // per run, no per-field dispatch.  Any other byte (a null, a malformed value) sends the row
  // to the generic interpreted plan, which decides.
  struct Run {
    uint8_t kind;
    uint8_t n;                // fields in the run
    int8_t col;               // first output column, -1 = skip
    uint8_t label;
    int16_t vb;               // union: the value branch's index byte (0x00 / 0x02); -1 = plain
  };
  std::vector<Run> runs_;
  bool fast_ = false;
  // 1 = decoded, -1 = not the common shape (the caller runs the generic plan)
  int decode_fast(const uint8_t* p, size_t n, float* out_row, uint8_t* label) const;
  FeedConfig cfg_;
  std::vector<std::unique_ptr<Part>> parts_;
  std::vector<Worker> workers_;
  std::vector<uintptr_t> slabs_;
  int64_t cap_ = 0;

  mutable std::mutex mu_;
  std::condition_variable cv_ready_, cv_free_;
  std::deque<int> free_;
  std::deque<std::pair<int, int64_t>> ready_;
  int live_workers_ = 0;
  bool stop_ = false;
  std::string error_;
  Stats stats_;

  void run(int w);
  int take_free(double& waited);
  void publish(int w, int slab, int64_t rows);
  std::vector<std::vector<std::pair<int, int64_t>>> marks_;   // per slab, see slab_marks()
};

}  // namespace feed
}  // namespace sml
