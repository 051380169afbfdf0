#include "scoreloop.h"

#include <chrono>
#include <stdexcept>
#include <thread>

#include "format.h"

namespace sml {
namespace serve {

int64_t steady_ns() {
  return std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now().time_since_epoch())
      .count();
}

namespace {

feed::FeedConfig decoder_config(const LoopConfig& c) {
  feed::FeedConfig f;
  f.feature_fields = c.feature_fields;
  f.label_field = -1;
  f.framing = c.framing;
  return f;
}

double secs(int64_t a, int64_t b) { return (double)(b - a) * 1e-9; }

}  // namespace

ScoreLoop::ScoreLoop(std::string bootstrap, kafka::ClientConfig ccfg, std::vector<avro::Field> fields, LoopConfig cfg,
                     const SmlScorerApi* api)
    : bootstrap_(bootstrap),
      ccfg_(ccfg),
      cfg_(std::move(cfg)),
      api_(api),
      decoder_(bootstrap, ccfg, std::move(fields), decoder_config(cfg_), {}) {
  if (!api_ || api_->version != SML_SCORER_API_VERSION || !api_->infer)
    throw std::invalid_argument("scoreloop: bad scorer API table");
  if (api_->dim != decoder_.features())
    throw std::invalid_argument("scoreloop: scorer dim != number of feature fields");
  if (cfg_.partitions.empty() || cfg_.starts.size() != cfg_.partitions.size() ||
      cfg_.result_partitions.size() != cfg_.partitions.size())
    throw std::invalid_argument("scoreloop: partitions / starts / result_partitions mismatch");
  if (cfg_.max_batch < 1) throw std::invalid_argument("scoreloop: max_batch >= 1");
  pos_ = cfg_.starts;
}

std::vector<int64_t> ScoreLoop::positions() const { return pos_; }

LoopStats ScoreLoop::run(int64_t max_events, double idle_timeout_s) {
  stop_ = false;
  kafka::Client cli(bootstrap_, ccfg_);
  const int D = api_->dim;
  const size_t np = cfg_.partitions.size();
  LoopStats st;
  std::string resp;
  size_t ro = 0, rl = 0;
  std::vector<float> rows, scores, recon;
  std::vector<uint32_t> flags;
  std::vector<int64_t> offs;
  std::vector<std::pair<const uint8_t*, int64_t>> keys;
  std::vector<kafka::Record> out;
  std::vector<char> dirty(np, 0);
  const int64_t t_start = steady_ns();
  int64_t last_data = t_start, last_commit = t_start;
  bool idle_round = false;
  auto commit_all = [&]() {
    if (cfg_.group.empty()) return;
    const int64_t t0 = steady_ns();
    for (size_t i = 0; i < np; ++i)
      if (dirty[i]) {
        cli.commit(cfg_.group, cfg_.topic, cfg_.partitions[i], pos_[i]);
        dirty[i] = 0;
        ++st.commits;
      }
    last_commit = steady_ns();
    st.commit_s += secs(t0, last_commit);
  };
  while (!stop_) {
    bool any = false;
    for (size_t pi = 0; pi < np && !stop_; ++pi) {
      // one partition: always long-poll; several: long-poll (briefly) only after an empty round
      const int32_t wait = np == 1 ? cfg_.max_wait_ms : (idle_round && pi == 0 ? std::min(cfg_.max_wait_ms, 2) : 0);
      int64_t t0 = steady_ns();
      cli.fetch_raw(cfg_.topic, cfg_.partitions[pi], pos_[pi], cfg_.max_bytes, wait, resp, ro, rl);
      int64_t t1 = steady_ns();
      st.fetch_s += secs(t0, t1);
      ++st.fetches;
      // decode every record at or past our position
      rows.clear();
      offs.clear();
      keys.clear();
      kafka::RecordSetCursor cur(reinterpret_cast<const uint8_t*>(resp.data()) + ro, rl);
      kafka::RecordView v;
      int64_t next = pos_[pi];
      while (cur.next(v)) {
        if (v.offset < pos_[pi]) continue;
        next = v.offset + 1;
        rows.resize(rows.size() + (size_t)D);
        uint8_t lab = 0;
        if (!decoder_.decode_row(v.value, (size_t)v.value_len, rows.data() + rows.size() - (size_t)D, &lab)) {
          rows.resize(rows.size() - (size_t)D);   // undecodable: skipped, not scored
          ++st.skipped;
          continue;
        }
        offs.push_back(v.offset);
        keys.emplace_back(v.key, v.key_len);
      }
      const int64_t t2 = steady_ns();
      st.decode_s += secs(t1, t2);
      if (next == pos_[pi]) {
        ++st.empty_fetches;
        continue;
      }
      any = true;
      pos_[pi] = next;
      dirty[pi] = 1;
      const int k = (int)offs.size();
      if (k > 0) {
        scores.resize((size_t)k);
        flags.resize((size_t)k);
        if (cfg_.emit_recon) recon.resize((size_t)k * (size_t)D);
        for (int b = 0; b < k; b += cfg_.max_batch) {
          const int n = std::min(cfg_.max_batch, k - b);
          if (api_->infer(api_->ctx, rows.data() + (size_t)b * D, n, scores.data() + b, flags.data() + b,
                          cfg_.emit_recon ? recon.data() + (size_t)b * D : nullptr, 10.0) != 0)
            throw std::runtime_error(std::string("scoreloop: scorer failed: ") +
                                     (api_->last_error ? api_->last_error(api_->ctx) : "?"));
        }
        const int64_t t3 = steady_ns();
        st.score_s += secs(t2, t3);
        out.resize((size_t)k);
        const int64_t now_ms = std::chrono::duration_cast<std::chrono::milliseconds>(
                                   std::chrono::system_clock::now().time_since_epoch())
                                   .count();
        for (int i = 0; i < k; ++i) {
          kafka::Record& r = out[(size_t)i];
          r.offset = i;
          r.timestamp = now_ms;
          r.key_null = keys[(size_t)i].second < 0;
          if (r.key_null) r.key.clear();
          else r.key.assign(reinterpret_cast<const char*>(keys[(size_t)i].first), (size_t)keys[(size_t)i].second);
          r.value.clear();
          fmt::score_record_json(keys[(size_t)i].first, keys[(size_t)i].second, cfg_.partitions[pi],
                                 offs[(size_t)i], scores[(size_t)i], flags[(size_t)i] != 0,
                                 cfg_.emit_recon ? recon.data() + (size_t)i * D : nullptr, D, r.value);
          st.anomalies += flags[(size_t)i] != 0;
        }
        const int64_t t4 = steady_ns();
        st.format_s += secs(t3, t4);
        cli.produce(cfg_.result_topic, cfg_.result_partitions[pi], out, 1);
        const int64_t t5 = steady_ns();
        st.produce_s += secs(t4, t5);
        if (cfg_.record_latency)
          for (int i = 0; i < k; ++i) {   // kLatCols per event (scoreloop.h)
            lat_.push_back(cfg_.partitions[pi]);
            lat_.push_back(offs[(size_t)i]);
            lat_.push_back(t5);
            lat_.push_back(t1);
            lat_.push_back(t3);
            lat_.push_back(t4);
          }
        st.events += (uint64_t)k;
        ++st.batches;
      }
      if (cfg_.commit_interval_s <= 0.0 || secs(last_commit, steady_ns()) >= cfg_.commit_interval_s) commit_all();
      if (max_events > 0 && (int64_t)st.events >= max_events) stop_ = true;
    }
    const int64_t now = steady_ns();
    if (any) last_data = now;
    idle_round = !any;
    if (!any && idle_timeout_s >= 0.0 && secs(last_data, now) >= idle_timeout_s) break;
  }
  commit_all();
  st.wall_s = secs(t_start, steady_ns());
  return st;
}

std::vector<int64_t> paced_produce(const std::string& bootstrap, kafka::ClientConfig ccfg, const std::string& topic,
                                   int partition, const std::string& values, const std::vector<int64_t>& offs,
                                   const std::vector<std::string>& keys, double qps) {
  if (offs.empty()) return {};
  const size_t n = offs.size() - 1;
  if (!keys.empty() && keys.size() != n) throw std::invalid_argument("paced_produce: keys length mismatch");
  kafka::Client cli(bootstrap, ccfg);
  std::vector<int64_t> sent(n);
  std::vector<kafka::Record> one(1);
  const int64_t gap = qps > 0 ? (int64_t)(1e9 / qps) : 0;
  int64_t next = steady_ns();
  for (size_t i = 0; i < n; ++i) {
    while (steady_ns() < next) std::this_thread::yield();
    kafka::Record& r = one[0];
    r.value.assign(values, (size_t)offs[i], (size_t)(offs[i + 1] - offs[i]));
    r.key_null = keys.empty();
    if (!keys.empty()) r.key = keys[i];
    r.timestamp = std::chrono::duration_cast<std::chrono::milliseconds>(
                      std::chrono::system_clock::now().time_since_epoch())
                      .count();
    sent[i] = steady_ns();
    cli.produce(topic, partition, one, 1);
    next += gap;
  }
  return sent;
}

}  // namespace serve
}  // namespace sml
