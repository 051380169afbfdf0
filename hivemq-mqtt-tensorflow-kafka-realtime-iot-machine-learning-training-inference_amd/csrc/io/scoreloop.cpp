#include "scoreloop.h"

#include <algorithm>
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

uint32_t key_share_hash(const uint8_t* key, int64_t len) {
  uint64_t h = 0xCBF29CE484222325ull;
  for (int64_t i = 0; i < len; ++i) {
    h ^= key[i];
    h *= 0x100000001B3ull;
  }
  h ^= h >> 33;   // fmix64: FNV-1a's top bits barely move for keys differing at the end
  h *= 0xFF51AFD7ED558CCDull;
  h ^= h >> 33;
  h *= 0xC4CEB9FE1A85EC53ull;
  h ^= h >> 33;
  return (uint32_t)(h >> 32);
}

ScoreLoop::ScoreLoop(std::string bootstrap, kafka::ClientConfig ccfg, std::vector<avro::Field> fields, LoopConfig cfg,
                     const SmlScorerApi* api)
    : bootstrap_(bootstrap),
      ccfg_(ccfg),
      cfg_(std::move(cfg)),
      api_(api),
      decoder_(bootstrap, ccfg, std::move(fields), decoder_config(cfg_), {}) {
  if (!api_ || api_->version != SML_SCORER_API_VERSION || !api_->infer)
    throw std::invalid_argument("scoreloop: bad scorer API table");
  if (api_->nkeys > 0 && !api_->infer_keyed) throw std::invalid_argument("scoreloop: keyed scorer without infer_keyed");
  if (!cfg_.json_columns.empty()) {
    json_ = std::make_unique<jsonrow::Plan>(cfg_.json_columns, "", cfg_.json_stamp);
    if (json_->width() != api_->dim) throw std::invalid_argument("scoreloop: scorer dim != number of JSON columns");
  } else if (api_->dim != decoder_.features()) {
    throw std::invalid_argument("scoreloop: scorer dim != number of feature fields");
  }
  if (cfg_.partitions.empty() || cfg_.starts.size() != cfg_.partitions.size() ||
      cfg_.result_partitions.size() != cfg_.partitions.size())
    throw std::invalid_argument("scoreloop: partitions / starts / result_partitions mismatch");
  if (!cfg_.hash_ranges.empty() && cfg_.hash_ranges.size() != cfg_.partitions.size())
    throw std::invalid_argument("scoreloop: one hash range per owned partition");
  if (cfg_.max_batch < 1) throw std::invalid_argument("scoreloop: max_batch >= 1");
  pos_ = cfg_.starts;
}

std::vector<int64_t> ScoreLoop::positions() const { return pos_; }

LoopStats ScoreLoop::run(int64_t max_events, double idle_timeout_s) {
  stop_ = false;
  kafka::Client cli(bootstrap_, ccfg_);
  const int D = api_->dim;
  const size_t np = cfg_.partitions.size();
  // Owned partitions that share a leader are fetched in ONE request, whose long poll wakes
  // on an append to any of them (and their results go out in one produce, their offsets in
  // one commit); otherwise one partition per fetch, round robin, long-polling briefly only
  // after a round that found nothing.
  const bool multi = np > 1 && cli.same_leader(cfg_.topic, cfg_.partitions);
  // The latency records of a bounded run are reserved up front: a doubling push_back inside
  // the loop copies every record so far (a 10-minute soak stalled 150 / 290 ms at the 256 /
  // 512 MB doublings); the reservation is only address space until the loop writes it.
  if (cfg_.record_latency && max_events > 0) {
    lat_.reserve(lat_.size() + (size_t)max_events * kLatCols);
  }
  LoopStats st;
  std::string resp;
  std::vector<kafka::Client::PartSlice> slices;
  std::vector<std::pair<int, int64_t>> want;
  std::vector<size_t> grp;
  std::vector<float> rows, scores, recon;
  std::vector<uint32_t> flags, kids;
  std::vector<int64_t> offs, stamps;
  std::vector<int> src;   // owned-partition index of each decoded row
  std::vector<std::pair<const uint8_t*, int64_t>> keys;
  std::vector<std::pair<int, std::vector<kafka::Record>>> outp;
  std::vector<int> res_slot(np, -1);
  std::vector<char> dirty(np, 0);
  const int64_t t_start = steady_ns();
  int64_t last_data = t_start, last_commit = t_start;
  bool idle_round = false, round_any = false;
  size_t rr = 0;
  auto commit_all = [&]() {
    if (cfg_.group.empty()) return;
    const int64_t t0 = steady_ns();
    std::vector<std::pair<int, int64_t>> co;
    for (size_t i = 0; i < np; ++i)
      if (dirty[i]) {
        co.emplace_back(cfg_.partitions[i], pos_[i]);
        dirty[i] = 0;
      }
    if (!co.empty()) {
      cli.commit_multi(cfg_.group, cfg_.topic, co);
      st.commits += co.size();
    }
    last_commit = steady_ns();
    st.commit_s += secs(t0, last_commit);
  };
  while (!stop_) {
    grp.clear();
    int32_t wait = cfg_.max_wait_ms;
    if (multi || np == 1) {
      for (size_t i = 0; i < np; ++i) grp.push_back(i);
    } else {
      grp.push_back(rr);
      wait = idle_round && rr == 0 ? std::min(cfg_.max_wait_ms, 2) : 0;
    }
    if (grp.size() > 1) {   // rotate the request order: a broker fills the response in request
      std::rotate(grp.begin(), grp.begin() + (long)(rot_ % grp.size()), grp.end());   // order up to
      rot_ = (rot_ + 1) % grp.size();                                               // max_bytes
    }
    want.clear();
    for (size_t i : grp) want.emplace_back(cfg_.partitions[i], pos_[i]);
    const int64_t t0 = steady_ns();
    try {
      if (grp.size() == 1) {
        slices.assign(1, kafka::Client::PartSlice{});
        slices[0].hwm = cli.fetch_raw(cfg_.topic, want[0].first, want[0].second, cfg_.max_bytes, wait, resp,
                                      slices[0].rec_off, slices[0].rec_len);
      } else {
        cli.fetch_multi_raw(cfg_.topic, want, cfg_.max_bytes, wait, resp, slices);
      }
    } catch (const kafka::Error& e) {
      // OFFSET_OUT_OF_RANGE: a position was deleted by the topic's retention -> auto.offset.reset
      // for every requested partition below its log start (or past its end)
      if (e.code != 1 || cfg_.offset_reset == 2) throw;
      for (size_t i : grp) {
        const int64_t lo = cli.list_offset(cfg_.topic, cfg_.partitions[i], -2);
        const int64_t hi = cli.list_offset(cfg_.topic, cfg_.partitions[i], -1);
        if (pos_[i] >= lo && pos_[i] <= hi) continue;
        const int64_t np = cfg_.offset_reset == 1 ? hi : lo;
        if (np > pos_[i]) st.reset_skipped += (uint64_t)(np - pos_[i]);
        pos_[i] = np;
        dirty[i] = 1;
      }
      continue;
    }
    const int64_t t1 = steady_ns();
    st.fetch_s += secs(t0, t1);
    ++st.fetches;
    // decode every record at or past our position, in partition order
    rows.clear();
    offs.clear();
    keys.clear();
    stamps.clear();
    src.clear();
    bool progress = false;
    for (size_t gi = 0; gi < grp.size(); ++gi) {
      const size_t pi = grp[gi];
      kafka::RecordSetCursor cur(reinterpret_cast<const uint8_t*>(resp.data()) + slices[gi].rec_off,
                                 slices[gi].rec_len);
      kafka::RecordView v;
      int64_t next = pos_[pi];
      const bool shared = !cfg_.hash_ranges.empty() &&
                          !(cfg_.hash_ranges[pi].first == 0 && cfg_.hash_ranges[pi].second >= (1ull << 32));
      while (cur.next(v)) {
        if (v.offset < pos_[pi]) continue;
        next = v.offset + 1;
        if (shared) {   // a car of this partition that another replica owns
          const uint64_t kh = key_share_hash(v.key, v.key_len < 0 ? 0 : v.key_len);
          if (kh < cfg_.hash_ranges[pi].first || kh >= cfg_.hash_ranges[pi].second) {
            ++st.foreign;
            continue;
          }
        }
        rows.resize(rows.size() + (size_t)D);
        uint8_t lab = 0;
        int64_t stamp = 0;
        float* row = rows.data() + rows.size() - (size_t)D;
        const bool ok = json_ ? json_->decode(v.value, (size_t)v.value_len, row, &lab, &stamp)
                              : decoder_.decode_row(v.value, (size_t)v.value_len, row, &lab);
        if (!ok) {
          rows.resize(rows.size() - (size_t)D);   // undecodable: skipped, not scored
          ++st.skipped;
          continue;
        }
        stamps.push_back(stamp);
        offs.push_back(v.offset);
        keys.emplace_back(v.key, v.key_len);
        src.push_back((int)pi);
      }
      if (next != pos_[pi]) {
        pos_[pi] = next;
        dirty[pi] = 1;
        progress = true;
      }
    }
    const int64_t t2 = steady_ns();
    st.decode_s += secs(t1, t2);
    if (!progress) ++st.empty_fetches;
    round_any |= progress;
    int k = (int)offs.size();
    if (k > 0 && api_->nkeys > 0) {   // record key -> the key's device slot
      {
        kids.resize((size_t)k);
        int w = 0;   // rows kept: a null key or a key past the slot table is skipped, counted
        for (int i = 0; i < k; ++i) {
          const auto& kv = keys[(size_t)i];
          if (kv.second < 0) {
            ++st.keys_dropped;
            continue;
          }
          std::string key(reinterpret_cast<const char*>(kv.first), (size_t)kv.second);
          auto it = key_ids_.find(key);
          if (it == key_ids_.end()) {
            if ((int64_t)key_ids_.size() >= api_->nkeys) {
              ++st.keys_dropped;
              continue;
            }
            it = key_ids_.emplace(std::move(key), (uint32_t)key_ids_.size()).first;
            st.keys = key_ids_.size();
          }
          if (w != i) {
            std::copy(rows.begin() + (size_t)i * D, rows.begin() + (size_t)(i + 1) * D, rows.begin() + (size_t)w * D);
            offs[(size_t)w] = offs[(size_t)i];
            keys[(size_t)w] = keys[(size_t)i];
            stamps[(size_t)w] = stamps[(size_t)i];
            src[(size_t)w] = src[(size_t)i];
          }
          kids[(size_t)w++] = it->second;
        }
        k = w;
      }
    }
    if (k > 0) {
      scores.resize((size_t)k);
      flags.resize((size_t)k);
      if (cfg_.emit_recon) recon.resize((size_t)k * (size_t)D);
      for (int b = 0; b < k; b += cfg_.max_batch) {
        const int n = std::min(cfg_.max_batch, k - b);
        float* rc = cfg_.emit_recon ? recon.data() + (size_t)b * D : nullptr;
        const int rc_err = api_->nkeys > 0
                               ? api_->infer_keyed(api_->ctx, rows.data() + (size_t)b * D, kids.data() + b, n,
                                                   scores.data() + b, flags.data() + b, rc, 10.0)
                               : api_->infer(api_->ctx, rows.data() + (size_t)b * D, n, scores.data() + b,
                                             flags.data() + b, rc, 10.0);
        if (rc_err != 0)
          throw std::runtime_error(std::string("scoreloop: scorer failed: ") +
                                   (api_->last_error ? api_->last_error(api_->ctx) : "?"));
      }
      const int64_t t3 = steady_ns();
      st.score_s += secs(t2, t3);
      // result records, grouped by result partition (a source partition's order is kept)
      for (auto& o : outp) o.second.clear();
      const int64_t now_ms = std::chrono::duration_cast<std::chrono::milliseconds>(
                                 std::chrono::system_clock::now().time_since_epoch())
                                 .count();
      for (int i = 0; i < k; ++i) {
        const int pi = src[(size_t)i];
        if (res_slot[(size_t)pi] < 0) {   // first result for this source partition
          const int rp = cfg_.result_partitions[(size_t)pi];
          int slot = -1;
          for (size_t q = 0; q < outp.size(); ++q)
            if (outp[q].first == rp) slot = (int)q;
          if (slot < 0) {
            outp.emplace_back(rp, std::vector<kafka::Record>());
            slot = (int)outp.size() - 1;
          }
          res_slot[(size_t)pi] = slot;
        }
        auto& vec = outp[(size_t)res_slot[(size_t)pi]].second;
        vec.emplace_back();
        kafka::Record& r = vec.back();
        r.offset = (int64_t)vec.size() - 1;
        r.timestamp = now_ms;
        r.key_null = keys[(size_t)i].second < 0;
        if (!r.key_null) r.key.assign(reinterpret_cast<const char*>(keys[(size_t)i].first), (size_t)keys[(size_t)i].second);
        // flag 1 = anomaly; a keyed forecaster's flag 2 = no previous forecast (score NaN)
        const bool anomaly = flags[(size_t)i] == 1;
        fmt::score_record_json(keys[(size_t)i].first, keys[(size_t)i].second, cfg_.partitions[(size_t)pi],
                               offs[(size_t)i], scores[(size_t)i], anomaly,
                               cfg_.emit_recon ? recon.data() + (size_t)i * D : nullptr, D, r.value);
        st.anomalies += anomaly;
      }
      const int64_t t4 = steady_ns();
      st.format_s += secs(t3, t4);
      if (outp.size() == 1) cli.produce(cfg_.result_topic, outp[0].first, outp[0].second, 1);
      else cli.produce_multi(cfg_.result_topic, outp, 1);
      const int64_t t5 = steady_ns();
      st.produce_s += secs(t4, t5);
      if (cfg_.record_latency)
        for (int i = 0; i < k; ++i) {   // kLatCols per event (scoreloop.h)
          lat_.push_back(cfg_.partitions[(size_t)src[(size_t)i]]);
          lat_.push_back(offs[(size_t)i]);
          lat_.push_back(t5);
          lat_.push_back(t1);
          lat_.push_back(t3);
          lat_.push_back(t4);
          lat_.push_back(stamps[(size_t)i]);
          lat_bytes_.store(lat_.size() * sizeof(int64_t), std::memory_order_relaxed);
        }
      st.events += (uint64_t)k;
      ++st.batches;
    }
    if (progress && (cfg_.commit_interval_s <= 0.0 || secs(last_commit, steady_ns()) >= cfg_.commit_interval_s))
      commit_all();
    if (max_events > 0 && (int64_t)st.events >= max_events) stop_ = true;
    // end of a round: every owned partition fetched once
    if (!multi && np > 1) {
      rr = (rr + 1) % np;
      if (rr != 0) continue;
    }
    const int64_t now = steady_ns();
    if (round_any) last_data = now;
    idle_round = !round_any;
    round_any = false;
    if (idle_round && idle_timeout_s >= 0.0 && secs(last_data, now) >= idle_timeout_s) break;
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
