// Native Kafka ingest feed (see feed.h).
#include "feed.h"

#include <chrono>
#include <cmath>
#include <cstring>
#include <stdexcept>

namespace sml {
namespace feed {

namespace {
using Clock = std::chrono::steady_clock;
double secs(Clock::time_point a, Clock::time_point b) { return std::chrono::duration<double>(b - a).count(); }

// zigzag varint, bounds checked; false on truncation / overlong
inline bool varlong(const uint8_t*& p, const uint8_t* e, int64_t& out) {
  uint64_t v = 0;
  for (int shift = 0; shift < 70 && p < e; shift += 7) {
    const uint8_t b = *p++;
    v |= (uint64_t)(b & 0x7f) << shift;
    if (!(b & 0x80)) {
      out = (int64_t)((v >> 1) ^ (~(v & 1) + 1));
      return true;
    }
  }
  return false;
}
}  // namespace

uint8_t label_code(const uint8_t* p, size_t n) {
  // case-insensitive "false" / "true" with surrounding blanks (streamml.data.stream.label_codes)
  while (n && (*p == ' ' || *p == '\t' || *p == '\n' || *p == '\r')) { ++p; --n; }
  while (n && (p[n - 1] == ' ' || p[n - 1] == '\t' || p[n - 1] == '\n' || p[n - 1] == '\r')) --n;
  auto eq = [&](const char* w, size_t k) {
    if (n != k) return false;
    for (size_t i = 0; i < k; ++i)
      if ((char)(p[i] | 0x20) != w[i]) return false;
    return true;
  };
  if (eq("false", 5)) return 0;
  if (eq("true", 4)) return 1;
  return 2;
}

Feed::Feed(std::string bootstrap, kafka::ClientConfig ccfg, std::vector<avro::Field> fields, FeedConfig cfg,
           std::vector<PartSpec> parts)
    : bootstrap_(std::move(bootstrap)), ccfg_(std::move(ccfg)), fields_(std::move(fields)), cfg_(std::move(cfg)) {
  if (cfg_.feature_fields.empty()) throw std::invalid_argument("feed: no feature fields");
  for (int f : cfg_.feature_fields)
    if (f < 0 || f >= (int)fields_.size() || !fields_[(size_t)f].is_numeric())
      throw std::invalid_argument("feed: feature field index must name a numeric schema field");
  if (cfg_.label_field >= (int)fields_.size() ||
      (cfg_.label_field >= 0 && fields_[(size_t)cfg_.label_field].kind != avro::K_STRING &&
       fields_[(size_t)cfg_.label_field].kind != avro::K_BYTES))
    throw std::invalid_argument("feed: label field must be a string / bytes schema field");
  col_of_.assign(fields_.size(), -1);
  for (size_t k = 0; k < cfg_.feature_fields.size(); ++k) col_of_[(size_t)cfg_.feature_fields[k]] = (int)k;
  if (cfg_.feature_fields.size() > 127) throw std::invalid_argument("feed: at most 127 features");
  for (size_t fi = 0; fi < fields_.size(); ++fi) {
    const avro::Field& f = fields_[fi];
    plan_.push_back(Op{(uint8_t)f.kind, (int8_t)f.null_branch, (int8_t)col_of_[fi],
                       (uint8_t)((int)fi == cfg_.label_field), f.fixed_size});
  }
  fast_ = true;
  for (const Op& op : plan_) {
    const bool num = op.kind == avro::K_FLOAT || op.kind == avro::K_INT || op.kind == avro::K_LONG ||
                     op.kind == avro::K_DOUBLE;
    if (op.null_branch > 1 || !(num || op.kind == avro::K_STRING || op.kind == avro::K_BYTES)) {
      fast_ = false;
      break;
    }
    const uint8_t k = op.kind == avro::K_LONG ? (uint8_t)avro::K_INT : op.kind;   // the same varint
    const int16_t vb = op.null_branch < 0 ? -1 : (int16_t)(2 * (1 - op.null_branch));   // zig-zag branch index
    if (!runs_.empty()) {
      Run& r = runs_.back();
      const bool same = r.kind == k && k != avro::K_STRING && k != avro::K_BYTES && !op.label && r.vb == vb &&
                        r.n < 255 && ((r.col < 0 && op.col < 0) || (r.col >= 0 && op.col == r.col + r.n));
      if (same) {
        ++r.n;
        continue;
      }
    }
    runs_.push_back(Run{k, 1, op.col, op.label, vb});
  }
  if (!fast_) runs_.clear();
  for (auto& s : parts) {
    auto p = std::make_unique<Part>();
    p->spec = s;
    p->pos = s.start;
    parts_.push_back(std::move(p));
  }
}

Feed::~Feed() { stop(); }

void Feed::start(const std::vector<uintptr_t>& slabs, int64_t cap_rows) {
  if (!workers_.empty()) throw std::logic_error("feed: already started");
  if (slabs.empty() || cap_rows <= 0) throw std::invalid_argument("feed: need slabs of > 0 rows");
  slabs_ = slabs;
  marks_.assign(slabs_.size(), {});
  cap_ = cap_rows;
  for (size_t i = 0; i < slabs_.size(); ++i) free_.push_back((int)i);
  const int nw = std::max(1, std::min(cfg_.workers, (int)parts_.size()));
  workers_.resize((size_t)nw);
  for (size_t i = 0; i < parts_.size(); ++i) workers_[i % (size_t)nw].parts.push_back((int)i);
  {
    std::lock_guard<std::mutex> g(mu_);
    live_workers_ = parts_.empty() ? 0 : nw;
  }
  if (parts_.empty()) return;
  for (int w = 0; w < nw; ++w) workers_[(size_t)w].th = std::thread([this, w] { run(w); });
}

void Feed::start_staged(const std::vector<uintptr_t>& slabs, int64_t cap_rows, const uint8_t* buf,
                        const int64_t* offs, int64_t n, int workers) {
  if (!workers_.empty()) throw std::logic_error("feed: already started");
  if (slabs.empty() || cap_rows <= 0) throw std::invalid_argument("feed: need slabs of > 0 rows");
  if (n < 0 || workers < 1) throw std::invalid_argument("feed: staged n >= 0, workers >= 1");
  slabs_ = slabs;
  marks_.assign(slabs_.size(), {});
  cap_ = cap_rows;
  for (size_t i = 0; i < slabs_.size(); ++i) free_.push_back((int)i);
  const int nw = (int)std::max<int64_t>(1, std::min<int64_t>(workers, std::max<int64_t>(n, 1)));
  workers_.resize((size_t)nw);
  {
    std::lock_guard<std::mutex> g(mu_);
    live_workers_ = nw;
  }
  for (int w = 0; w < nw; ++w) {
    const int64_t a = n * w / nw, b = n * (w + 1) / nw;
    workers_[(size_t)w].th = std::thread([this, w, buf, offs, a, b] { run_staged(w, buf, offs, a, b); });
  }
}

void Feed::run_staged(int w, const uint8_t* buf, const int64_t* offs, int64_t a, int64_t b) {
  const size_t F = cfg_.feature_fields.size();
  Stats loc;
  int slab = -1;
  int64_t n = 0;
  float* rows = nullptr;
  uint8_t* labs = nullptr;
  std::string err;
  try {
    const auto t1 = Clock::now();
    for (int64_t i = a; i < b; ++i) {
      if (slab < 0) {
        const auto tw = Clock::now();
        slab = take_free(loc.wait_slab_s);
        loc.decode_s -= secs(tw, Clock::now());   // the wait is not decode time
        if (slab < 0) break;   // stopping
        n = 0;
        rows = reinterpret_cast<float*>(slabs_[(size_t)slab]);
        labs = reinterpret_cast<uint8_t*>(slabs_[(size_t)slab]) + (size_t)cap_ * F * 4;
      }
      const size_t len = (size_t)(offs[i + 1] - offs[i]);
      ++loc.records;
      loc.bytes += len;
      float* row = rows + (size_t)n * F;
      uint8_t lab = cfg_.label_field >= 0 ? 2 : 0;
      if (!decode_row(buf + offs[i], len, row, &lab)) {
        ++loc.errors;
        for (size_t k = 0; k < F; ++k) row[k] = NAN;
        lab = 2;
      }
      if (cfg_.keep_label >= 0 && lab != (uint8_t)cfg_.keep_label) {
        ++loc.dropped;
        continue;
      }
      labs[n] = lab;
      ++n;
      ++loc.rows;
      if (n == cap_) {
        publish(w, slab, n);
        slab = -1;
      }
    }
    loc.decode_s += secs(t1, Clock::now());
  } catch (const std::exception& e) {
    err = e.what();
  }
  if (slab >= 0) {
    if (n > 0) {
      publish(w, slab, n);
    } else {
      std::lock_guard<std::mutex> g(mu_);
      free_.push_back(slab);
    }
  }
  {
    std::lock_guard<std::mutex> g(mu_);
    stats_.records += loc.records;
    stats_.rows += loc.rows;
    stats_.dropped += loc.dropped;
    stats_.errors += loc.errors;
    stats_.bytes += loc.bytes;
    stats_.decode_s += loc.decode_s;
    stats_.wait_slab_s += loc.wait_slab_s;
    if (!err.empty() && error_.empty()) error_ = "feed worker " + std::to_string(w) + ": " + err;
    --live_workers_;
  }
  cv_ready_.notify_all();
  cv_free_.notify_all();
}

void Feed::stop() {
  {
    std::lock_guard<std::mutex> g(mu_);
    stop_ = true;
  }
  cv_free_.notify_all();
  cv_ready_.notify_all();
  for (auto& w : workers_)
    if (w.th.joinable()) w.th.join();
}

int Feed::pop(int& slab, int64_t& rows, int timeout_ms) {
  std::unique_lock<std::mutex> g(mu_);
  auto ready = [&] { return !ready_.empty() || live_workers_ == 0 || !error_.empty(); };
  if (timeout_ms < 0) cv_ready_.wait(g, ready);
  else   // system_clock deadline (pthread_cond_timedwait; see kafka.cpp retention_loop)
    cv_ready_.wait_until(g, std::chrono::system_clock::now() + std::chrono::milliseconds(timeout_ms), ready);
  if (!error_.empty()) throw std::runtime_error(error_);
  if (!ready_.empty()) {
    slab = ready_.front().first;
    rows = ready_.front().second;
    ready_.pop_front();
    return 1;
  }
  return live_workers_ == 0 ? -1 : 0;
}

void Feed::recycle(int slab) {
  if (slab < 0 || slab >= (int)slabs_.size()) throw std::out_of_range("feed: bad slab");
  {
    std::lock_guard<std::mutex> g(mu_);
    free_.push_back(slab);
  }
  cv_free_.notify_one();
}

Stats Feed::stats() const {
  std::lock_guard<std::mutex> g(mu_);
  return stats_;
}

std::vector<int64_t> Feed::positions() const {
  std::vector<int64_t> out;
  for (const auto& p : parts_) out.push_back(p->pos.load());
  return out;
}

int Feed::take_free(double& waited) {
  const auto t0 = Clock::now();
  std::unique_lock<std::mutex> g(mu_);
  cv_free_.wait(g, [&] { return !free_.empty() || stop_; });
  waited += secs(t0, Clock::now());
  if (stop_) return -1;
  const int s = free_.front();
  free_.pop_front();
  return s;
}

std::vector<std::pair<int, int64_t>> Feed::slab_marks(int slab) const {
  if (slab < 0 || slab >= (int)slabs_.size()) throw std::out_of_range("feed: bad slab");
  std::lock_guard<std::mutex> g(mu_);
  return marks_[(size_t)slab];
}

void Feed::publish(int w, int slab, int64_t rows) {
  // labels were staged after the slab's `cap` rows; move them right behind the `rows` rows
  char* base = reinterpret_cast<char*>(slabs_[(size_t)slab]);
  const size_t F = cfg_.feature_fields.size();
  std::memmove(base + (size_t)rows * F * 4, base + (size_t)cap_ * F * 4, (size_t)rows);
  {
    std::lock_guard<std::mutex> g(mu_);
    auto& mk = marks_[(size_t)slab];
    mk.clear();
    for (int pi : workers_[(size_t)w].parts) mk.emplace_back(pi, parts_[(size_t)pi]->pos.load());
    ready_.emplace_back(slab, rows);
    ++stats_.slabs;
  }
  cv_ready_.notify_one();
}

int Feed::decode_fast(const uint8_t* p, size_t n, float* out_row, uint8_t* label) const {
  const uint8_t* e = p + n;
  if (cfg_.framing) {
    if (n < 5 || p[0] != 0) return -1;
    p += 5;
  }
  for (const Run& r : runs_) {
    const int u = r.vb >= 0 ? 1 : 0;   // union branch byte before each value
    switch (r.kind) {
      case avro::K_FLOAT:
      case avro::K_DOUBLE: {   // raw little-endian values (KSQL's DOUBLE columns narrowed)
        const int w = r.kind == avro::K_FLOAT ? 4 : 8, stride = u + w;
        if (e - p < (ptrdiff_t)stride * r.n) return -1;
        for (int k = 0; k < r.n; ++k, p += stride) {
          if (u && p[0] != (uint8_t)r.vb) return -1;
          float x;
          if (w == 4) {
            std::memcpy(&x, p + u, 4);
          } else {
            double v;
            std::memcpy(&v, p + u, 8);
            x = (float)v;
          }
          if (r.col >= 0) out_row[r.col + k] = x;
        }
        break;
      }
      case avro::K_INT: {      // zig-zag varints (int and long)
        for (int k = 0; k < r.n; ++k) {
          if (u) {
            if (p >= e || p[0] != (uint8_t)r.vb) return -1;
            ++p;
          }
          int64_t x;
          if (p < e && !(*p & 0x80)) {
            const uint8_t b = *p++;
            x = (int64_t)((b >> 1) ^ (~(b & 1) + 1));
          } else if (!varlong(p, e, x)) {
            return -1;
          }
          if (r.col >= 0) out_row[r.col + k] = (float)x;
        }
        break;
      }
      default: {               // string / bytes
        if (u) {
          if (p >= e || p[0] != (uint8_t)r.vb) return -1;
          ++p;
        }
        int64_t len;
        if (!varlong(p, e, len) || len < 0 || len > e - p) return -1;
        if (r.label) *label = label_code(p, (size_t)len);
        p += len;
      }
    }
  }
  return p == e ? 1 : -1;
}

double Feed::decode_throughput(const uint8_t* buf, const int64_t* offs, int64_t n, int workers, int repeats,
                               int64_t* rows_out) const {
  if (workers < 1 || n < 1) throw std::invalid_argument("decode_throughput: workers >= 1, n >= 1");
  const int F = features();
  double best = 0.0;
  for (int r = 0; r < repeats; ++r) {
    std::vector<int64_t> kept((size_t)workers, 0);
    std::vector<std::thread> th;
    const auto t0 = std::chrono::steady_clock::now();
    for (int w = 0; w < workers; ++w)
      th.emplace_back([&, w] {
        const int64_t a = n * w / workers, b = n * (w + 1) / workers;
        std::vector<float> slab((size_t)(b - a + 1) * (size_t)F);   // the worker's own slab, written row by row
        int64_t k = 0;
        uint8_t lab = 0;
        for (int64_t i = a; i < b; ++i)
          if (decode_row(buf + offs[i], (size_t)(offs[i + 1] - offs[i]), slab.data() + (size_t)k * F, &lab) &&
              (cfg_.keep_label < 0 || lab == cfg_.keep_label))
            ++k;
        kept[(size_t)w] = k;
      });
    for (auto& t : th) t.join();
    const double dt = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    int64_t tot = 0;
    for (int64_t k : kept) tot += k;
    if (rows_out) *rows_out = tot;
    best = std::max(best, (double)n / dt);
  }
  return best;
}

bool Feed::decode_row(const uint8_t* p, size_t n, float* out_row, uint8_t* label) const {
  if (fast_ && decode_fast(p, n, out_row, label) == 1) return true;
  const uint8_t* e = p + n;
  if (cfg_.framing) {
    if (n < 5 || p[0] != 0) return false;
    p += 5;
  }
  for (const Op& op : plan_) {
    bool is_null = op.kind == avro::K_NULL;
    if (op.null_branch >= 0) {
      // union branch index: 0 or 1, one zigzag byte (0x00 / 0x02)
      if (p >= e) return false;
      const uint8_t b = *p++;
      if (b != 0 && b != 2) return false;
      is_null = (b >> 1) == (uint8_t)op.null_branch;
    }
    if (is_null) {
      if (op.col >= 0) out_row[op.col] = NAN;
      if (op.label) *label = 2;
      continue;
    }
    switch (op.kind) {
      case avro::K_DOUBLE: {
        if (e - p < 8) return false;
        double v;
        std::memcpy(&v, p, 8);
        p += 8;
        if (op.col >= 0) out_row[op.col] = (float)v;
        break;
      }
      case avro::K_INT:
      case avro::K_LONG: {
        int64_t x;
        if (p < e && !(*p & 0x80)) {   // one-byte varint fast path
          const uint8_t b = *p++;
          x = (int64_t)((b >> 1) ^ (~(b & 1) + 1));
        } else if (!varlong(p, e, x)) {
          return false;
        }
        if (op.col >= 0) out_row[op.col] = (float)x;
        break;
      }
      case avro::K_FLOAT: {
        if (e - p < 4) return false;
        float x;
        std::memcpy(&x, p, 4);
        p += 4;
        if (op.col >= 0) out_row[op.col] = x;
        break;
      }
      case avro::K_BOOLEAN:
        if (p >= e) return false;
        if (op.col >= 0) out_row[op.col] = *p ? 1.f : 0.f;
        ++p;
        break;
      case avro::K_STRING:
      case avro::K_BYTES: {
        int64_t len;
        if (!varlong(p, e, len) || len < 0 || len > e - p) return false;
        if (op.label) *label = label_code(p, (size_t)len);
        p += len;
        break;
      }
      case avro::K_FIXED:
        if (e - p < op.fixed) return false;
        p += op.fixed;
        break;
      case avro::K_ENUM: {
        int64_t idx;
        if (!varlong(p, e, idx) || idx < 0) return false;
        break;
      }
      default:
        return false;
    }
  }
  return p == e;
}

void Feed::run(int w) {
  const std::vector<int>& mine = workers_[(size_t)w].parts;
  const size_t F = cfg_.feature_fields.size();
  struct PState {
    std::string resp;
    kafka::RecordSetCursor cur;
    bool have = false;
  };
  std::vector<PState> st(mine.size());
  Stats loc;
  int slab = -1;
  int64_t n = 0;
  float* rows = nullptr;
  uint8_t* labs = nullptr;
  auto last_data = Clock::now();
  size_t rr = 0;
  std::string err;
  auto flush_stats = [&] {
    std::lock_guard<std::mutex> g(mu_);
    stats_.records += loc.records;
    stats_.rows += loc.rows;
    stats_.dropped += loc.dropped;
    stats_.errors += loc.errors;
    stats_.bytes += loc.bytes;
    stats_.fetches += loc.fetches;
    stats_.fetch_s += loc.fetch_s;
    stats_.decode_s += loc.decode_s;
    stats_.reset_skipped += loc.reset_skipped;
    stats_.wait_slab_s += loc.wait_slab_s;
    loc = Stats();
  };
  std::unique_ptr<kafka::Client> cl;
  // long-poll policy (as scoreloop.cpp): a worker that owns several partitions fetches with
  // wait 0 while any of them made progress in the last round; only after an empty round does
  // it long-poll, and then on one partition, so an idle partition never stalls busy ones
  bool prev_progress = true;
  try {
    cl = std::make_unique<kafka::Client>(bootstrap_, ccfg_);   // one broker connection per worker
    for (;;) {
      {
        std::lock_guard<std::mutex> g(mu_);
        if (stop_) break;
      }
      bool all_done = true, progressed = false;
      for (size_t q = 0; q < mine.size(); ++q) {
        const size_t qi = (rr + q) % mine.size();
        Part& P = *parts_[(size_t)mine[qi]];
        if (P.done) continue;
        all_done = false;
        PState& S = st[qi];
        if (!S.have) {
          const int64_t pos = P.pos.load();
          if (P.spec.end >= 0 && pos >= P.spec.end) {
            P.done = true;
            continue;
          }
          const auto t0 = Clock::now();
          size_t off = 0, len = 0;
          const int wait = (mine.size() == 1 || (!prev_progress && q == 0)) ? cfg_.max_wait_ms : 0;
          try {
            cl->fetch_raw(P.spec.topic, P.spec.partition, pos, cfg_.max_bytes, wait, S.resp, off, len);
          } catch (const kafka::Error& e) {
            if (e.code != 1 || cfg_.offset_reset == 2) throw;   // 1: OFFSET_OUT_OF_RANGE
            int64_t np = cl->list_offset(P.spec.topic, P.spec.partition, cfg_.offset_reset == 1 ? -1 : -2);
            if (P.spec.end >= 0) np = std::min(np, P.spec.end);
            if (np > pos) loc.reset_skipped += (uint64_t)(np - pos);
            P.pos.store(np, std::memory_order_relaxed);
            continue;
          }
          loc.fetch_s += secs(t0, Clock::now());
          ++loc.fetches;
          if (len == 0) continue;
          loc.bytes += len;
          S.cur = kafka::RecordSetCursor(reinterpret_cast<const uint8_t*>(S.resp.data()) + off, len, cfg_.check_crcs);
          S.have = true;
        }
        const auto t1 = Clock::now();
        kafka::RecordView v;
        for (;;) {
          if (slab < 0) {
            slab = take_free(loc.wait_slab_s);
            if (slab < 0) goto out;   // stopping
            n = 0;
            rows = reinterpret_cast<float*>(slabs_[(size_t)slab]);
            labs = reinterpret_cast<uint8_t*>(slabs_[(size_t)slab]) + (size_t)cap_ * F * 4;
          }
          if (!S.cur.next(v)) {
            S.have = false;
            break;
          }
          // pos is written only by this worker: relaxed per record (a seq_cst store is a locked
          // xchg on x86, ~20 cycles a record); publish() takes the feed mutex, which orders it
          if (v.offset < P.pos.load(std::memory_order_relaxed)) continue;
          if (P.spec.end >= 0 && v.offset >= P.spec.end) {
            S.have = false;
            P.done = true;
            break;
          }
          P.pos.store(v.offset + 1, std::memory_order_relaxed);
          ++loc.records;
          float* row = rows + (size_t)n * F;
          uint8_t lab = cfg_.label_field >= 0 ? 2 : 0;
          if (!decode_row(v.value, (size_t)v.value_len, row, &lab)) {
            ++loc.errors;
            for (size_t k = 0; k < F; ++k) row[k] = NAN;
            lab = 2;
          }
          if (cfg_.keep_label >= 0 && lab != (uint8_t)cfg_.keep_label) {
            ++loc.dropped;
            continue;
          }
          labs[n] = lab;
          ++n;
          ++loc.rows;
          progressed = true;
          if (n == cap_) {
            publish(w, slab, n);
            slab = -1;
            flush_stats();
          }
        }
        loc.decode_s += secs(t1, Clock::now());
      }
      ++rr;
      prev_progress = progressed;
      if (all_done) break;
      if (progressed) {
        last_data = Clock::now();
      } else {
        // nothing new on any of this worker's partitions (a followed, unbounded log):
        // hand over what is buffered, and give up after the idle timeout
        if (slab >= 0 && n > 0) {
          publish(w, slab, n);
          slab = -1;
        }
        if (cfg_.idle_timeout_s >= 0 && secs(last_data, Clock::now()) > cfg_.idle_timeout_s) break;
      }
    }
  } catch (const std::exception& e) {
    err = e.what();
  }
out:
  if (slab >= 0) {
    if (n > 0) {
      publish(w, slab, n);
    } else {
      std::lock_guard<std::mutex> g(mu_);
      free_.push_back(slab);
    }
  }
  flush_stats();
  {
    std::lock_guard<std::mutex> g(mu_);
    if (!err.empty() && error_.empty()) error_ = "feed worker " + std::to_string(w) + ": " + err;
    --live_workers_;
  }
  cv_ready_.notify_all();
  cv_free_.notify_all();
}

}  // namespace feed
}  // namespace sml
