// Kafka wire protocol client + in-process broker (see kafka.h).
#include "kafka.h"

#include <pthread.h>
#include <sched.h>

#include <arpa/inet.h>
#include <netdb.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <sys/socket.h>
#include <sys/uio.h>
#include <unistd.h>

#include <algorithm>
#include <cerrno>
#include <chrono>
#include <cstring>
#include <sstream>

#include "avro.h"  // zigzag varints

namespace sml {
namespace kafka {

// ---------------------------------------------------------------------------
// CRC-32C (Castagnoli), table driven
// ---------------------------------------------------------------------------
namespace {
struct Crc32cTable {
  uint32_t t[256];
  Crc32cTable() {
    for (uint32_t i = 0; i < 256; ++i) {
      uint32_t c = i;
      for (int k = 0; k < 8; ++k) c = (c & 1) ? (c >> 1) ^ 0x82F63B78u : (c >> 1);
      t[i] = c;
    }
  }
};
const Crc32cTable kCrc;

uint32_t crc32c_table(const uint8_t* p, size_t n, uint32_t crc) {
  crc = ~crc;
  for (size_t i = 0; i < n; ++i) crc = kCrc.t[(crc ^ p[i]) & 0xff] ^ (crc >> 8);
  return ~crc;
}

#if defined(__x86_64__)
// SSE4.2 crc32 instruction (CRC-32C polynomial): 8 bytes per instruction instead of
// one table lookup per byte.  Every record batch is checksummed twice (producer /
// broker encode, consumer verify), so on the ingest path this is the hot loop.
__attribute__((target("sse4.2"))) uint32_t crc32c_hw(const uint8_t* p, size_t n, uint32_t crc) {
  uint64_t c = ~crc & 0xffffffffu;
  while (n >= 8) {
    uint64_t v;
    std::memcpy(&v, p, 8);
    c = __builtin_ia32_crc32di(c, v);
    p += 8;
    n -= 8;
  }
  uint32_t c32 = (uint32_t)c;
  while (n--) c32 = __builtin_ia32_crc32qi(c32, *p++);
  return ~c32;
}
#endif
}  // namespace

uint32_t crc32c(const uint8_t* p, size_t n, uint32_t crc) {
#if defined(__x86_64__)
  static const bool hw = __builtin_cpu_supports("sse4.2");
  if (hw) return crc32c_hw(p, n, crc);
#endif
  return crc32c_table(p, n, crc);
}


// ---------------------------------------------------------------------------
// big-endian writer / reader
// ---------------------------------------------------------------------------
namespace {
struct W {
  std::string s;
  void i8(int8_t v) { s.push_back((char)v); }
  void i16(int16_t v) { u(v, 2); }
  void i32(int32_t v) { u(v, 4); }
  void i64(int64_t v) { u(v, 8); }
  void u(uint64_t v, int n) {
    for (int i = n - 1; i >= 0; --i) s.push_back((char)((v >> (8 * i)) & 0xff));
  }
  void str(const std::string& v) {
    i16((int16_t)v.size());
    s += v;
  }
  void nullstr() { i16(-1); }
  void bytes(const std::string& v) {
    i32((int32_t)v.size());
    s += v;
  }
  void arr(int32_t n) { i32(n); }
  size_t pos() const { return s.size(); }
  void put32(size_t at, int32_t v) {
    for (int i = 3; i >= 0; --i) s[at + 3 - i] = (char)((v >> (8 * i)) & 0xff);
  }
};

struct R {
  const uint8_t* p;
  size_t n;
  size_t i = 0;
  void need(size_t k) const {
    if (k > n - i) throw Error("kafka: truncated message");
  }
  uint64_t u(int k) {
    need((size_t)k);
    uint64_t v = 0;
    for (int j = 0; j < k; ++j) v = (v << 8) | p[i + j];
    i += (size_t)k;
    return v;
  }
  int8_t i8() { return (int8_t)u(1); }
  int16_t i16() { return (int16_t)u(2); }
  int32_t i32() { return (int32_t)u(4); }
  int64_t i64() { return (int64_t)u(8); }
  std::string str() {
    const int16_t len = i16();
    if (len < 0) return std::string();
    need((size_t)len);
    std::string v(reinterpret_cast<const char*>(p + i), (size_t)len);
    i += (size_t)len;
    return v;
  }
  // returns pointer + length of a BYTES field (length -1 => null => n = 0)
  std::pair<const uint8_t*, size_t> bytes() {
    const int32_t len = i32();
    if (len < 0) return {nullptr, 0};
    need((size_t)len);
    auto r = std::make_pair(p + i, (size_t)len);
    i += (size_t)len;
    return r;
  }
  int32_t arr() {
    const int32_t n_ = i32();
    if (n_ > (int32_t)(n - i)) throw Error("kafka: implausible array length");
    return n_;
  }
  int64_t varlong() {   // zigzag varint, inline (hot in the record-set walk)
    uint64_t v = 0;
    for (int shift = 0; shift < 70 && i < n; shift += 7) {
      const uint8_t b = p[i++];
      v |= (uint64_t)(b & 0x7f) << shift;
      if (!(b & 0x80)) return (int64_t)((v >> 1) ^ (~(v & 1) + 1));
    }
    throw Error("kafka: bad varint");
  }
};

void vl(std::string& s, int64_t v) { avro::write_varlong(s, v); }

enum Api : int16_t {
  API_PRODUCE = 0, API_FETCH = 1, API_LIST_OFFSETS = 2, API_METADATA = 3, API_OFFSET_COMMIT = 8,
  API_OFFSET_FETCH = 9, API_FIND_COORDINATOR = 10, API_SASL_HANDSHAKE = 17, API_API_VERSIONS = 18,
  API_SASL_AUTH = 36,
};
enum Err : int16_t {
  E_NONE = 0, E_OFFSET_OUT_OF_RANGE = 1, E_UNKNOWN_TOPIC = 3, E_NOT_LEADER = 6, E_MESSAGE_TOO_LARGE = 10,
  E_ILLEGAL_SASL_STATE = 34, E_UNSUPPORTED_SASL = 33, E_SASL_AUTH_FAILED = 58,
};
}  // namespace

// ---------------------------------------------------------------------------
// record batch v2
// ---------------------------------------------------------------------------
namespace {
// largest record batch (baseOffset + batchLength + batchLength bytes) of a record set
int64_t max_batch_size(const uint8_t* p, size_t n) {
  int64_t best = 0;
  size_t o = 0;
  while (o + 12 <= n) {
    const int32_t len = (int32_t)((uint32_t)p[o + 8] << 24 | (uint32_t)p[o + 9] << 16 | (uint32_t)p[o + 10] << 8 |
                                  (uint32_t)p[o + 11]);
    if (len < 0) break;
    best = std::max<int64_t>(best, 12 + (int64_t)len);
    o += 12 + (size_t)len;
  }
  return best;
}
}  // namespace
std::string encode_record_batch(int64_t base_offset, const std::vector<Record>& recs) {
  return encode_record_batch(base_offset, recs.data(), recs.size());
}

std::string encode_record_set(const std::vector<Record>& recs, size_t max_batch_bytes) {
  // a producer's record set: consecutive batches, each under the broker's message.max.bytes
  std::string out;
  size_t k = 0;
  while (k < recs.size()) {
    size_t bytes = 0, m = 0;
    while (k + m < recs.size()) {
      const size_t rb = recs[k + m].value.size() + recs[k + m].key.size() + 32;   // + varint framing
      if (m > 0 && bytes + rb > max_batch_bytes) break;
      bytes += rb;
      ++m;
    }
    out += encode_record_batch(0, recs.data() + k, m);
    k += m;
  }
  return out;
}

std::string encode_record_batch(int64_t base_offset, const Record* recs, size_t n) {
  if (n == 0) return std::string();
  const int64_t first_ts = recs[0].timestamp;
  int64_t max_ts = first_ts;
  std::string body;  // from attributes to the end (CRC scope)
  W h;
  h.i16(0);                                   // attributes: no compression
  h.i32((int32_t)(n - 1));                    // lastOffsetDelta
  h.i64(first_ts);
  for (size_t k = 0; k < n; ++k) max_ts = std::max(max_ts, recs[k].timestamp);
  h.i64(max_ts);
  h.i64(-1);                                  // producerId
  h.i16(-1);                                  // producerEpoch
  h.i32(-1);                                  // baseSequence
  h.i32((int32_t)n);
  body = h.s;
  for (size_t k = 0; k < n; ++k) {
    const Record& r = recs[k];
    std::string rec;
    rec.push_back(0);                         // attributes
    vl(rec, r.timestamp - first_ts);
    vl(rec, (int64_t)k);
    if (r.key_null) vl(rec, -1);
    else { vl(rec, (int64_t)r.key.size()); rec += r.key; }
    vl(rec, (int64_t)r.value.size());
    rec += r.value;
    vl(rec, 0);                               // headers
    vl(body, (int64_t)rec.size());
    body += rec;
  }
  const uint32_t crc = crc32c(reinterpret_cast<const uint8_t*>(body.data()), body.size());
  W b;
  b.i64(base_offset);
  b.i32((int32_t)(4 + 1 + 4 + body.size()));  // batchLength: epoch + magic + crc + body
  b.i32(0);                                   // partitionLeaderEpoch
  b.i8(2);                                    // magic
  b.u(crc, 4);
  b.s += body;
  return b.s;
}

void decode_record_batches(const uint8_t* p, size_t n, int64_t min_offset, FetchResult& out) {
  size_t pos = 0;
  while (n - pos >= 12) {
    R hdr{p + pos, n - pos};
    const int64_t base = hdr.i64();
    const int32_t blen = hdr.i32();
    if (blen < 0 || (size_t)blen > n - pos - 12) break;  // partial trailing batch
    R b{p + pos + 12, (size_t)blen};
    b.i32();  // leader epoch
    const int8_t magic = b.i8();
    if (magic != 2) throw Error("kafka: unsupported record batch magic " + std::to_string(magic));
    const uint32_t crc = (uint32_t)b.u(4);
    const uint32_t calc = crc32c(p + pos + 12 + b.i, (size_t)blen - b.i);
    if (crc != calc) throw Error("kafka: record batch CRC mismatch");
    const int16_t attrs = b.i16();
    if (attrs & 0x7) throw Error("kafka: compressed record batches are not supported");
    b.i32();                     // lastOffsetDelta
    const int64_t first_ts = b.i64();
    b.i64();                     // max ts
    b.i64();
    b.i16();
    b.i32();
    const int32_t count = b.i32();
    const bool control = attrs & 0x20;
    for (int32_t k = 0; k < count; ++k) {
      const int64_t len = b.varlong();
      if (len < 0 || (size_t)len > b.n - b.i) throw Error("kafka: bad record length");
      R r{b.p + b.i, (size_t)len};
      b.i += (size_t)len;
      r.i8();
      const int64_t ts_delta = r.varlong();
      const int64_t off_delta = r.varlong();
      const int64_t klen = r.varlong();
      std::string key;
      if (klen >= 0) {
        r.need((size_t)klen);
        key.assign(reinterpret_cast<const char*>(r.p + r.i), (size_t)klen);
        r.i += (size_t)klen;
      }
      const int64_t vlen = r.varlong();
      const int64_t off = base + off_delta;
      if (control || off < min_offset) {
        if (vlen > 0) r.i += (size_t)vlen;
        continue;
      }
      if (vlen > 0) {
        r.need((size_t)vlen);
        out.values.append(reinterpret_cast<const char*>(r.p + r.i), (size_t)vlen);
        r.i += (size_t)vlen;
      }
      out.value_offsets.push_back((int64_t)out.values.size());
      out.offsets.push_back(off);
      out.timestamps.push_back(first_ts + ts_delta);
      out.keys.push_back(std::move(key));
    }
    pos += 12 + (size_t)blen;
  }
}

bool RecordSetCursor::next(RecordView& out) {
  for (;;) {
    while (left_ > 0) {
      --left_;
      R b{bp_, bn_};
      b.i = bi_;
      const int64_t len = b.varlong();
      if (len < 0 || (size_t)len > b.n - b.i) throw Error("kafka: bad record length");
      R r{b.p + b.i, (size_t)len};
      bi_ = b.i + (size_t)len;
      r.i8();
      const int64_t ts_delta = r.varlong();
      const int64_t off_delta = r.varlong();
      const int64_t klen = r.varlong();
      const uint8_t* key = nullptr;
      if (klen >= 0) {
        r.need((size_t)klen);
        key = r.p + r.i;
        r.i += (size_t)klen;
      }
      const int64_t vlen = r.varlong();
      if (vlen > 0) r.need((size_t)vlen);
      if (control_) continue;
      out.offset = base_ + off_delta;
      out.timestamp = first_ts_ + ts_delta;
      out.key = key;
      out.key_len = klen;
      out.value = r.p + r.i;
      out.value_len = vlen > 0 ? vlen : 0;
      return true;
    }
    if (n_ - pos_ < 12) return false;
    R hdr{p_ + pos_, n_ - pos_};
    base_ = hdr.i64();
    const int32_t blen = hdr.i32();
    if (blen < 0 || (size_t)blen > n_ - pos_ - 12) return false;  // partial trailing batch
    R b{p_ + pos_ + 12, (size_t)blen};
    b.i32();  // leader epoch
    const int8_t magic = b.i8();
    if (magic != 2) throw Error("kafka: unsupported record batch magic " + std::to_string(magic));
    const uint32_t crc = (uint32_t)b.u(4);
    if (crc_ && crc != crc32c(p_ + pos_ + 12 + b.i, (size_t)blen - b.i)) throw Error("kafka: record batch CRC mismatch");
    const int16_t attrs = b.i16();
    if (attrs & 0x7) throw Error("kafka: compressed record batches are not supported");
    b.i32();
    first_ts_ = b.i64();
    b.i64();
    b.i64();
    b.i16();
    b.i32();
    left_ = b.i32();
    control_ = attrs & 0x20;
    bp_ = b.p;
    bn_ = b.n;
    bi_ = b.i;
    pos_ += 12 + (size_t)blen;
  }
}

// ---------------------------------------------------------------------------
// connection
// ---------------------------------------------------------------------------
class Connection {
 public:
  Connection(const std::string& host, int port, int timeout_ms) {
    addrinfo hints{};
    hints.ai_family = AF_INET;
    hints.ai_socktype = SOCK_STREAM;
    addrinfo* res = nullptr;
    const std::string ps = std::to_string(port);
    if (getaddrinfo(host.c_str(), ps.c_str(), &hints, &res) != 0 || !res)
      throw Error("kafka: cannot resolve " + host);
    fd_ = ::socket(res->ai_family, res->ai_socktype, res->ai_protocol);
    if (fd_ < 0) {
      freeaddrinfo(res);
      throw Error("kafka: socket() failed");
    }
    timeval tv{timeout_ms / 1000, (timeout_ms % 1000) * 1000};
    setsockopt(fd_, SOL_SOCKET, SO_RCVTIMEO, &tv, sizeof(tv));
    setsockopt(fd_, SOL_SOCKET, SO_SNDTIMEO, &tv, sizeof(tv));
    int one = 1;
    setsockopt(fd_, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
    int sz = 4 << 20;   // multi-megabyte fetch responses in few recv() calls
    setsockopt(fd_, SOL_SOCKET, SO_RCVBUF, &sz, sizeof(sz));
    const int rc = ::connect(fd_, res->ai_addr, res->ai_addrlen);
    freeaddrinfo(res);
    if (rc != 0) {
      ::close(fd_);
      fd_ = -1;
      throw Error("kafka: connect to " + host + ":" + ps + " failed");
    }
  }
  ~Connection() {
    if (fd_ >= 0) ::close(fd_);
  }
  void send_all(const std::string& s) {
    size_t off = 0;
    while (off < s.size()) {
      const ssize_t k = ::send(fd_, s.data() + off, s.size() - off, MSG_NOSIGNAL);
      if (k <= 0) throw Error("kafka: send failed");
      off += (size_t)k;
    }
  }
  void recv_all(char* p, size_t n) {
    size_t off = 0;
    if (spin_us_ > 0) {   // busy-poll first: the response usually lands within microseconds
      const auto t_end = std::chrono::steady_clock::now() + std::chrono::microseconds(spin_us_);
      while (off < n) {
        const ssize_t k = ::recv(fd_, p + off, n - off, MSG_DONTWAIT);
        if (k > 0) {
          off += (size_t)k;
          continue;
        }
        if (k == 0) throw Error("kafka: connection closed");
        if (errno != EAGAIN && errno != EWOULDBLOCK && errno != EINTR) throw Error("kafka: recv failed");
        if (std::chrono::steady_clock::now() >= t_end) break;
#if defined(__x86_64__)
        __builtin_ia32_pause();
#endif
      }
    }
    while (off < n) {
      const ssize_t k = ::recv(fd_, p + off, n - off, 0);
      if (k <= 0) throw Error("kafka: connection closed / timed out");
      off += (size_t)k;
    }
  }
  void set_spin_us(int us) { spin_us_ = us; }
  bool authed = false;

 private:
  int fd_ = -1;
  int spin_us_ = 0;
};

// ---------------------------------------------------------------------------
// client
// ---------------------------------------------------------------------------
Client::Client(const std::string& bootstrap, ClientConfig cfg) : cfg_(std::move(cfg)) {
  std::stringstream ss(bootstrap);
  std::string item;
  while (std::getline(ss, item, ',')) {
    if (item.empty()) continue;
    const auto c = item.rfind(':');
    if (c == std::string::npos) throw Error("kafka: bootstrap server needs host:port: " + item);
    bootstrap_.push_back({item.substr(0, c), std::stoi(item.substr(c + 1))});
  }
  if (bootstrap_.empty()) throw Error("kafka: no bootstrap servers");
}

Client::~Client() = default;

std::unique_ptr<Connection> Client::open(const BrokerAddr& a) {
  auto c = std::make_unique<Connection>(a.host, a.port, cfg_.timeout_ms);
  c->set_spin_us(cfg_.spin_us);
  if (!cfg_.sasl_mechanism.empty()) {
    W hs;
    hs.str(cfg_.sasl_mechanism);
    std::string resp = call(*c, API_SASL_HANDSHAKE, 1, hs.s);
    R r{reinterpret_cast<const uint8_t*>(resp.data()), resp.size()};
    const int16_t ec = r.i16();
    if (ec != E_NONE) throw Error("kafka: SASL handshake rejected", ec);
    std::string tok;
    tok.push_back('\0');
    tok += cfg_.sasl_username;
    tok.push_back('\0');
    tok += cfg_.sasl_password;
    W au;
    au.bytes(tok);
    resp = call(*c, API_SASL_AUTH, 0, au.s);
    R ra{reinterpret_cast<const uint8_t*>(resp.data()), resp.size()};
    const int16_t ec2 = ra.i16();
    if (ec2 != E_NONE) throw Error("kafka: SASL/PLAIN authentication failed", ec2);
    c->authed = true;
  }
  return c;
}

std::string Client::call(Connection& c, int16_t api, int16_t ver, const std::string& body) {
  W w;
  w.i32(0);  // size placeholder
  w.i16(api);
  w.i16(ver);
  const int32_t corr = corr_++;
  w.i32(corr);
  w.str(cfg_.client_id);
  w.s += body;
  w.put32(0, (int32_t)(w.s.size() - 4));
  c.send_all(w.s);
  char hdr[8];
  c.recv_all(hdr, 8);
  const int32_t size = (int32_t)(((uint32_t)(uint8_t)hdr[0] << 24) | ((uint32_t)(uint8_t)hdr[1] << 16) |
                                 ((uint32_t)(uint8_t)hdr[2] << 8) | (uint8_t)hdr[3]);
  const int32_t rcorr = (int32_t)(((uint32_t)(uint8_t)hdr[4] << 24) | ((uint32_t)(uint8_t)hdr[5] << 16) |
                                  ((uint32_t)(uint8_t)hdr[6] << 8) | (uint8_t)hdr[7]);
  if (size < 4 || size > (1 << 30)) throw Error("kafka: bad response size");
  if (rcorr != corr) throw Error("kafka: correlation id mismatch");
  std::string resp((size_t)size - 4, '\0');
  if (!resp.empty()) c.recv_all(&resp[0], resp.size());
  bytes_rx_ += (uint64_t)size + 4;
  return resp;
}

size_t Client::call_into(Connection& c, int16_t api, int16_t ver, const std::string& body, std::string& resp) {
  W w;
  w.i32(0);
  w.i16(api);
  w.i16(ver);
  const int32_t corr = corr_++;
  w.i32(corr);
  w.str(cfg_.client_id);
  w.s += body;
  w.put32(0, (int32_t)(w.s.size() - 4));
  c.send_all(w.s);
  char hdr[8];
  c.recv_all(hdr, 8);
  const int32_t size = (int32_t)(((uint32_t)(uint8_t)hdr[0] << 24) | ((uint32_t)(uint8_t)hdr[1] << 16) |
                                 ((uint32_t)(uint8_t)hdr[2] << 8) | (uint8_t)hdr[3]);
  const int32_t rcorr = (int32_t)(((uint32_t)(uint8_t)hdr[4] << 24) | ((uint32_t)(uint8_t)hdr[5] << 16) |
                                  ((uint32_t)(uint8_t)hdr[6] << 8) | (uint8_t)hdr[7]);
  if (size < 4 || size > (1 << 30)) throw Error("kafka: bad response size");
  if (rcorr != corr) throw Error("kafka: correlation id mismatch");
  const size_t n = (size_t)size - 4;
  if (resp.size() < n) resp.resize(n + n / 4);
  if (n) c.recv_all(&resp[0], n);
  bytes_rx_ += (uint64_t)size + 4;
  return n;
}

Connection& Client::any_conn() {
  if (!any_) {
    std::string last;
    for (const auto& b : bootstrap_) {
      try {
        any_ = open(b);
        break;
      } catch (const Error& e) {
        last = e.what();
      }
    }
    if (!any_) throw Error("kafka: no bootstrap server reachable: " + last);
  }
  return *any_;
}

void Client::refresh_metadata(const std::string& topic) {
  W w;
  if (topic.empty()) {
    w.arr(-1);  // all topics
  } else {
    w.arr(1);
    w.str(topic);
  }
  const std::string resp = call(any_conn(), API_METADATA, 1, w.s);
  R r{reinterpret_cast<const uint8_t*>(resp.data()), resp.size()};
  brokers_.clear();
  if (topic.empty()) leaders_.clear();
  for (int32_t nb = r.arr(), i = 0; i < nb; ++i) {
    const int32_t id = r.i32();
    std::string host = r.str();
    const int32_t port = r.i32();
    r.str();  // rack
    brokers_[id] = {host, port};
  }
  r.i32();  // controller
  for (int32_t nt = r.arr(), i = 0; i < nt; ++i) {
    const int16_t terr = r.i16();
    const std::string name = r.str();
    r.i8();
    std::vector<int32_t> lead;
    for (int32_t np = r.arr(), k = 0; k < np; ++k) {
      r.i16();
      const int32_t pid = r.i32();
      const int32_t leader = r.i32();
      for (int32_t x = r.arr(), q = 0; q < x; ++q) r.i32();
      for (int32_t x = r.arr(), q = 0; q < x; ++q) r.i32();
      if ((int32_t)lead.size() <= pid) lead.resize((size_t)pid + 1, -1);
      lead[(size_t)pid] = leader;
    }
    if (terr == E_NONE && !lead.empty()) leaders_[name] = lead;
  }
  conns_.clear();
}

std::map<std::string, int> Client::partitions() {
  std::lock_guard<std::mutex> g(mu_);
  refresh_metadata();
  std::map<std::string, int> out;
  for (const auto& kv : leaders_) out[kv.first] = (int)kv.second.size();
  return out;
}

Connection& Client::conn_for(const std::string& topic, int partition) {
  auto it = leaders_.find(topic);
  if (it == leaders_.end() || partition >= (int)it->second.size()) {
    // a named Metadata request auto-creates the topic on brokers that allow it; a
    // freshly created topic may report LEADER_NOT_AVAILABLE once, so ask twice.
    for (int attempt = 0; attempt < 3; ++attempt) {
      refresh_metadata(topic);
      it = leaders_.find(topic);
      if (it != leaders_.end()) break;
      std::this_thread::sleep_for(std::chrono::milliseconds(50 * (attempt + 1)));
    }
    if (it == leaders_.end()) throw Error("kafka: unknown topic " + topic, E_UNKNOWN_TOPIC);
    if (partition >= (int)it->second.size()) throw Error("kafka: unknown partition", E_UNKNOWN_TOPIC);
  }
  const int32_t leader = it->second[(size_t)partition];
  auto ct = conns_.find(leader);
  if (ct == conns_.end()) {
    auto bt = brokers_.find(leader);
    if (bt == brokers_.end()) throw Error("kafka: leader not in metadata", E_NOT_LEADER);
    ct = conns_.emplace(leader, open({bt->second.host, bt->second.port})).first;
  }
  return *ct->second;
}

int64_t Client::list_offset(const std::string& topic, int partition, int64_t time) {
  std::lock_guard<std::mutex> g(mu_);
  W w;
  w.i32(-1);
  w.arr(1);
  w.str(topic);
  w.arr(1);
  w.i32(partition);
  w.i64(time);
  const std::string resp = call(conn_for(topic, partition), API_LIST_OFFSETS, 1, w.s);
  R r{reinterpret_cast<const uint8_t*>(resp.data()), resp.size()};
  r.arr();
  r.str();
  r.arr();
  r.i32();
  const int16_t ec = r.i16();
  if (ec != E_NONE) throw Error("kafka: ListOffsets error " + std::to_string(ec), ec);
  r.i64();
  return r.i64();
}

FetchResult Client::fetch(const std::string& topic, int partition, int64_t offset, int32_t max_bytes,
                          int32_t max_wait_ms) {
  std::lock_guard<std::mutex> g(mu_);
  for (int attempt = 0;; ++attempt) {
    W w;
    w.i32(-1);          // replica id
    w.i32(max_wait_ms);
    w.i32(1);           // min bytes
    w.i32(max_bytes);
    w.i8(0);            // read uncommitted
    w.arr(1);
    w.str(topic);
    w.arr(1);
    w.i32(partition);
    w.i64(offset);
    w.i32(max_bytes);
    FetchResult out;
    std::string resp;
    try {
      resp = call(conn_for(topic, partition), API_FETCH, 4, w.s);
    } catch (const Error& e) {
      if (attempt >= cfg_.max_retries) throw;
      conns_.clear();
      any_.reset();
      refresh_metadata();
      continue;
    }
    R r{reinterpret_cast<const uint8_t*>(resp.data()), resp.size()};
    r.i32();  // throttle
    r.arr();
    r.str();
    r.arr();
    r.i32();
    const int16_t ec = r.i16();
    out.high_watermark = r.i64();
    r.i64();  // last stable
    const int32_t naborted = r.i32();
    for (int32_t k = 0; k < naborted; ++k) {
      r.i64();
      r.i64();
    }
    auto rec = r.bytes();
    out.error_code = ec;
    if (ec == E_NOT_LEADER && attempt < cfg_.max_retries) {  // leadership moved: refresh and retry
      refresh_metadata();
      continue;
    }
    if (ec != E_NONE) throw Error("kafka: Fetch error " + std::to_string(ec), ec);
    if (rec.first) decode_record_batches(rec.first, rec.second, offset, out);
    return out;
  }
}

int64_t Client::fetch_raw(const std::string& topic, int partition, int64_t offset, int32_t max_bytes,
                          int32_t max_wait_ms, std::string& resp, size_t& rec_off, size_t& rec_len) {
  std::lock_guard<std::mutex> g(mu_);
  for (int attempt = 0;; ++attempt) {
    W w;
    w.i32(-1);
    w.i32(max_wait_ms);
    w.i32(1);
    w.i32(max_bytes);
    w.i8(0);
    w.arr(1);
    w.str(topic);
    w.arr(1);
    w.i32(partition);
    w.i64(offset);
    w.i32(max_bytes);
    size_t used = 0;
    try {
      used = call_into(conn_for(topic, partition), API_FETCH, 4, w.s, resp);
    } catch (const Error& e) {
      if (attempt >= cfg_.max_retries) throw;
      conns_.clear();
      any_.reset();
      refresh_metadata();
      continue;
    }
    R r{reinterpret_cast<const uint8_t*>(resp.data()), used};
    r.i32();
    r.arr();
    r.str();
    r.arr();
    r.i32();
    const int16_t ec = r.i16();
    const int64_t hwm = r.i64();
    r.i64();
    const int32_t naborted = r.i32();
    for (int32_t k = 0; k < naborted; ++k) {
      r.i64();
      r.i64();
    }
    if (ec == E_NOT_LEADER && attempt < cfg_.max_retries) {
      refresh_metadata();
      continue;
    }
    if (ec != E_NONE) throw Error("kafka: Fetch error " + std::to_string(ec), ec);
    auto rec = r.bytes();
    rec_off = rec.first ? (size_t)(rec.first - reinterpret_cast<const uint8_t*>(resp.data())) : 0;
    rec_len = rec.second;
    return hwm;
  }
}

bool Client::same_leader(const std::string& topic, const std::vector<int>& partitions) {
  std::lock_guard<std::mutex> g(mu_);
  Connection* first = nullptr;
  for (int p : partitions) {
    Connection* c = &conn_for(topic, p);
    if (first && c != first) return false;
    first = c;
  }
  return true;
}

void Client::fetch_multi_raw(const std::string& topic, const std::vector<std::pair<int, int64_t>>& want,
                             int32_t max_bytes, int32_t max_wait_ms, std::string& resp, std::vector<PartSlice>& parts) {
  std::lock_guard<std::mutex> g(mu_);
  if (want.empty()) throw Error("kafka: fetch_multi_raw with no partitions");
  for (int attempt = 0;; ++attempt) {
    W w;
    w.i32(-1);
    w.i32(max_wait_ms);
    w.i32(1);
    w.i32(max_bytes);
    w.i8(0);
    w.arr(1);
    w.str(topic);
    w.arr((int32_t)want.size());
    for (const auto& pw : want) {
      w.i32(pw.first);
      w.i64(pw.second);
      w.i32(max_bytes);
    }
    size_t used = 0;
    try {
      used = call_into(conn_for(topic, want[0].first), API_FETCH, 4, w.s, resp);
    } catch (const Error& e) {
      if (attempt >= cfg_.max_retries) throw;
      conns_.clear();
      any_.reset();
      refresh_metadata();
      continue;
    }
    R r{reinterpret_cast<const uint8_t*>(resp.data()), used};
    r.i32();
    const int32_t nt = r.arr();
    parts.assign(want.size(), PartSlice{});
    bool retry = false;
    for (int32_t t = 0; t < nt; ++t) {
      r.str();
      const int32_t np = r.arr();
      for (int32_t k = 0; k < np; ++k) {
        const int32_t p = r.i32();
        const int16_t ec = r.i16();
        const int64_t hwm = r.i64();
        r.i64();
        const int32_t naborted = r.i32();
        for (int32_t a = 0; a < naborted; ++a) {
          r.i64();
          r.i64();
        }
        auto rec = r.bytes();
        if (ec == E_NOT_LEADER) {
          retry = true;
          continue;
        }
        if (ec != E_NONE) throw Error("kafka: Fetch error " + std::to_string(ec) + " on partition " + std::to_string(p), ec);
        for (size_t i = 0; i < want.size(); ++i)
          if (want[i].first == p) {
            parts[i].hwm = hwm;
            parts[i].rec_off = rec.first ? (size_t)(rec.first - reinterpret_cast<const uint8_t*>(resp.data())) : 0;
            parts[i].rec_len = rec.second;
          }
      }
    }
    if (retry && attempt < cfg_.max_retries) {
      refresh_metadata();
      continue;
    }
    if (retry) throw Error("kafka: Fetch error: not leader", E_NOT_LEADER);
    return;
  }
}

void Client::commit_multi(const std::string& group, const std::string& topic,
                          const std::vector<std::pair<int, int64_t>>& offsets) {
  if (offsets.empty()) return;
  std::lock_guard<std::mutex> g(mu_);
  W w;
  w.str(group);
  w.i32(-1);
  w.str("");
  w.i64(-1);
  w.arr(1);
  w.str(topic);
  w.arr((int32_t)offsets.size());
  for (const auto& po : offsets) {
    w.i32(po.first);
    w.i64(po.second);
    w.nullstr();
  }
  const std::string resp = call(any_conn(), API_OFFSET_COMMIT, 2, w.s);
  R r{reinterpret_cast<const uint8_t*>(resp.data()), resp.size()};
  const int32_t nt = r.arr();
  for (int32_t t = 0; t < nt; ++t) {
    r.str();
    const int32_t np = r.arr();
    for (int32_t k = 0; k < np; ++k) {
      r.i32();
      const int16_t ec = r.i16();
      if (ec != E_NONE) throw Error("kafka: OffsetCommit error " + std::to_string(ec), ec);
    }
  }
}

int64_t Client::produce(const std::string& topic, int partition, const std::vector<Record>& recs, int16_t acks) {
  std::lock_guard<std::mutex> g(mu_);
  W w;
  w.nullstr();  // transactional id
  w.i16(acks);
  w.i32(cfg_.timeout_ms);
  w.arr(1);
  w.str(topic);
  w.arr(1);
  w.i32(partition);
  w.bytes(encode_record_set(recs));
  const std::string resp = call(conn_for(topic, partition), API_PRODUCE, 3, w.s);
  if (acks == 0) return -1;
  R r{reinterpret_cast<const uint8_t*>(resp.data()), resp.size()};
  r.arr();
  r.str();
  r.arr();
  r.i32();
  const int16_t ec = r.i16();
  const int64_t base = r.i64();
  if (ec != E_NONE) throw Error("kafka: Produce error " + std::to_string(ec), ec);
  return base;
}

void Client::produce_multi(const std::string& topic, const std::vector<std::pair<int, std::vector<Record>>>& parts,
                           int16_t acks) {
  std::lock_guard<std::mutex> g(mu_);
  std::vector<std::pair<Connection*, std::vector<size_t>>> by_leader;
  for (size_t i = 0; i < parts.size(); ++i) {
    if (parts[i].second.empty()) continue;
    Connection* c = &conn_for(topic, parts[i].first);
    auto it = std::find_if(by_leader.begin(), by_leader.end(), [&](const auto& e) { return e.first == c; });
    if (it == by_leader.end()) by_leader.push_back({c, {i}});
    else it->second.push_back(i);
  }
  for (const auto& lead : by_leader) {
    W w;
    w.nullstr();  // transactional id
    w.i16(acks);
    w.i32(cfg_.timeout_ms);
    w.arr(1);
    w.str(topic);
    w.arr((int32_t)lead.second.size());
    for (size_t i : lead.second) {
      w.i32(parts[i].first);
      w.bytes(encode_record_set(parts[i].second));
    }
    const std::string resp = call(*lead.first, API_PRODUCE, 3, w.s);
    if (acks == 0) continue;
    R r{reinterpret_cast<const uint8_t*>(resp.data()), resp.size()};
    const int32_t nt = r.arr();
    for (int32_t t = 0; t < nt; ++t) {
      r.str();
      const int32_t np = r.arr();
      for (int32_t k = 0; k < np; ++k) {
        const int32_t p = r.i32();
        const int16_t ec = r.i16();
        r.i64();
        r.i64();   // log append time (v2+)
        if (ec != E_NONE)
          throw Error("kafka: Produce error " + std::to_string(ec) + " on partition " + std::to_string(p), ec);
      }
    }
  }
}

void Client::commit(const std::string& group, const std::string& topic, int partition, int64_t offset) {
  std::lock_guard<std::mutex> g(mu_);
  W w;
  w.str(group);
  w.i32(-1);
  w.str("");
  w.i64(-1);
  w.arr(1);
  w.str(topic);
  w.arr(1);
  w.i32(partition);
  w.i64(offset);
  w.nullstr();
  const std::string resp = call(any_conn(), API_OFFSET_COMMIT, 2, w.s);
  R r{reinterpret_cast<const uint8_t*>(resp.data()), resp.size()};
  r.arr();
  r.str();
  r.arr();
  r.i32();
  const int16_t ec = r.i16();
  if (ec != E_NONE) throw Error("kafka: OffsetCommit error " + std::to_string(ec), ec);
}

int64_t Client::committed(const std::string& group, const std::string& topic, int partition) {
  std::lock_guard<std::mutex> g(mu_);
  W w;
  w.str(group);
  w.arr(1);
  w.str(topic);
  w.arr(1);
  w.i32(partition);
  const std::string resp = call(any_conn(), API_OFFSET_FETCH, 1, w.s);
  R r{reinterpret_cast<const uint8_t*>(resp.data()), resp.size()};
  r.arr();
  r.str();
  r.arr();
  r.i32();
  const int64_t off = r.i64();
  r.str();
  const int16_t ec = r.i16();
  if (ec != E_NONE) throw Error("kafka: OffsetFetch error " + std::to_string(ec), ec);
  return off;
}

// ---------------------------------------------------------------------------
// in-process broker
// ---------------------------------------------------------------------------
Broker::Broker(BrokerConfig cfg) : cfg_(std::move(cfg)) {
  listen_fd_ = ::socket(AF_INET, SOCK_STREAM, 0);
  if (listen_fd_ < 0) throw Error("broker: socket() failed");
  int one = 1;
  setsockopt(listen_fd_, SOL_SOCKET, SO_REUSEADDR, &one, sizeof(one));
  sockaddr_in addr{};
  addr.sin_family = AF_INET;
  addr.sin_addr.s_addr = htonl(INADDR_LOOPBACK);
  addr.sin_port = htons((uint16_t)cfg_.port);
  if (::bind(listen_fd_, reinterpret_cast<sockaddr*>(&addr), sizeof(addr)) != 0 || ::listen(listen_fd_, 64) != 0) {
    ::close(listen_fd_);
    throw Error("broker: cannot listen on 127.0.0.1:" + std::to_string(cfg_.port));
  }
  socklen_t len = sizeof(addr);
  getsockname(listen_fd_, reinterpret_cast<sockaddr*>(&addr), &len);
  port_ = ntohs(addr.sin_port);
  running_ = true;
  accept_thread_ = std::thread([this] { accept_loop(); });
  retention_thread_ = std::thread([this] { retention_loop(); });
}

static int64_t steady_ms() {
  return std::chrono::duration_cast<std::chrono::milliseconds>(std::chrono::steady_clock::now().time_since_epoch())
      .count();
}

void Broker::retention_loop() {
  std::unique_lock<std::mutex> g(mu_);
  while (running_) {
    // system_clock: wait_for maps to pthread_cond_clockwait, which the ThreadSanitizer runtime here
    // does not model (it then reports the broker mutex as double-locked; mqtt.cpp wait_ms)
    retention_cv_.wait_until(g, std::chrono::system_clock::now() +
                                    std::chrono::milliseconds(std::max(cfg_.retention_check_ms, 10)));
    if (!running_) break;
    std::vector<std::shared_ptr<const std::string>> dead;
    enforce_locked(steady_ms(), dead);
    g.unlock();   // a second's worth of segments is freed without stalling produce / fetch
    dead.clear();
    g.lock();
  }
}

size_t Broker::enforce_retention() {
  std::vector<std::shared_ptr<const std::string>> dead;
  std::lock_guard<std::mutex> g(mu_);
  return enforce_locked(steady_ms(), dead);
}

// Kafka's log cleaner in delete mode: per partition, whole segments oldest first -- while the
// oldest is older than retention.ms (time), or while the log would still hold retention.bytes
// without it (size; the newest segment is always kept).  A consumer positioned inside a deleted
// range then gets OFFSET_OUT_OF_RANGE and follows its auto.offset.reset.  Segment bytes are
// shared: a fetch still sending one keeps it alive until it is done.
size_t Broker::enforce_locked(int64_t now_ms, std::vector<std::shared_ptr<const std::string>>& dead) {
  size_t dropped_total = 0;
  for (auto& tp : topics_) {
    int64_t ms = cfg_.retention_ms, by = cfg_.retention_bytes;
    auto rt = retention_.find(tp.first);
    if (rt != retention_.end()) {
      if (rt->second.ms != -2) ms = rt->second.ms;
      if (rt->second.bytes != -2) by = rt->second.bytes;
    }
    if (ms < 0 && by < 0) continue;
    for (Partition& p : tp.second) {
      size_t drop = 0;
      int64_t bytes = p.bytes, recs = 0;
      while (drop < p.segs.size()) {
        const Segment& sg = p.segs[drop];
        const bool old = ms >= 0 && now_ms - sg.append_ms > ms;
        const bool big = by >= 0 && drop + 1 < p.segs.size() && bytes - (int64_t)sg.bytes->size() >= by;
        if (!old && !big) break;
        bytes -= (int64_t)sg.bytes->size();
        recs += sg.count;
        ++drop;
      }
      if (!drop) continue;
      for (size_t i = 0; i < drop; ++i) {
        dead.push_back(std::move(p.segs.front().bytes));
        p.segs.pop_front();
      }
      p.bytes = bytes;
      p.start = p.segs.empty() ? p.end : p.segs.front().base;
      if (p.tbase >= 0 && p.tbase < p.start) {   // append times of deleted offsets go too
        const int64_t k = std::min<int64_t>(p.start - p.tbase, (int64_t)p.tappend.size());
        p.tappend.erase(p.tappend.begin(), p.tappend.begin() + (std::ptrdiff_t)k);   // deque: O(k)
        p.tbase += k;
      }
      deleted_segs_ += drop;
      deleted_recs_ += (uint64_t)recs;
      dropped_total += drop;
    }
  }
  return dropped_total;
}

int64_t Broker::log_bytes() {
  std::lock_guard<std::mutex> g(mu_);
  int64_t t = 0;
  for (auto& tp : topics_)
    for (const Partition& p : tp.second) t += p.bytes;
  return t;
}

size_t Broker::log_segments() {
  std::lock_guard<std::mutex> g(mu_);
  size_t t = 0;
  for (auto& tp : topics_)
    for (const Partition& p : tp.second) t += p.segs.size();
  return t;
}

Broker::~Broker() { stop(); }

void Broker::stop() {
  if (!running_.exchange(false)) return;
  {
    std::lock_guard<std::mutex> g(mu_);
    data_cv_.notify_all();
  }
  {
    std::lock_guard<std::mutex> g(mu_);   // under the lock: the loop checks running_ while holding it
    retention_cv_.notify_all();
  }
  if (retention_thread_.joinable()) retention_thread_.join();
  ::shutdown(listen_fd_, SHUT_RDWR);
  ::close(listen_fd_);
  if (accept_thread_.joinable()) accept_thread_.join();
  {
    std::lock_guard<std::mutex> g(mu_);
    for (int fd : client_fds_) ::shutdown(fd, SHUT_RDWR);
  }
  for (auto& t : workers_)
    if (t.joinable()) t.join();
  workers_.clear();
}

void Broker::accept_loop() {
  while (running_) {
    const int fd = ::accept(listen_fd_, nullptr, nullptr);
    if (fd < 0) {
      if (!running_) break;
      continue;
    }
    int one = 1;
    setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
    int sz = 4 << 20;
    setsockopt(fd, SOL_SOCKET, SO_SNDBUF, &sz, sizeof(sz));
    std::lock_guard<std::mutex> g(mu_);
    // join the connection threads that have finished (serve closed its fd and took it off client_fds_)
    for (size_t i = 0; i < workers_.size();) {
      if (worker_done_[i]->load(std::memory_order_acquire)) {
        workers_[i].join();
        workers_.erase(workers_.begin() + (std::ptrdiff_t)i);
        worker_done_.erase(worker_done_.begin() + (std::ptrdiff_t)i);   // (serve removed its own fd)
      } else {
        ++i;
      }
    }
    client_fds_.push_back(fd);
    auto done = std::make_shared<std::atomic<bool>>(false);
    worker_done_.push_back(done);
    workers_.emplace_back([this, fd, done] {
      serve(fd);
      done->store(true, std::memory_order_release);
    });
    if (!thread_cpus_.empty()) {
      cpu_set_t set;
      CPU_ZERO(&set);
      for (int c : thread_cpus_)
        if (c >= 0 && c < CPU_SETSIZE) CPU_SET(c, &set);
      pthread_setaffinity_np(workers_.back().native_handle(), sizeof(set), &set);   // best effort
    }
  }
}

void Broker::set_thread_cpus(const std::vector<int>& cpus) {
  std::lock_guard<std::mutex> g(mu_);
  thread_cpus_ = cpus;
}

void Broker::create_topic(const std::string& name, int partitions, int64_t retention_ms, int64_t retention_bytes) {
  std::lock_guard<std::mutex> g(mu_);
  auto& t = topics_[name];
  if ((int)t.size() < partitions) t.resize((size_t)partitions);
  if (retention_ms != -2 || retention_bytes != -2) {
    TopicRetention& r = retention_[name];
    if (retention_ms != -2) r.ms = retention_ms;
    if (retention_bytes != -2) r.bytes = retention_bytes;
  }
}

void Broker::record_append_times(bool on) { record_times_ = on; }

std::vector<int64_t> Broker::append_times(const std::string& topic, int partition, int64_t start, int64_t count) {
  std::lock_guard<std::mutex> g(mu_);
  const Partition& p = topics_.at(topic).at((size_t)partition);
  std::vector<int64_t> out((size_t)std::max<int64_t>(count, 0), -1);
  for (int64_t i = 0; i < count; ++i) {
    const int64_t k = start + i - p.tbase;
    if (p.tbase >= 0 && k >= 0 && k < (int64_t)p.tappend.size()) out[(size_t)i] = p.tappend[(size_t)k];
  }
  return out;
}

// Low-latency mode (spin_us > 0): take the broker lock by spinning on try_lock for up to
// `spin_us` before blocking.  The lock is only ever held for microseconds (picking segments,
// appending a batch); a blocked lock() parks the thread in the kernel and costs a
// scheduler wake-up (several microseconds) on exactly the append -> fetch path the
// low-latency serving loop measures.
static void lock_spin(std::unique_lock<std::mutex>& g, int spin_us) {
  if (spin_us > 0) {
    const auto t_end = std::chrono::steady_clock::now() + std::chrono::microseconds(spin_us);
    for (uint32_t i = 0;; ++i) {
      if (g.try_lock()) return;
#if defined(__x86_64__)
      __builtin_ia32_pause();
#endif
      if ((i & 63) == 63 && std::chrono::steady_clock::now() >= t_end) break;
    }
  }
  g.lock();
}

int64_t Broker::append_locked(Partition& p, const Record* recs, size_t n) {
  const int64_t base = p.end;
  if (record_times_.load(std::memory_order_relaxed)) {
    const int64_t now = std::chrono::duration_cast<std::chrono::nanoseconds>(
                            std::chrono::steady_clock::now().time_since_epoch()).count();
    if (p.tbase < 0) p.tbase = base;
    p.tappend.resize((size_t)(base - p.tbase), -1);   // offsets appended while recording was off
    p.tappend.insert(p.tappend.end(), n, now);
  }
  const int64_t now_ms = steady_ms();
  for (size_t k = 0; k < n; k += kSegmentRecords) {
    const size_t m = std::min(kSegmentRecords, n - k);
    Segment sg;
    sg.base = p.end;
    sg.count = (int32_t)m;
    sg.append_ms = now_ms;
    sg.bytes = std::make_shared<const std::string>(encode_record_batch(p.end, recs + k, m));
    p.bytes += (int64_t)sg.bytes->size();
    p.segs.push_back(std::move(sg));
    p.end += (int64_t)m;
  }
  // record-count retention: whole segments, oldest first, while the rest still holds the limit
  // (Kafka deletes log segments, not records); time / size retention: retention_loop
  if (cfg_.retention_records > 0) {
    size_t drop = 0;
    int64_t recs_dropped = 0;
    while (drop + 1 < p.segs.size() && p.end - (p.segs[drop].base + p.segs[drop].count) >= cfg_.retention_records) {
      p.bytes -= (int64_t)p.segs[drop].bytes->size();
      recs_dropped += p.segs[drop].count;
      ++drop;
    }
    if (drop) {
      p.segs.erase(p.segs.begin(), p.segs.begin() + (std::ptrdiff_t)drop);
      deleted_segs_ += drop;
      deleted_recs_ += (uint64_t)recs_dropped;
    }
  }
  p.start = p.segs.empty() ? p.end : p.segs.front().base;
  append_seq_.fetch_add(1, std::memory_order_release);
  data_cv_.notify_all();   // wake long-polling fetches
  return base;
}

int64_t Broker::append(const std::string& topic, int partition, const std::vector<Record>& recs) {
  std::lock_guard<std::mutex> g(mu_);
  auto it = topics_.find(topic);
  if (it == topics_.end() || partition < 0 || partition >= (int)it->second.size())
    throw Error("broker: unknown topic/partition", E_UNKNOWN_TOPIC);
  return append_locked(it->second[(size_t)partition], recs.data(), recs.size());
}

int64_t Broker::end_offset(const std::string& topic, int partition) {
  std::lock_guard<std::mutex> g(mu_);
  return topics_.at(topic).at((size_t)partition).end;
}

int64_t Broker::start_offset(const std::string& topic, int partition) {
  std::lock_guard<std::mutex> g(mu_);
  return topics_.at(topic).at((size_t)partition).start;
}

std::vector<Record> Broker::read(const std::string& topic, int partition, int64_t offset, size_t max_records) {
  std::vector<std::shared_ptr<const std::string>> segs;
  {
    std::lock_guard<std::mutex> g(mu_);
    const Partition& p = topics_.at(topic).at((size_t)partition);
    for (const Segment& sg : p.segs)
      if (sg.base + sg.count > offset) segs.push_back(sg.bytes);
  }
  std::vector<Record> out;
  for (const auto& sp : segs) {
    RecordSetCursor cur(reinterpret_cast<const uint8_t*>(sp->data()), sp->size());
    RecordView v;
    while (out.size() < max_records && cur.next(v)) {
      if (v.offset < offset) continue;
      Record r;
      r.offset = v.offset;
      r.timestamp = v.timestamp;
      r.key_null = v.key_len < 0;
      if (v.key_len > 0) r.key.assign(reinterpret_cast<const char*>(v.key), (size_t)v.key_len);
      r.value.assign(reinterpret_cast<const char*>(v.value), (size_t)v.value_len);
      out.push_back(std::move(r));
    }
    if (out.size() >= max_records) break;
  }
  return out;
}

size_t Broker::FetchReply::total() const {
  size_t t = meta.size();
  for (const auto& sp : splice) t += sp.second->size();
  return t;
}

Broker::FetchReply Broker::handle_fetch(const uint8_t* body, size_t n) {
  R r{body, n};
  const uint64_t nth = ++fetches_;
  r.i32();                              // replica id
  const int32_t max_wait_ms = r.i32();  // long poll: an empty fetch waits up to this long
  const int32_t min_bytes = r.i32();    //   for at least one byte of new records
  r.i32();
  r.i8();
  struct Want {
    std::string topic;
    int32_t partition, pmax;
    int64_t off;
    int16_t err = E_NONE;
    int64_t hwm = -1;
    std::vector<std::shared_ptr<const std::string>> segs;
  };
  std::vector<std::pair<std::string, std::vector<Want>>> req;
  const int32_t nt = r.arr();
  for (int32_t i = 0; i < nt; ++i) {
    req.emplace_back(r.str(), std::vector<Want>());
    const int32_t np = r.arr();
    for (int32_t k = 0; k < np; ++k) {
      Want wt;
      wt.topic = req.back().first;
      wt.partition = r.i32();
      wt.off = r.i64();
      wt.pmax = r.i32();
      req.back().second.push_back(std::move(wt));
    }
  }
  {
    // only to pick the segments: the copy runs unlocked.  Kafka's fetch.min.bytes /
    // fetch.max.wait.ms: when nothing is available yet the request parks on data_cv_
    // (signalled by every append) instead of returning empty, so a consumer sees a new
    // record one wake-up after it is appended, without polling.
    std::unique_lock<std::mutex> g(mu_, std::defer_lock);
    lock_spin(g, spin_us_.load());
    const int fe = fail_every_.load();
    const bool fail = fe > 0 && nth % (uint64_t)fe == 0;
    auto pick = [&]() {   // -> (any bytes, any error)
      bool avail = false, errs = false;
      for (auto& tp : req)
        for (Want& wt : tp.second) {
          wt.err = E_NONE;
          wt.segs.clear();
          auto it = topics_.find(wt.topic);
          if (fail) {
            wt.err = E_NOT_LEADER;
          } else if (it == topics_.end() || wt.partition < 0 || wt.partition >= (int32_t)it->second.size()) {
            wt.err = E_UNKNOWN_TOPIC;
          } else {
            const Partition& part = it->second[(size_t)wt.partition];
            wt.hwm = part.end;
            if (wt.off < part.start || wt.off > part.end) {
              wt.err = E_OFFSET_OUT_OF_RANGE;
            } else {
              auto sg = std::upper_bound(part.segs.begin(), part.segs.end(), wt.off,
                                         [](int64_t o, const Segment& s_) { return o < s_.base + s_.count; });
              size_t bytes = 0;
              for (; sg != part.segs.end() && (bytes == 0 || bytes < (size_t)std::max(wt.pmax, 0)); ++sg) {
                wt.segs.push_back(sg->bytes);
                bytes += sg->bytes->size();
              }
              avail |= bytes > 0;
            }
          }
          errs |= wt.err != E_NONE;
        }
      return std::make_pair(avail, errs);
    };
    auto st = pick();
    if (fail) ++failures_;
    const int spin = spin_us_.load();
    if (!st.first && !st.second && min_bytes > 0 && max_wait_ms > 0 && spin > 0) {
      // low-latency mode: watch the append counter without the lock before parking
      const uint64_t seq0 = append_seq_.load(std::memory_order_acquire);
      g.unlock();
      const auto t_end = std::chrono::steady_clock::now() + std::chrono::microseconds(std::min(spin, max_wait_ms * 1000));
      while (running_ && append_seq_.load(std::memory_order_acquire) == seq0 && std::chrono::steady_clock::now() < t_end) {
#if defined(__x86_64__)
        __builtin_ia32_pause();
#endif
      }
      lock_spin(g, spin);
      st = pick();
    }
    if (!st.first && !st.second && min_bytes > 0 && max_wait_ms > 0) {
      // system_clock deadline: pthread_cond_timedwait (the steady_clock form maps to
      // pthread_cond_clockwait, which the ThreadSanitizer runtime here does not model)
      const auto deadline = std::chrono::system_clock::now() + std::chrono::milliseconds(max_wait_ms);
      while (running_ && !st.first && !st.second) {
        const bool timed_out = data_cv_.wait_until(g, deadline) == std::cv_status::timeout;
        st = pick();
        if (timed_out) break;
      }
    }
  }
  FetchReply out;
  W w;
  w.i32(0);
  w.arr(nt);
  for (auto& tp : req) {
    w.str(tp.first);
    w.arr((int32_t)tp.second.size());
    for (Want& wt : tp.second) {
      w.i32(wt.partition);
      w.i16(wt.err);
      w.i64(wt.hwm);
      w.i64(wt.hwm);
      w.i32(0);  // no aborted transactions
      if (wt.err != E_NONE) {
        w.i32(-1);
        continue;
      }
      size_t total = 0;
      for (const auto& sp : wt.segs) total += sp->size();
      w.i32((int32_t)total);
      for (auto& sp : wt.segs) out.splice.emplace_back(w.s.size(), std::move(sp));
    }
  }
  const int dm = delay_ms_.load();
  if (dm > 0) std::this_thread::sleep_for(std::chrono::milliseconds(dm));
  out.meta = std::move(w.s);
  return out;
}

void Broker::serve(int fd) {
  bool authed = cfg_.sasl_username.empty();
  bool handshaken = false;
  std::string buf;
  while (running_) {
    uint8_t hdr[4];
    size_t got = 0;
    if (const int spin = spin_us_.load(); spin > 0) {
      // low-latency mode: the next request on a serving connection usually follows within
      // microseconds; busy-poll it instead of paying a blocked recv's thread wake-up
      const auto t_end = std::chrono::steady_clock::now() + std::chrono::microseconds(spin);
      while (got < 4 && running_) {
        const ssize_t k = ::recv(fd, hdr + got, 4 - got, MSG_DONTWAIT);
        if (k > 0) {
          got += (size_t)k;
          continue;
        }
        if (k == 0 || (errno != EAGAIN && errno != EWOULDBLOCK && errno != EINTR)) goto done;
        if (std::chrono::steady_clock::now() >= t_end) break;
#if defined(__x86_64__)
        __builtin_ia32_pause();
#endif
      }
    }
    while (got < 4) {
      const ssize_t k = ::recv(fd, hdr + got, 4 - got, 0);
      if (k <= 0) goto done;
      got += (size_t)k;
    }
    {
      const int32_t size = (int32_t)(((uint32_t)hdr[0] << 24) | ((uint32_t)hdr[1] << 16) | ((uint32_t)hdr[2] << 8) | hdr[3]);
      if (size < 8 || size > (1 << 28)) goto done;
      buf.resize((size_t)size);
      got = 0;
      while (got < (size_t)size) {
        const ssize_t k = ::recv(fd, &buf[got], (size_t)size - got, 0);
        if (k <= 0) goto done;
        got += (size_t)k;
      }
      std::string resp_body;
      int32_t corr = 0;
      FetchReply fr;
      bool is_fetch = false;
      try {
        R r{reinterpret_cast<const uint8_t*>(buf.data()), buf.size()};
        const int16_t api = r.i16();
        const int16_t ver = r.i16();
        corr = r.i32();
        r.str();  // client id
        is_fetch = api == API_FETCH && authed;
        if (is_fetch) fr = handle_fetch(r.p + r.i, r.n - r.i);
        else resp_body = handle(api, ver, r.p + r.i, r.n - r.i, authed, handshaken);
      } catch (const std::exception&) {
        goto done;  // malformed request: drop the connection (like a real broker)
      }
      if (is_fetch) {
        // zero-copy reply: header + framing + segment bytes gathered by the kernel
        W h;
        h.i32((int32_t)(fr.total() + 4));
        h.i32(corr);
        std::vector<iovec> iov;
        iov.push_back({&h.s[0], h.s.size()});
        size_t at = 0;
        for (const auto& sp : fr.splice) {
          if (sp.first > at) iov.push_back({&fr.meta[at], sp.first - at});
          iov.push_back({const_cast<char*>(sp.second->data()), sp.second->size()});
          at = sp.first;
        }
        if (fr.meta.size() > at) iov.push_back({&fr.meta[at], fr.meta.size() - at});
        size_t k0 = 0;
        while (k0 < iov.size()) {
          msghdr mh{};
          mh.msg_iov = &iov[k0];
          mh.msg_iovlen = std::min<size_t>(iov.size() - k0, 512);
          ssize_t k = ::sendmsg(fd, &mh, MSG_NOSIGNAL);
          if (k <= 0) goto done;
          while (k > 0 && k0 < iov.size()) {   // advance over what was sent
            if ((size_t)k >= iov[k0].iov_len) {
              k -= (ssize_t)iov[k0].iov_len;
              ++k0;
            } else {
              iov[k0].iov_base = static_cast<char*>(iov[k0].iov_base) + k;
              iov[k0].iov_len -= (size_t)k;
              k = 0;
            }
          }
        }
        continue;
      }
      W w;
      w.i32((int32_t)(resp_body.size() + 4));
      w.i32(corr);
      // header, then the body straight from its buffer (no concatenated copy of a
      // multi-megabyte fetch response)
      for (int part = 0; part < 2; ++part) {
        const std::string& out = part == 0 ? w.s : resp_body;
        size_t off = 0;
        while (off < out.size()) {
          const ssize_t k = ::send(fd, out.data() + off, out.size() - off,
                                   MSG_NOSIGNAL | (part == 0 && !resp_body.empty() ? MSG_MORE : 0));
          if (k <= 0) goto done;
          off += (size_t)k;
        }
      }
    }
  }
done:
  ::close(fd);
  std::lock_guard<std::mutex> g(mu_);
  client_fds_.erase(std::remove(client_fds_.begin(), client_fds_.end(), fd), client_fds_.end());
}

std::string Broker::handle(int16_t api, int16_t ver, const uint8_t* body, size_t n, bool& authed,
                           bool& handshaken) {
  R r{body, n};
  W w;
  if (api == API_API_VERSIONS) {
    w.i16(E_NONE);
    const int16_t apis[][3] = {{API_PRODUCE, 3, 3}, {API_FETCH, 4, 4}, {API_LIST_OFFSETS, 1, 1},
                               {API_METADATA, 1, 1}, {API_OFFSET_COMMIT, 2, 2}, {API_OFFSET_FETCH, 1, 1},
                               {API_FIND_COORDINATOR, 1, 1}, {API_SASL_HANDSHAKE, 1, 1},
                               {API_API_VERSIONS, 0, 0}, {API_SASL_AUTH, 0, 0}};
    w.arr(10);
    for (auto& a : apis) {
      w.i16(a[0]);
      w.i16(a[1]);
      w.i16(a[2]);
    }
    return w.s;
  }
  if (api == API_SASL_HANDSHAKE) {
    const std::string mech = r.str();
    const bool ok = mech == "PLAIN";
    handshaken = ok;
    w.i16(ok ? E_NONE : E_UNSUPPORTED_SASL);
    w.arr(1);
    w.str("PLAIN");
    return w.s;
  }
  if (api == API_SASL_AUTH) {
    auto tok = r.bytes();
    std::string t(reinterpret_cast<const char*>(tok.first), tok.second);
    // [authzid] \0 user \0 pass
    const auto a = t.find('\0');
    const auto b = a == std::string::npos ? std::string::npos : t.find('\0', a + 1);
    bool ok = false;
    if (handshaken && b != std::string::npos)
      ok = t.substr(a + 1, b - a - 1) == cfg_.sasl_username && t.substr(b + 1) == cfg_.sasl_password;
    authed = authed || ok;
    w.i16(handshaken ? (ok ? E_NONE : E_SASL_AUTH_FAILED) : E_ILLEGAL_SASL_STATE);
    w.nullstr();
    w.bytes("");
    return w.s;
  }
  if (!authed) throw Error("broker: unauthenticated request");
  if (api == API_FETCH) {   // served by handle_fetch + sendmsg in serve(); kept for completeness
    FetchReply fr = handle_fetch(body, n);
    std::string flat;
    flat.reserve(fr.total());
    size_t at = 0;
    for (const auto& sp : fr.splice) {
      flat.append(fr.meta, at, sp.first - at);
      flat += *sp.second;
      at = sp.first;
    }
    flat.append(fr.meta, at, std::string::npos);
    return flat;
  }
  std::unique_lock<std::mutex> g(mu_, std::defer_lock);
  lock_spin(g, spin_us_.load());
  switch (api) {
    case API_METADATA: {
      const int32_t nt = r.i32();
      std::vector<std::string> want;
      for (int32_t i = 0; i < nt; ++i) want.push_back(r.str());
      w.arr(1);
      w.i32(0);
      w.str("127.0.0.1");
      w.i32(port_);
      w.nullstr();
      w.i32(0);  // controller
      std::vector<std::string> names;
      if (nt < 0) for (const auto& kv : topics_) names.push_back(kv.first);
      else names = want;
      if (cfg_.auto_create_topics)
        for (const auto& name : want)
          if (!name.empty() && topics_.find(name) == topics_.end()) topics_[name].resize(1);
      w.arr((int32_t)names.size());
      for (const auto& name : names) {
        auto it = topics_.find(name);
        w.i16(it == topics_.end() ? E_UNKNOWN_TOPIC : E_NONE);
        w.str(name);
        w.i8(0);
        const int32_t np = it == topics_.end() ? 0 : (int32_t)it->second.size();
        w.arr(np);
        for (int32_t p = 0; p < np; ++p) {
          w.i16(E_NONE);
          w.i32(p);
          w.i32(0);
          w.arr(1);
          w.i32(0);
          w.arr(1);
          w.i32(0);
        }
      }
      return w.s;
    }
    case API_LIST_OFFSETS: {
      r.i32();
      const int32_t nt = r.arr();
      w.arr(nt);
      for (int32_t i = 0; i < nt; ++i) {
        const std::string name = r.str();
        const int32_t np = r.arr();
        w.str(name);
        w.arr(np);
        for (int32_t k = 0; k < np; ++k) {
          const int32_t p = r.i32();
          const int64_t t = r.i64();
          auto it = topics_.find(name);
          w.i32(p);
          if (it == topics_.end() || p < 0 || p >= (int32_t)it->second.size()) {
            w.i16(E_UNKNOWN_TOPIC);
            w.i64(-1);
            w.i64(-1);
            continue;
          }
          const Partition& part = it->second[(size_t)p];
          w.i16(E_NONE);
          w.i64(-1);
          w.i64(t == -2 ? part.start : part.end);
        }
      }
      return w.s;
    }
    case API_PRODUCE: {
      r.str();
      const int16_t acks = r.i16();
      (void)acks;
      r.i32();
      const int32_t nt = r.arr();
      w.arr(nt);
      for (int32_t i = 0; i < nt; ++i) {
        const std::string name = r.str();
        const int32_t np = r.arr();
        w.str(name);
        w.arr(np);
        for (int32_t k = 0; k < np; ++k) {
          const int32_t p = r.i32();
          auto recs = r.bytes();
          auto it = topics_.find(name);
          w.i32(p);
          if (it == topics_.end() || p < 0 || p >= (int32_t)it->second.size()) {
            w.i16(E_UNKNOWN_TOPIC);
            w.i64(-1);
            w.i64(-1);
            continue;
          }
          if (cfg_.message_max_bytes > 0 && max_batch_size(recs.first, recs.second) > cfg_.message_max_bytes) {
            w.i16(E_MESSAGE_TOO_LARGE);   // a record batch over message.max.bytes: nothing appended
            w.i64(-1);
            w.i64(-1);
            continue;
          }
          FetchResult tmp;
          decode_record_batches(recs.first, recs.second, INT64_MIN, tmp);
          std::vector<Record> recs_in(tmp.size());
          for (size_t q = 0; q < tmp.size(); ++q) {
            Record& rec = recs_in[q];
            rec.timestamp = tmp.timestamps[q];
            rec.key = tmp.keys[q];
            rec.key_null = tmp.keys[q].empty();
            rec.value.assign(tmp.values.data() + tmp.value_offsets[q],
                             (size_t)(tmp.value_offsets[q + 1] - tmp.value_offsets[q]));
          }
          const int64_t base = append_locked(it->second[(size_t)p], recs_in.data(), recs_in.size());
          w.i16(E_NONE);
          w.i64(base);
          w.i64(-1);
        }
      }
      w.i32(0);  // throttle
      return w.s;
    }
    case API_FIND_COORDINATOR: {
      r.str();
      w.i32(0);
      w.i16(E_NONE);
      w.nullstr();
      w.i32(0);
      w.str("127.0.0.1");
      w.i32(port_);
      return w.s;
    }
    case API_OFFSET_COMMIT: {
      const std::string group = r.str();
      r.i32();
      r.str();
      r.i64();
      const int32_t nt = r.arr();
      w.arr(nt);
      for (int32_t i = 0; i < nt; ++i) {
        const std::string name = r.str();
        const int32_t np = r.arr();
        w.str(name);
        w.arr(np);
        for (int32_t k = 0; k < np; ++k) {
          const int32_t p = r.i32();
          const int64_t off = r.i64();
          r.str();
          group_offsets_[group + "/" + name + "/" + std::to_string(p)] = off;
          w.i32(p);
          w.i16(E_NONE);
        }
      }
      return w.s;
    }
    case API_OFFSET_FETCH: {
      const std::string group = r.str();
      const int32_t nt = r.arr();
      w.arr(nt);
      for (int32_t i = 0; i < nt; ++i) {
        const std::string name = r.str();
        const int32_t np = r.arr();
        w.str(name);
        w.arr(np);
        for (int32_t k = 0; k < np; ++k) {
          const int32_t p = r.i32();
          auto it = group_offsets_.find(group + "/" + name + "/" + std::to_string(p));
          w.i32(p);
          w.i64(it == group_offsets_.end() ? -1 : it->second);
          w.nullstr();
          w.i16(E_NONE);
        }
      }
      return w.s;
    }
    default:
      (void)ver;
      throw Error("broker: unsupported api " + std::to_string(api));
  }
}

}  // namespace kafka
}  // namespace sml
