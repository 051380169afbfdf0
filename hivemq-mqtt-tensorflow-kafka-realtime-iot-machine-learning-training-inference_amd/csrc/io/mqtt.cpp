// MQTT broker + Kafka bridge + client + device simulator (see mqtt.h).
//
// Broker design: one accept thread and a few epoll I/O threads; every connection is
// non-blocking and owned by one I/O thread (reads, parsing, protocol handling).
// Outbound bytes go through a per-session buffer: the writer appends and tries an
// immediate send(); a short write arms EPOLLOUT and the owning thread drains the
// rest.  Routing takes the broker lock only to collect the target sessions, then
// delivers outside it.  The Kafka bridge is a separate thread that drains a queue
// in batches and produces with the native Kafka client (kafka.h), partitioning by
// Kafka's default murmur2 partitioner on the record key (= the MQTT topic), as the
// HiveMQ Kafka extension does.
#include "mqtt.h"

#include <arpa/inet.h>
#include <fcntl.h>
#include <netdb.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <poll.h>
#include <sys/epoll.h>
#include <sys/socket.h>
#include <unistd.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstring>
#include <random>
#include <set>

namespace sml {
namespace mqtt {

namespace {

int64_t now_ms() {
  return std::chrono::duration_cast<std::chrono::milliseconds>(std::chrono::system_clock::now().time_since_epoch())
      .count();
}

struct W {
  std::string s;
  void u8(uint8_t v) { s.push_back((char)v); }
  void u16(uint16_t v) {
    s.push_back((char)(v >> 8));
    s.push_back((char)(v & 0xff));
  }
  void str(const std::string& v) {
    if (v.size() > 0xffff) throw Error("mqtt: string longer than 65535 bytes");
    u16((uint16_t)v.size());
    s += v;
  }
  void props_empty() { s.push_back('\0'); }  // v5: zero-length property block
};

struct R {
  const uint8_t* p;
  size_t n, i = 0;
  R(const uint8_t* p_, size_t n_) : p(p_), n(n_) {}
  void need(size_t k) const {
    if (i + k > n) throw Error("mqtt: truncated packet");
  }
  uint8_t u8() {
    need(1);
    return p[i++];
  }
  uint16_t u16() {
    need(2);
    const uint16_t v = (uint16_t)((p[i] << 8) | p[i + 1]);
    i += 2;
    return v;
  }
  std::string str() {
    const uint16_t k = u16();
    need(k);
    std::string v(reinterpret_cast<const char*>(p + i), k);
    i += k;
    return v;
  }
  uint32_t varint() {
    uint32_t v = 0;
    for (int sh = 0; sh < 28; sh += 7) {
      const uint8_t b = u8();
      v |= (uint32_t)(b & 0x7f) << sh;
      if (!(b & 0x80)) return v;
    }
    throw Error("mqtt: malformed variable byte integer");
  }
  void skip_props() {
    const uint32_t k = varint();
    need(k);
    i += k;
  }
  std::string rest() {
    std::string v(reinterpret_cast<const char*>(p + i), n - i);
    i = n;
    return v;
  }
  bool done() const { return i >= n; }
};

// Timed condition-variable wait against the system clock.  libstdc++ implements
// wait_for() with pthread_cond_clockwait, which GCC 11's ThreadSanitizer does not
// intercept (it then reports the held mutex as double-locked); wait_until() on
// system_clock uses pthread_cond_timedwait, which every sanitizer understands.
template <class Pred>
bool cv_wait_ms(std::condition_variable& cv, std::unique_lock<std::mutex>& g, int64_t ms, Pred pred) {
  return cv.wait_until(g, std::chrono::system_clock::now() + std::chrono::milliseconds(ms), pred);
}

void set_nonblock(int fd) { ::fcntl(fd, F_SETFL, ::fcntl(fd, F_GETFL, 0) | O_NONBLOCK); }

bool send_all_blocking(int fd, const std::string& s) {
  size_t off = 0;
  while (off < s.size()) {
    const ssize_t k = ::send(fd, s.data() + off, s.size() - off, MSG_NOSIGNAL);
    if (k < 0) {
      if (errno == EINTR) continue;
      if (errno == EAGAIN || errno == EWOULDBLOCK) {
        pollfd pf{fd, POLLOUT, 0};
        ::poll(&pf, 1, 1000);
        continue;
      }
      return false;
    }
    off += (size_t)k;
  }
  return true;
}

std::string ack_packet(uint8_t type, uint16_t id) {
  W w;
  w.u16(id);
  return frame(type, type == PUBREL ? 0x2 : 0x0, w.s);
}

}  // namespace

// ---- codec --------------------------------------------------------------------
void put_varint(std::string& s, uint32_t v) {
  do {
    uint8_t b = v & 0x7f;
    v >>= 7;
    if (v) b |= 0x80;
    s.push_back((char)b);
  } while (v);
}

std::string frame(uint8_t type, uint8_t flags, const std::string& body) {
  std::string s;
  s.reserve(body.size() + 5);
  s.push_back((char)((type << 4) | (flags & 0x0f)));
  put_varint(s, (uint32_t)body.size());
  s += body;
  return s;
}

size_t parse_packet(const uint8_t* p, size_t n, Packet& out) {
  if (n < 2) return 0;
  uint32_t len = 0;
  size_t i = 1;
  for (int sh = 0;; sh += 7) {
    if (i >= n) return 0;
    if (sh > 21) throw Error("mqtt: malformed remaining length");
    const uint8_t b = p[i++];
    len |= (uint32_t)(b & 0x7f) << sh;
    if (!(b & 0x80)) break;
  }
  if (len > (256u << 20)) throw Error("mqtt: packet too large");
  if (n - i < len) return 0;
  out.type = p[0] >> 4;
  out.flags = p[0] & 0x0f;
  out.body.assign(reinterpret_cast<const char*>(p + i), len);
  return i + len;
}

std::string encode_connect(const std::string& client_id, int version, uint16_t keepalive, bool clean,
                           const std::string& username, const std::string& password) {
  W w;
  w.str("MQTT");
  w.u8((uint8_t)version);
  uint8_t fl = clean ? 0x02 : 0x00;
  if (!username.empty()) fl |= 0x80;
  if (!password.empty()) fl |= 0x40;
  w.u8(fl);
  w.u16(keepalive);
  if (version == 5) w.props_empty();
  w.str(client_id);
  if (!username.empty()) w.str(username);
  if (!password.empty()) w.str(password);
  return frame(CONNECT, 0, w.s);
}

std::string encode_publish(const Message& m, int version) {
  W w;
  w.str(m.topic);
  if (m.qos > 0) w.u16(m.packet_id);
  if (version == 5) w.props_empty();
  w.s += m.payload;
  const uint8_t fl = (uint8_t)((m.dup ? 0x8 : 0) | ((m.qos & 3) << 1) | (m.retain ? 1 : 0));
  return frame(PUBLISH, fl, w.s);
}

Message decode_publish(const Packet& pk, int version) {
  Message m;
  m.dup = pk.flags & 0x8;
  m.qos = (pk.flags >> 1) & 3;
  m.retain = pk.flags & 1;
  if (m.qos == 3) throw Error("mqtt: PUBLISH with QoS 3");
  R r(reinterpret_cast<const uint8_t*>(pk.body.data()), pk.body.size());
  m.topic = r.str();
  if (m.qos > 0) m.packet_id = r.u16();
  if (version == 5) r.skip_props();
  m.payload = r.rest();
  return m;
}

std::string encode_subscribe(uint16_t packet_id, const std::vector<std::pair<std::string, int>>& filters,
                             int version) {
  W w;
  w.u16(packet_id);
  if (version == 5) w.props_empty();
  for (const auto& f : filters) {
    w.str(f.first);
    w.u8((uint8_t)(f.second & 3));
  }
  return frame(SUBSCRIBE, 0x2, w.s);
}

bool valid_filter(const std::string& f) {
  if (f.empty()) return false;
  size_t start = 0;
  while (true) {
    const size_t end = f.find('/', start);
    const std::string lvl = f.substr(start, end == std::string::npos ? std::string::npos : end - start);
    if (lvl.find('#') != std::string::npos && (lvl != "#" || end != std::string::npos)) return false;
    if (lvl.find('+') != std::string::npos && lvl != "+") return false;
    if (end == std::string::npos) break;
    start = end + 1;
  }
  return true;
}

bool topic_matches(const std::string& filter, const std::string& topic) {
  if (!topic.empty() && topic[0] == '$' && !filter.empty() && (filter[0] == '+' || filter[0] == '#')) return false;
  size_t fi = 0, ti = 0;
  while (true) {
    const size_t fe = filter.find('/', fi);
    const std::string fl = filter.substr(fi, fe == std::string::npos ? std::string::npos : fe - fi);
    if (fl == "#") return true;  // matches this level and everything below (incl. the parent)
    if (ti > topic.size()) return false;
    const size_t te = topic.find('/', ti);
    const std::string tl = topic.substr(ti, te == std::string::npos ? std::string::npos : te - ti);
    if (fl != "+" && fl != tl) return false;
    const bool fend = fe == std::string::npos, tend = te == std::string::npos;
    if (fend && tend) return true;
    if (tend) {  // topic exhausted: only a trailing "/#" still matches ("a/#" matches "a")
      return !fend && filter.compare(fe + 1, std::string::npos, "#") == 0;
    }
    if (fend) return false;
    fi = fe + 1;
    ti = te + 1;
  }
}

uint32_t murmur2(const std::string& key) {
  const uint32_t seed = 0x9747b28c, m = 0x5bd1e995;
  const int r = 24;
  const size_t len = key.size();
  uint32_t h = seed ^ (uint32_t)len;
  const uint8_t* d = reinterpret_cast<const uint8_t*>(key.data());
  const size_t n4 = len / 4;
  for (size_t i = 0; i < n4; ++i) {
    uint32_t k = (uint32_t)d[4 * i] | ((uint32_t)d[4 * i + 1] << 8) | ((uint32_t)d[4 * i + 2] << 16) |
                 ((uint32_t)d[4 * i + 3] << 24);
    k *= m;
    k ^= k >> r;
    k *= m;
    h *= m;
    h ^= k;
  }
  const size_t t = len & ~(size_t)3;
  switch (len % 4) {
    case 3: h ^= (uint32_t)d[t + 2] << 16; [[fallthrough]];
    case 2: h ^= (uint32_t)d[t + 1] << 8; [[fallthrough]];
    case 1:
      h ^= (uint32_t)d[t];
      h *= m;
  }
  h ^= h >> 13;
  h *= m;
  h ^= h >> 15;
  return h;
}

int kafka_partition(const std::string& key, int partitions) {
  if (partitions <= 1) return 0;
  return (int)((murmur2(key) & 0x7fffffff) % (uint32_t)partitions);
}

// ---- broker ---------------------------------------------------------------------
struct Broker::Session {
  int fd = -1;
  int ep = -1;  // owning epoll fd
  std::string client_id;
  int version = 4;
  bool connected = false;
  bool clean = true;
  std::string in;  // owned by the I/O thread
  std::mutex out_mu;
  std::string out;
  bool want_out = false;
  uint16_t next_id = 1;
  std::set<uint16_t> qos2_in;  // inbound QoS 2 ids awaiting PUBREL (I/O thread only)
  std::atomic<bool> closed{false};

  void send(const std::string& bytes) {
    std::lock_guard<std::mutex> g(out_mu);
    if (closed) return;
    if (out.empty()) {
      size_t off = 0;
      while (off < bytes.size()) {
        const ssize_t k = ::send(fd, bytes.data() + off, bytes.size() - off, MSG_NOSIGNAL);
        if (k > 0) {
          off += (size_t)k;
          continue;
        }
        if (k < 0 && errno == EINTR) continue;
        break;  // EAGAIN or error: buffer the rest
      }
      if (off == bytes.size()) return;
      out.assign(bytes, off, std::string::npos);
    } else {
      out += bytes;
    }
    if (!want_out) {
      want_out = true;
      epoll_event ev{};
      ev.events = EPOLLIN | EPOLLOUT;
      ev.data.fd = fd;
      ::epoll_ctl(ep, EPOLL_CTL_MOD, fd, &ev);
    }
  }
  // EPOLLOUT: drain what is buffered (I/O thread)
  void flush_out() {
    std::lock_guard<std::mutex> g(out_mu);
    size_t off = 0;
    while (off < out.size()) {
      const ssize_t k = ::send(fd, out.data() + off, out.size() - off, MSG_NOSIGNAL);
      if (k > 0) {
        off += (size_t)k;
        continue;
      }
      if (k < 0 && errno == EINTR) continue;
      break;
    }
    out.erase(0, off);
    if (out.empty() && want_out) {
      want_out = false;
      epoll_event ev{};
      ev.events = EPOLLIN;
      ev.data.fd = fd;
      ::epoll_ctl(ep, EPOLL_CTL_MOD, fd, &ev);
    }
  }
  uint16_t alloc_id() {
    std::lock_guard<std::mutex> g(out_mu);
    const uint16_t id = next_id;
    next_id = next_id == 0xffff ? 1 : next_id + 1;
    return id;
  }
};

namespace {
constexpr int kIoThreads = 4;
}

Broker::Broker(BrokerConfig cfg) : cfg_(std::move(cfg)) {
  for (auto& mp : cfg_.mappings) {
    for (auto& f : mp.filters)
      if (!valid_filter(f)) throw Error("mqtt: invalid topic filter in mapping: " + f);
    map_counts_.emplace_back(new std::atomic<uint64_t>(0));
  }
  listen_fd_ = ::socket(AF_INET, SOCK_STREAM, 0);
  if (listen_fd_ < 0) throw Error("mqtt: socket() failed");
  int one = 1;
  ::setsockopt(listen_fd_, SOL_SOCKET, SO_REUSEADDR, &one, sizeof(one));
  sockaddr_in a{};
  a.sin_family = AF_INET;
  a.sin_addr.s_addr = htonl(INADDR_LOOPBACK);
  if (cfg_.port > 0) a.sin_addr.s_addr = htonl(INADDR_ANY);
  a.sin_port = htons((uint16_t)cfg_.port);
  if (::bind(listen_fd_, reinterpret_cast<sockaddr*>(&a), sizeof(a)) != 0 || ::listen(listen_fd_, 1024) != 0) {
    ::close(listen_fd_);
    throw Error("mqtt: bind/listen failed on port " + std::to_string(cfg_.port));
  }
  socklen_t al = sizeof(a);
  ::getsockname(listen_fd_, reinterpret_cast<sockaddr*>(&a), &al);
  port_ = ntohs(a.sin_port);
  running_ = true;
  for (int t = 0; t < kIoThreads; ++t) {
    const int ep = ::epoll_create1(0);
    if (ep < 0) throw Error("mqtt: epoll_create1 failed");
    fds_.push_back(ep);
    workers_.emplace_back([this, ep] {
      std::map<int, std::shared_ptr<Session>> conns;  // fd -> session (this thread's)
      epoll_event evs[64];
      char buf[65536];
      while (running_) {
        const int k = ::epoll_wait(ep, evs, 64, 100);
        for (int e = 0; e < k; ++e) {
          const int fd = evs[e].data.fd;
          auto it = conns.find(fd);
          std::shared_ptr<Session> s;
          if (it == conns.end()) {  // first event of an accepted fd: adopt it
            s = std::make_shared<Session>();
            s->fd = fd;
            s->ep = ep;
            conns[fd] = s;
          } else {
            s = it->second;
          }
          bool drop = (evs[e].events & (EPOLLERR | EPOLLHUP)) != 0;
          if (!drop && (evs[e].events & EPOLLOUT)) s->flush_out();
          if (!drop && (evs[e].events & EPOLLIN)) {
            // bytes that arrived together with the peer's FIN are still handled
            // (a QoS 0 PUBLISH followed by close must not be lost)
            bool eof = false;
            while (true) {
              const ssize_t r = ::recv(fd, buf, sizeof(buf), 0);
              if (r > 0) {
                s->in.append(buf, (size_t)r);
                continue;
              }
              if (r == 0) eof = true;
              else if (errno != EAGAIN && errno != EWOULDBLOCK && errno != EINTR) eof = true;
              break;
            }
            // parse and handle every complete packet
            size_t off = 0;
            try {
              while (!drop) {
                Packet pk;
                const size_t used =
                    parse_packet(reinterpret_cast<const uint8_t*>(s->in.data()) + off, s->in.size() - off, pk);
                if (!used) break;
                off += used;
                // --- protocol ---
                if (!s->connected) {
                  if (pk.type != CONNECT) {
                    drop = true;
                    break;
                  }
                  R r(reinterpret_cast<const uint8_t*>(pk.body.data()), pk.body.size());
                  const std::string proto = r.str();
                  const uint8_t level = r.u8();
                  const uint8_t fl = r.u8();
                  r.u16();  // keep-alive (the broker does not expire idle sessions)
                  if (proto != "MQTT" || (level != 4 && level != 5)) {
                    W w;
                    w.u8(0);
                    w.u8(level == 5 ? 0x84 : 0x01);  // unsupported protocol version
                    if (level == 5) w.props_empty();
                    send_all_blocking(fd, frame(CONNACK, 0, w.s));
                    drop = true;
                    break;
                  }
                  s->version = level;
                  if (level == 5) r.skip_props();
                  std::string cid = r.str();
                  if (fl & 0x04) {  // will message: parsed, not retained by this broker
                    if (level == 5) r.skip_props();
                    r.str();
                    r.str();
                  }
                  std::string user, pass;
                  if (fl & 0x80) user = r.str();
                  if (fl & 0x40) pass = r.str();
                  s->clean = (fl & 0x02) != 0;
                  uint8_t rc = 0;
                  if (!cfg_.username.empty() && (user != cfg_.username || pass != cfg_.password))
                    rc = level == 5 ? 0x86 : 0x04;  // bad user name or password
                  if (cid.empty()) {
                    if (!s->clean && level == 4) rc = 0x02;  // identifier rejected
                    cid = "auto-" + std::to_string(fd) + "-" + std::to_string(now_ms());
                  }
                  bool present = false;
                  if (rc == 0) {
                    std::lock_guard<std::mutex> g(mu_);
                    auto si = sessions_.find(cid);
                    // take-over: close the older connection of this client id.  Its fd is
                    // still open -- a dropping session leaves sessions_ (under mu_) before
                    // its fd is closed -- so the shutdown cannot hit a reused descriptor.
                    if (si != sessions_.end() && si->second.get() != s.get()) ::shutdown(si->second->fd, SHUT_RDWR);
                    sessions_[cid] = s;
                    if (s->clean) subs_.erase(cid);
                    else present = subs_.count(cid) > 0;
                  }
                  s->client_id = cid;
                  W w;
                  w.u8(present ? 1 : 0);
                  w.u8(rc);
                  if (level == 5) w.props_empty();
                  s->send(frame(CONNACK, 0, w.s));
                  if (rc != 0) {
                    drop = true;
                    break;
                  }
                  s->connected = true;
                  conn_cur_++;
                  conn_tot_++;
                  continue;
                }
                switch (pk.type) {
                  case PUBLISH: {
                    Message m = decode_publish(pk, s->version);
                    if (m.topic.empty() || m.topic.find_first_of("+#") != std::string::npos) {
                      drop = true;
                      break;
                    }
                    // the acknowledgement flow follows the QoS the client sent; the routed
                    // (and retained) copy is capped at the broker's maximum QoS
                    const int in_qos = m.qos;
                    if (m.qos > cfg_.max_qos) m.qos = cfg_.max_qos;
                    if (in_qos == 2) {
                      const bool fresh = s->qos2_in.insert(m.packet_id).second;
                      if (fresh) route(m, s->client_id);
                      s->send(ack_packet(PUBREC, m.packet_id));
                    } else {
                      route(m, s->client_id);
                      if (in_qos == 1) s->send(ack_packet(PUBACK, m.packet_id));
                    }
                    break;
                  }
                  case PUBREL: {
                    R r(reinterpret_cast<const uint8_t*>(pk.body.data()), pk.body.size());
                    const uint16_t id = r.u16();
                    s->qos2_in.erase(id);
                    s->send(ack_packet(PUBCOMP, id));
                    break;
                  }
                  case PUBREC: {  // our outbound QoS 2 delivery: release it
                    R r(reinterpret_cast<const uint8_t*>(pk.body.data()), pk.body.size());
                    s->send(ack_packet(PUBREL, r.u16()));
                    break;
                  }
                  case PUBACK:
                  case PUBCOMP:
                    break;  // outbound QoS 1/2 completed (no redelivery store)
                  case SUBSCRIBE: {
                    R r(reinterpret_cast<const uint8_t*>(pk.body.data()), pk.body.size());
                    const uint16_t id = r.u16();
                    if (s->version == 5) r.skip_props();
                    std::vector<uint8_t> codes;
                    std::vector<std::string> plain_filters;
                    std::vector<int> plain_qos;
                    while (!r.done()) {
                      std::string f = r.str();
                      const int q = std::min<int>(r.u8() & 3, cfg_.max_qos);
                      std::string group;
                      if (f.rfind("$share/", 0) == 0) {
                        const size_t sl = f.find('/', 7);
                        if (sl == std::string::npos || sl == 7) {
                          codes.push_back(0x80);
                          continue;
                        }
                        group = f.substr(7, sl - 7);
                        f = f.substr(sl + 1);
                      }
                      if (!valid_filter(f)) {
                        codes.push_back(0x80);
                        continue;
                      }
                      {
                        std::lock_guard<std::mutex> g(mu_);
                        auto& v = subs_[s->client_id];
                        bool found = false;
                        for (auto& sb : v)
                          if (sb.filter == f && sb.share_group == group) {
                            sb.qos = q;
                            found = true;
                          }
                        if (!found) v.push_back(Sub{f, q, group});
                        if (!group.empty()) {
                          auto& sg = shared_[{group, f}];
                          if (std::find(sg.members.begin(), sg.members.end(), s->client_id) == sg.members.end())
                            sg.members.push_back(s->client_id);
                        }
                      }
                      codes.push_back((uint8_t)q);
                      if (group.empty()) {
                        plain_filters.push_back(f);
                        plain_qos.push_back(q);
                      }
                    }
                    W w;
                    w.u16(id);
                    if (s->version == 5) w.props_empty();
                    for (uint8_t c : codes) w.u8(c);
                    s->send(frame(SUBACK, 0, w.s));
                    // retained messages for the new (non-shared) subscriptions
                    std::vector<std::pair<Message, int>> ret;
                    {
                      std::lock_guard<std::mutex> g(mu_);
                      for (size_t k = 0; k < plain_filters.size(); ++k)
                        for (const auto& rm : retained_)
                          if (topic_matches(plain_filters[k], rm.first)) ret.emplace_back(rm.second, plain_qos[k]);
                    }
                    for (auto& rq : ret) {
                      Message m = rq.first;
                      const int q = std::min(m.qos, rq.second);
                      m.qos = q;
                      m.retain = true;
                      m.dup = false;
                      m.packet_id = q > 0 ? s->alloc_id() : 0;
                      s->send(encode_publish(m, s->version));
                      out_pub_++;
                    }
                    break;
                  }
                  case UNSUBSCRIBE: {
                    R r(reinterpret_cast<const uint8_t*>(pk.body.data()), pk.body.size());
                    const uint16_t id = r.u16();
                    if (s->version == 5) r.skip_props();
                    std::vector<uint8_t> codes;
                    while (!r.done()) {
                      std::string f = r.str();
                      std::string group;
                      if (f.rfind("$share/", 0) == 0) {
                        const size_t sl = f.find('/', 7);
                        group = sl == std::string::npos ? "" : f.substr(7, sl - 7);
                        f = sl == std::string::npos ? f : f.substr(sl + 1);
                      }
                      std::lock_guard<std::mutex> g(mu_);
                      auto& v = subs_[s->client_id];
                      const size_t before = v.size();
                      v.erase(std::remove_if(v.begin(), v.end(),
                                             [&](const Sub& sb) { return sb.filter == f && sb.share_group == group; }),
                              v.end());
                      if (!group.empty()) {
                        auto gi = shared_.find({group, f});
                        if (gi != shared_.end()) {
                          auto& mem = gi->second.members;
                          mem.erase(std::remove(mem.begin(), mem.end(), s->client_id), mem.end());
                        }
                      }
                      codes.push_back(v.size() < before ? 0x00 : 0x11);  // success / no subscription existed
                    }
                    W w;
                    w.u16(id);
                    if (s->version == 5) {
                      w.props_empty();
                      for (uint8_t c : codes) w.u8(c);
                    }
                    s->send(frame(UNSUBACK, 0, w.s));
                    break;
                  }
                  case PINGREQ:
                    s->send(frame(PINGRESP, 0, std::string()));
                    break;
                  case DISCONNECT:
                    drop = true;
                    break;
                  default:
                    drop = true;  // protocol error
                }
              }
            } catch (const std::exception&) {
              drop = true;  // malformed packet: close the network connection
            }
            s->in.erase(0, off);
            drop = drop || eof;
          }
          if (drop) {
            ::epoll_ctl(ep, EPOLL_CTL_DEL, fd, nullptr);
            {
              std::lock_guard<std::mutex> g(s->out_mu);
              s->closed = true;
            }
            if (s->connected) {
              conn_cur_--;
              std::lock_guard<std::mutex> g(mu_);
              auto si = sessions_.find(s->client_id);
              if (si != sessions_.end() && si->second.get() == s.get()) {
                sessions_.erase(si);
                if (s->clean) {
                  auto sv = subs_.find(s->client_id);
                  if (sv != subs_.end()) {
                    for (const auto& sb : sv->second)
                      if (!sb.share_group.empty()) {
                        auto gi = shared_.find({sb.share_group, sb.filter});
                        if (gi != shared_.end()) {
                          auto& mem = gi->second.members;
                          mem.erase(std::remove(mem.begin(), mem.end(), s->client_id), mem.end());
                        }
                      }
                    subs_.erase(sv);
                  }
                }
              }
            }
            ::close(fd);
            conns.erase(fd);
          }
        }
      }
      for (auto& c : conns) ::close(c.first);
    });
  }
  accept_thread_ = std::thread([this] { accept_loop(); });
  if (!cfg_.kafka_bootstrap.empty() && !cfg_.mappings.empty()) bridge_thread_ = std::thread([this] { bridge_loop(); });
}

Broker::~Broker() { stop(); }

void Broker::stop() {
  if (!running_.exchange(false)) return;
  ::shutdown(listen_fd_, SHUT_RDWR);
  ::close(listen_fd_);
  if (accept_thread_.joinable()) accept_thread_.join();
  for (auto& t : workers_)
    if (t.joinable()) t.join();
  for (int ep : fds_) ::close(ep);
  bq_cv_.notify_all();
  if (bridge_thread_.joinable()) bridge_thread_.join();
}

void Broker::accept_loop() {
  size_t rr = 0;
  while (running_) {
    pollfd pf{listen_fd_, POLLIN, 0};
    if (::poll(&pf, 1, 100) <= 0) continue;
    const int fd = ::accept(listen_fd_, nullptr, nullptr);
    if (fd < 0) continue;
    int one = 1;
    ::setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
    set_nonblock(fd);
    epoll_event ev{};
    ev.events = EPOLLIN;
    ev.data.fd = fd;
    // the owning I/O thread creates the session on the first event of this fd
    ::epoll_ctl(fds_[rr++ % fds_.size()], EPOLL_CTL_ADD, fd, &ev);
  }
}

void Broker::publish(const Message& m) {
  Message c = m;
  if (c.qos > cfg_.max_qos) c.qos = cfg_.max_qos;
  route(c, std::string());
}

void Broker::route(const Message& m, const std::string& /*from_client*/) {
  in_pub_++;
  // Kafka bridge (kafka-config.yaml topic-mappings): key = MQTT topic, value = payload
  if (!cfg_.kafka_bootstrap.empty()) {
    for (size_t k = 0; k < cfg_.mappings.size(); ++k) {
      bool hit = false;
      for (const auto& f : cfg_.mappings[k].filters) hit = hit || topic_matches(f, m.topic);
      if (!hit) continue;
      std::unique_lock<std::mutex> g(bq_mu_);
      // back-pressure: the publisher's I/O thread waits while the bridge is saturated
      cv_wait_ms(bq_done_cv_, g, 5000, [&] { return bq_.size() < cfg_.bridge_queue_max || !running_; });
      bq_.push_back(BridgeRec{(int)k, m.topic, m.payload, now_ms()});
      b_enq_++;
      g.unlock();
      bq_cv_.notify_one();
    }
  }
  std::vector<std::pair<std::shared_ptr<Session>, int>> targets;
  {
    std::lock_guard<std::mutex> g(mu_);
    if (m.retain) {
      if (m.payload.empty()) retained_.erase(m.topic);
      else retained_[m.topic] = m;
    }
    for (const auto& cs : subs_) {
      int best = -1;
      for (const auto& sb : cs.second)
        if (sb.share_group.empty() && topic_matches(sb.filter, m.topic)) best = std::max(best, sb.qos);
      if (best < 0) continue;
      auto si = sessions_.find(cs.first);
      if (si != sessions_.end()) targets.emplace_back(si->second, best);
    }
    for (auto& gs : shared_) {
      if (!topic_matches(gs.first.second, m.topic)) continue;
      auto& mem = gs.second.members;
      for (size_t tries = 0; tries < mem.size(); ++tries) {  // next connected member, round-robin
        const std::string& cid = mem[gs.second.next++ % mem.size()];
        auto si = sessions_.find(cid);
        if (si == sessions_.end()) continue;
        int q = 0;
        for (const auto& sb : subs_[cid])
          if (sb.share_group == gs.first.first && sb.filter == gs.first.second) q = sb.qos;
        targets.emplace_back(si->second, q);
        break;
      }
    }
  }
  for (auto& t : targets) deliver(t.first, m, t.second);
}

void Broker::deliver(const std::shared_ptr<Session>& s, Message m, int sub_qos) {
  m.qos = std::min(m.qos, sub_qos);
  m.retain = false;  // retain-as-published off: live deliveries clear RETAIN (MQTT 3.3.1.3)
  m.dup = false;
  m.packet_id = m.qos > 0 ? s->alloc_id() : 0;
  s->send(encode_publish(m, s->version));
  out_pub_++;
}

void Broker::bridge_loop() {
  std::unique_ptr<kafka::Client> kc;
  std::map<std::string, int> nparts;
  while (true) {
    std::vector<BridgeRec> batch;
    {
      std::unique_lock<std::mutex> g(bq_mu_);
      cv_wait_ms(bq_cv_, g, 100, [&] { return !bq_.empty() || !running_; });
      if (!running_) {  // stopped: records not yet produced are dropped (flush() first to keep them)
        kafka_failed_ += bq_.size();
        b_done_ += bq_.size();
        bq_.clear();
        break;
      }
      if (bq_.empty()) continue;
      if (cfg_.bridge_linger_ms > 0 && (int)bq_.size() < cfg_.bridge_batch && running_) {  // linger for a fuller batch
        g.unlock();
        std::this_thread::sleep_for(std::chrono::milliseconds(cfg_.bridge_linger_ms));
        g.lock();
      }
      const size_t n = std::min(bq_.size(), (size_t)cfg_.bridge_batch * 8);
      batch.assign(std::make_move_iterator(bq_.begin()), std::make_move_iterator(bq_.begin() + (long)n));
      bq_.erase(bq_.begin(), bq_.begin() + (long)n);
    }
    bq_done_cv_.notify_all();
    size_t failed = 0, sent = 0;
    try {
      if (!kc) kc.reset(new kafka::Client(cfg_.kafka_bootstrap, cfg_.kafka));
      // group by (kafka topic, partition), keep arrival order inside a group
      std::map<std::pair<std::string, int>, std::vector<kafka::Record>> groups;
      std::map<std::pair<std::string, int>, int> gmap;
      for (auto& br : batch) {
        const std::string& kt = cfg_.mappings[(size_t)br.mapping].kafka_topic;
        auto pi = nparts.find(kt);
        if (pi == nparts.end()) {
          kc->refresh_metadata(kt);  // auto-creates the topic like the extension's producer
          const auto all = kc->partitions();
          auto f = all.find(kt);
          pi = nparts.emplace(kt, f == all.end() ? 1 : std::max(1, f->second)).first;
        }
        kafka::Record rec;
        rec.key = br.key;
        rec.key_null = false;
        rec.value = std::move(br.value);
        rec.timestamp = br.ts;
        const auto gk = std::make_pair(kt, kafka_partition(br.key, pi->second));
        groups[gk].push_back(std::move(rec));
        gmap[gk] = br.mapping;
      }
      // A partition's records go out in record batches of at most bridge_batch records and
      // kBridgeBatchBytes bytes (a broker refuses a batch over message.max.bytes, 1 MB by
      // default).  Request j of a topic carries batch j of each of its partitions: one
      // Produce per topic per round, every partition in it.
      using Round = std::vector<std::pair<int, std::vector<kafka::Record>>>;
      std::map<std::string, std::vector<Round>> rounds;
      std::map<std::string, std::vector<std::vector<std::pair<int, size_t>>>> round_counts;   // (mapping, records)
      const size_t max_recs = (size_t)std::max(1, cfg_.bridge_batch);
      for (auto& gr : groups) {
        auto& rs = rounds[gr.first.first];
        auto& rc = round_counts[gr.first.first];
        size_t j = 0, bytes = 0;
        std::vector<kafka::Record> cur;
        auto close_chunk = [&]() {
          if (cur.empty()) return;
          if (rs.size() <= j) {
            rs.emplace_back();
            rc.emplace_back();
          }
          rc[j].emplace_back(gmap[gr.first], cur.size());
          rs[j].emplace_back(gr.first.second, std::move(cur));
          cur.clear();
          bytes = 0;
          ++j;
        };
        for (auto& r : gr.second) {
          const size_t rb = r.value.size() + r.key.size() + 32;   // + record framing
          if (!cur.empty() && (cur.size() >= max_recs || bytes + rb > kBridgeBatchBytes)) close_chunk();
          bytes += rb;
          cur.push_back(std::move(r));
        }
        close_chunk();
      }
      bool broken = false;   // a failed request: this connection's later requests are not tried
      for (auto& tr : rounds) {
        auto& counts = round_counts[tr.first];
        for (size_t j = 0; j < tr.second.size(); ++j) {
          size_t n = 0;
          for (const auto& mc : counts[j]) n += mc.second;
          if (!broken) {
            try {
              kc->produce_multi(tr.first, tr.second[j], 1);
              for (const auto& mc : counts[j]) map_counts_[(size_t)mc.first]->fetch_add(mc.second);
              kafka_sent_ += n;
              sent += n;
              continue;
            } catch (const std::exception&) {
              broken = true;
            }
          }
          failed += n;
        }
      }
      if (broken) {
        kafka_failed_ += failed;
        kc.reset();  // reconnect on the next batch
        nparts.clear();
      }
    } catch (const std::exception&) {   // connect / metadata: nothing of the rest went out
      failed = batch.size() - sent;
      kafka_failed_ += failed;
      kc.reset();
      nparts.clear();
    }
    {
      std::lock_guard<std::mutex> g(bq_mu_);
      b_done_ += batch.size();
    }
    bq_done_cv_.notify_all();
  }
}

bool Broker::flush(int timeout_ms) {
  std::unique_lock<std::mutex> g(bq_mu_);
  const uint64_t target = b_enq_;
  return cv_wait_ms(bq_done_cv_, g, timeout_ms, [&] { return b_done_ >= target; });
}

BrokerStats Broker::stats() {
  BrokerStats st;
  st.incoming_publish = in_pub_;
  st.outgoing_publish = out_pub_;
  st.connections_current = conn_cur_;
  st.connections_total = conn_tot_;
  st.kafka_sent = kafka_sent_;
  st.kafka_failed = kafka_failed_;
  {
    std::lock_guard<std::mutex> g(mu_);
    st.retained = retained_.size();
  }
  {
    std::lock_guard<std::mutex> g(bq_mu_);
    st.kafka_queued = bq_.size();
  }
  return st;
}

std::map<std::string, uint64_t> Broker::mapping_counts() {
  std::map<std::string, uint64_t> out;
  for (size_t k = 0; k < cfg_.mappings.size(); ++k) out[cfg_.mappings[k].id] = map_counts_[k]->load();
  return out;
}

// ---- client ---------------------------------------------------------------------
Client::~Client() {
  if (fd_ >= 0) ::close(fd_);
}

uint16_t Client::alloc_id() {
  const uint16_t id = next_id_;
  next_id_ = next_id_ == 0xffff ? 1 : next_id_ + 1;
  return id;
}

void Client::send_raw(const std::string& s) {
  if (fd_ < 0 || !send_all_blocking(fd_, s)) throw Error("mqtt: send failed (not connected)");
}

bool Client::read_packet(Packet& pk, int timeout_ms) {
  const auto t_end = std::chrono::steady_clock::now() + std::chrono::milliseconds(timeout_ms);
  while (true) {
    const size_t used = parse_packet(reinterpret_cast<const uint8_t*>(rx_.data()), rx_.size(), pk);
    if (used) {
      rx_.erase(0, used);
      return true;
    }
    const int left = (int)std::chrono::duration_cast<std::chrono::milliseconds>(t_end - std::chrono::steady_clock::now())
                         .count();
    if (left <= 0) return false;
    pollfd pf{fd_, POLLIN, 0};
    const int pr = ::poll(&pf, 1, left);
    if (pr <= 0) continue;
    char buf[65536];
    const ssize_t k = ::recv(fd_, buf, sizeof(buf), 0);
    if (k <= 0) {
      if (k < 0 && (errno == EINTR || errno == EAGAIN)) continue;
      ::close(fd_);
      fd_ = -1;
      throw Error("mqtt: connection closed by broker");
    }
    rx_.append(buf, (size_t)k);
  }
}

int Client::connect(const std::string& host, int port, const std::string& client_id, int version,
                    uint16_t keepalive, bool clean, const std::string& username, const std::string& password,
                    int timeout_ms, const std::string& source_ip) {
  if (version != 4 && version != 5) throw Error("mqtt: version must be 4 (3.1.1) or 5");
  if (fd_ >= 0) disconnect();
  addrinfo hints{}, *res = nullptr;
  hints.ai_family = AF_INET;
  hints.ai_socktype = SOCK_STREAM;
  if (::getaddrinfo(host.c_str(), std::to_string(port).c_str(), &hints, &res) != 0 || !res)
    throw Error("mqtt: cannot resolve " + host);
  fd_ = ::socket(res->ai_family, res->ai_socktype, 0);
  if (fd_ < 0) {
    ::freeaddrinfo(res);
    throw Error("mqtt: socket() failed (descriptor limit?)");
  }
  if (!source_ip.empty()) {
    int one = 1;   // port chosen at connect(): ports are then unique per 4-tuple, not per source
    ::setsockopt(fd_, IPPROTO_IP, IP_BIND_ADDRESS_NO_PORT, &one, sizeof(one));
    sockaddr_in src{};
    src.sin_family = AF_INET;
    src.sin_port = 0;
    if (::inet_pton(AF_INET, source_ip.c_str(), &src.sin_addr) != 1 ||
        ::bind(fd_, reinterpret_cast<sockaddr*>(&src), sizeof(src)) != 0) {
      ::close(fd_);
      fd_ = -1;
      ::freeaddrinfo(res);
      throw Error("mqtt: cannot bind source address " + source_ip);
    }
  }
  const int rc = ::connect(fd_, res->ai_addr, res->ai_addrlen);
  ::freeaddrinfo(res);
  if (rc != 0) {
    ::close(fd_);
    fd_ = -1;
    throw Error("mqtt: connect to " + host + ":" + std::to_string(port) + " failed");
  }
  int one = 1;
  ::setsockopt(fd_, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
  version_ = version;
  rx_.clear();
  inbox_.clear();
  send_raw(encode_connect(client_id, version, keepalive, clean, username, password));
  Packet pk;
  if (!read_packet(pk, timeout_ms) || pk.type != CONNACK) throw Error("mqtt: no CONNACK");
  R r(reinterpret_cast<const uint8_t*>(pk.body.data()), pk.body.size());
  session_present_ = (r.u8() & 1) != 0;
  const int code = r.u8();
  if (code != 0) {
    ::close(fd_);
    fd_ = -1;
  }
  return code;
}

void Client::handle_incoming(const Packet& pk) {
  if (pk.type == PUBLISH) {
    Message m = decode_publish(pk, version_);
    if (m.qos == 1) send_raw(ack_packet(PUBACK, m.packet_id));
    if (m.qos == 2) send_raw(ack_packet(PUBREC, m.packet_id));
    inbox_.push_back(std::move(m));
  } else if (pk.type == PUBREL) {
    R r(reinterpret_cast<const uint8_t*>(pk.body.data()), pk.body.size());
    send_raw(ack_packet(PUBCOMP, r.u16()));
  }
}

void Client::publish(const std::string& topic, const std::string& payload, int qos, bool retain) {
  std::lock_guard<std::mutex> g(mu_);
  Message m;
  m.topic = topic;
  m.payload = payload;
  m.qos = qos;
  m.retain = retain;
  m.packet_id = qos > 0 ? alloc_id() : 0;
  send_raw(encode_publish(m, version_));
  if (qos == 0) return;
  const uint8_t want = qos == 1 ? PUBACK : PUBREC;
  for (int stage = 0; stage < (qos == 2 ? 2 : 1); ++stage) {
    const uint8_t w = stage == 0 ? want : PUBCOMP;
    while (true) {
      Packet pk;
      if (!read_packet(pk, 10000)) throw Error("mqtt: publish acknowledgement timed out");
      if (pk.type == w) {
        R r(reinterpret_cast<const uint8_t*>(pk.body.data()), pk.body.size());
        if (r.u16() != m.packet_id) continue;
        if (w == PUBREC) send_raw(ack_packet(PUBREL, m.packet_id));
        break;
      }
      handle_incoming(pk);
    }
  }
}

std::vector<int> Client::subscribe(const std::vector<std::pair<std::string, int>>& filters) {
  std::lock_guard<std::mutex> g(mu_);
  const uint16_t id = alloc_id();
  send_raw(encode_subscribe(id, filters, version_));
  while (true) {
    Packet pk;
    if (!read_packet(pk, 10000)) throw Error("mqtt: SUBACK timed out");
    if (pk.type != SUBACK) {
      handle_incoming(pk);
      continue;
    }
    R r(reinterpret_cast<const uint8_t*>(pk.body.data()), pk.body.size());
    if (r.u16() != id) continue;
    if (version_ == 5) r.skip_props();
    std::vector<int> codes;
    while (!r.done()) codes.push_back(r.u8());
    return codes;
  }
}

void Client::unsubscribe(const std::vector<std::string>& filters) {
  std::lock_guard<std::mutex> g(mu_);
  const uint16_t id = alloc_id();
  W w;
  w.u16(id);
  if (version_ == 5) w.props_empty();
  for (const auto& f : filters) w.str(f);
  send_raw(frame(UNSUBSCRIBE, 0x2, w.s));
  while (true) {
    Packet pk;
    if (!read_packet(pk, 10000)) throw Error("mqtt: UNSUBACK timed out");
    if (pk.type == UNSUBACK) return;
    handle_incoming(pk);
  }
}

bool Client::receive(Message& out, int timeout_ms) {
  std::lock_guard<std::mutex> g(mu_);
  const auto t_end = std::chrono::steady_clock::now() + std::chrono::milliseconds(timeout_ms);
  while (inbox_.empty()) {
    const int left = (int)std::chrono::duration_cast<std::chrono::milliseconds>(t_end - std::chrono::steady_clock::now())
                         .count();
    if (left <= 0) return false;
    Packet pk;
    if (!read_packet(pk, left)) return false;
    handle_incoming(pk);
  }
  out = std::move(inbox_.front());
  inbox_.pop_front();
  return true;
}

bool Client::ping(int timeout_ms) {
  std::lock_guard<std::mutex> g(mu_);
  send_raw(frame(PINGREQ, 0, std::string()));
  while (true) {
    Packet pk;
    if (!read_packet(pk, timeout_ms)) return false;
    if (pk.type == PINGRESP) return true;
    handle_incoming(pk);
  }
}

void Client::disconnect() {
  std::lock_guard<std::mutex> g(mu_);
  if (fd_ < 0) return;
  std::string body;
  if (version_ == 5) {
    body.push_back('\0');  // normal disconnection
    body.push_back('\0');  // no properties
  }
  send_all_blocking(fd_, frame(DISCONNECT, 0, body));
  ::shutdown(fd_, SHUT_WR);
  ::close(fd_);
  fd_ = -1;
}

// ---- device simulator ---------------------------------------------------------------
namespace {
const char* kSensorFields[18] = {
    "coolant_temp", "intake_air_temp", "intake_air_flow_speed", "battery_percentage", "battery_voltage",
    "current_draw", "speed", "engine_vibration_amplitude", "throttle_pos", "tire_pressure11", "tire_pressure12",
    "tire_pressure21", "tire_pressure22", "accelerometer11_value", "accelerometer12_value",
    "accelerometer21_value", "accelerometer22_value", "control_unit_firmware"};

uint64_t splitmix(uint64_t& x) {
  uint64_t z = (x += 0x9E3779B97F4A7C15ull);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
double unif(uint64_t& st) { return (double)(splitmix(st) >> 11) * (1.0 / 9007199254740992.0); }

std::string client_name(const SimConfig& c, uint64_t i) {
  std::string num = std::to_string(i + (uint64_t)c.id_offset);
  if ((int)num.size() < c.id_digits) num = std::string((size_t)(c.id_digits - (int)num.size()), '0') + num;
  return c.client_prefix + num;
}
}  // namespace

std::string car_payload_json(const SimConfig& cfg, uint64_t car, uint64_t seq, int64_t ts_ms, int64_t sent_ns) {
  // each car has a stable operating point (seeded by car id) plus per-event noise
  uint64_t cst = cfg.seed * 0x100000001B3ull + car * 0x9E3779B97F4A7C15ull + 1;
  uint64_t est = cst ^ (seq * 0xD1B54A32D192ED03ull + 7);
  std::string s = "{";
  for (int f = 0; f < 18; ++f) {
    const double lo = f < (int)cfg.lo.size() ? cfg.lo[(size_t)f] : 0.0;
    const double hi = f < (int)cfg.hi.size() ? cfg.hi[(size_t)f] : 1.0;
    const double point = 0.15 + 0.7 * unif(cst);
    // sum of uniforms ~ approx normal noise, sd ~0.05 of the range
    const double noise = (unif(est) + unif(est) + unif(est) - 1.5) * 0.1;
    double u = std::min(1.0, std::max(0.0, point + noise));
    double v = lo + u * (hi - lo);
    char buf[64];
    const bool isint = f < (int)cfg.is_int.size() && cfg.is_int[(size_t)f];
    if (std::string(kSensorFields[f]) == "control_unit_firmware") {
      std::snprintf(buf, sizeof(buf), "%d", point > 0.5 ? 2000 : 1000);
    } else if (isint) {
      std::snprintf(buf, sizeof(buf), "%d", (int)std::lround(v));
    } else {
      std::snprintf(buf, sizeof(buf), "%.6g", v);
    }
    s += "\"";
    s += kSensorFields[f];
    s += "\":";
    s += buf;
    s += ",";
  }
  const bool fail = unif(est) < cfg.failure_rate;
  s += "\"failure_occurred\":\"";
  s += fail ? "true" : "false";
  s += "\",\"timestamp\":" + std::to_string(ts_ms);
  if (sent_ns >= 0) s += ",\"sent_ns\":" + std::to_string(sent_ns);
  s += "}";
  return s;
}

SimStats simulate(const SimConfig& cfg, std::atomic<bool>* stop) {
  SimStats st;
  std::atomic<uint64_t> connected{0}, cfail{0}, published{0}, acked{0}, pfail{0}, late{0};
  using Clock = std::chrono::steady_clock;
  const auto t0 = Clock::now();
  const int T = std::max(1, std::min(cfg.threads, cfg.clients));
  std::vector<std::thread> th;
  std::atomic<int> conn_done{0};
  std::atomic<int64_t> conn_end_ns{0}, first_pub_ns{INT64_MAX}, last_pub_ns{0}, max_lag_ns{0};
  auto ns_since = [&](Clock::time_point t) {
    return (int64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(t - t0).count();
  };
  auto atomic_max = [](std::atomic<int64_t>& a, int64_t v) {
    int64_t cur = a.load();
    while (v > cur && !a.compare_exchange_weak(cur, v)) {
    }
  };
  auto atomic_min = [](std::atomic<int64_t>& a, int64_t v) {
    int64_t cur = a.load();
    while (v < cur && !a.compare_exchange_weak(cur, v)) {
    }
  };
  for (int t = 0; t < T; ++t) {
    th.emplace_back([&, t] {
      const int lo = (int)((int64_t)cfg.clients * t / T), hi = (int)((int64_t)cfg.clients * (t + 1) / T);
      std::vector<std::unique_ptr<Client>> cl((size_t)(hi - lo));
      auto at = [&](double sec) { return t0 + std::chrono::microseconds((int64_t)(sec * 1e6)); };
      // connect stage: client i at ramp * i / clients
      for (int i = lo; i < hi; ++i) {
        if (stop && *stop) break;
        if (cfg.ramp_s > 0) std::this_thread::sleep_until(at(cfg.ramp_s * i / std::max(1, cfg.clients)));
        auto c = std::make_unique<Client>();
        const std::string& src =
            cfg.source_ips.empty() ? std::string() : cfg.source_ips[(size_t)i % cfg.source_ips.size()];
        try {
          if (c->connect(cfg.host, cfg.port, client_name(cfg, (uint64_t)i), cfg.version, 60, true, cfg.username,
                         cfg.password, 5000, src) == 0) {
            connected++;
            cl[(size_t)(i - lo)] = std::move(c);
            continue;
          }
        } catch (const std::exception&) {
        }
        cfail++;
      }
      atomic_max(conn_end_ns, ns_since(Clock::now()));
      Clock::time_point pub0 = t0 + std::chrono::microseconds((int64_t)(cfg.ramp_s * 1e6));
      if (cfg.paced) {   // every thread of this process connected, then one common start
        conn_done++;
        while (conn_done.load() < T && !(stop && *stop)) std::this_thread::sleep_for(std::chrono::microseconds(200));
        pub0 = t0 + std::chrono::nanoseconds(conn_end_ns.load()) + std::chrono::milliseconds(20);
        if (cfg.start_at_unix > 0) {
          const double now_unix = std::chrono::duration<double>(std::chrono::system_clock::now().time_since_epoch()).count();
          pub0 = std::max(pub0, Clock::now() + std::chrono::microseconds((int64_t)((cfg.start_at_unix - now_unix) * 1e6)));
        }
      }
      // publish stage: message k of client i at its offset + k * interval
      for (int k = 0; k < cfg.messages_per_client; ++k) {
        for (int i = lo; i < hi; ++i) {
          if (stop && *stop) return;
          Client* c = cl[(size_t)(i - lo)].get();
          if (!c || !c->connected()) continue;
          const double off = cfg.paced ? cfg.interval_s * (i + 0.5) / std::max(1, cfg.clients)
                                       : cfg.ramp_s * i / std::max(1, cfg.clients);
          const auto due = pub0 + std::chrono::microseconds((int64_t)((off + k * cfg.interval_s) * 1e6));
          std::this_thread::sleep_until(due);
          const auto now = Clock::now();
          if (cfg.paced) {
            const int64_t lag = (int64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(now - due).count();
            atomic_max(max_lag_ns, lag);
            if (lag > 10000000) late++;
          }
          const std::string name = client_name(cfg, (uint64_t)i);
          const int64_t sent = cfg.stamp_ns
                                   ? (int64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(
                                         Clock::now().time_since_epoch())
                                         .count()
                                   : -1;
          try {
            c->publish(cfg.topic_prefix + name,
                       car_payload_json(cfg, (uint64_t)(i + cfg.id_offset), (uint64_t)k, now_ms(), sent), cfg.qos);
            published++;
            if (cfg.qos > 0) acked++;
            const int64_t tn = ns_since(Clock::now());
            atomic_min(first_pub_ns, tn);
            atomic_max(last_pub_ns, tn);
          } catch (const std::exception&) {
            pfail++;
          }
        }
      }
      for (auto& c : cl)
        if (c) try {
            c->disconnect();
          } catch (const std::exception&) {
          }
    });
  }
  for (auto& x : th) x.join();
  st.connected = connected;
  st.connect_failed = cfail;
  st.published = published;
  st.acked = acked;
  st.publish_failed = pfail;
  st.elapsed_s = std::chrono::duration<double>(Clock::now() - t0).count();
  st.connect_s = (double)conn_end_ns.load() * 1e-9;
  st.publish_s = last_pub_ns.load() > first_pub_ns.load() ? (double)(last_pub_ns - first_pub_ns) * 1e-9 : 0.0;
  st.max_lag_ms = (double)max_lag_ns.load() * 1e-6;
  st.late_10ms = late;
  return st;
}

}  // namespace mqtt
}  // namespace sml
