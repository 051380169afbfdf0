#include "jsonrow.h"

#include <algorithm>
#include <charconv>
#include <cmath>
#include <cstring>
#include <stdexcept>

#include "feed.h"

namespace sml {
namespace jsonrow {
namespace {

inline uint64_t fnv_step(uint64_t h, uint8_t c) { return (h ^ c) * 0x100000001B3ull; }
constexpr uint64_t kFnv0 = 0xCBF29CE484222325ull;

inline const uint8_t* ws(const uint8_t* p, const uint8_t* e) {
  while (p < e && (*p == ' ' || *p == '\t' || *p == '\n' || *p == '\r')) ++p;
  return p;
}

// end of a JSON string whose opening quote is at p[-1]: pointer to the closing quote (or e)
inline const uint8_t* str_end(const uint8_t* p, const uint8_t* e) {
  while (p < e && *p != '"') p += (*p == '\\') ? 2 : 1;
  return p < e ? p : e;
}

// skip one nested object / array starting at p ('{' or '['); returns past its end, or e
const uint8_t* skip_nested(const uint8_t* p, const uint8_t* e) {
  int depth = 0;
  while (p < e) {
    const uint8_t c = *p++;
    if (c == '"') {
      p = str_end(p, e);
      if (p < e) ++p;
    } else if (c == '{' || c == '[') {
      ++depth;
    } else if (c == '}' || c == ']') {
      if (--depth == 0) return p;
    }
  }
  return e;
}

bool parse_double(const uint8_t* p, const uint8_t* e, double& v) {
  p = ws(p, e);
  if (p < e && *p == '+') ++p;   // from_chars takes no leading '+'
  const auto r = std::from_chars(reinterpret_cast<const char*>(p), reinterpret_cast<const char*>(e), v);
  return r.ec == std::errc();
}

bool parse_i64(const uint8_t* p, const uint8_t* e, int64_t& v) {
  p = ws(p, e);
  if (p < e && *p == '+') ++p;
  const auto r = std::from_chars(reinterpret_cast<const char*>(p), reinterpret_cast<const char*>(e), v);
  if (r.ec == std::errc() && (r.ptr == reinterpret_cast<const char*>(e) || (*r.ptr != '.' && *r.ptr != 'e' &&
                                                                           *r.ptr != 'E')))
    return true;
  double d;   // "1.7e18" or "123.0": through double
  if (!parse_double(p, e, d) || !std::isfinite(d)) return false;
  v = (int64_t)d;
  return true;
}

}  // namespace

std::string canonical(const std::string& key) {
  std::string out;
  for (char c : key) {
    if (c == '_') continue;
    out.push_back((c >= 'A' && c <= 'Z') ? (char)(c | 0x20) : c);
  }
  return out;
}

Plan::Plan(const std::vector<std::pair<std::string, int>>& columns, const std::string& label_key,
           const std::string& stamp_key) {
  for (const auto& kv : columns) {
    if (kv.second < 0 || kv.second > 4096) throw std::invalid_argument("jsonrow: column out of range");
    add(kv.first, (int16_t)kv.second);
    width_ = std::max(width_, kv.second + 1);
  }
  if (!label_key.empty()) add(label_key, kLabel);
  if (!stamp_key.empty()) add(stamp_key, kStamp);
}

void Plan::add(const std::string& key, int16_t target) {
  const std::string c = canonical(key);
  if (c.empty() || c.size() >= sizeof(Slot::key)) throw std::invalid_argument("jsonrow: key too long: " + key);
  uint64_t h = kFnv0;
  for (char ch : c) h = fnv_step(h, (uint8_t)ch);
  for (int i = 0; i < kSlots; ++i) {
    Slot& s = slots_[(h + (uint64_t)i) & (kSlots - 1)];
    if (s.target == -1) {
      s.h = h;
      s.len = (uint8_t)c.size();
      std::memcpy(s.key, c.data(), c.size());
      s.target = target;
      return;
    }
    if (s.h == h && s.len == c.size() && std::memcmp(s.key, c.data(), c.size()) == 0)
      throw std::invalid_argument("jsonrow: duplicate key " + key);
  }
  throw std::invalid_argument("jsonrow: too many keys");
}

const Plan::Slot* Plan::find(const char* k, size_t n, uint64_t h) const {
  for (int i = 0; i < kSlots; ++i) {
    const Slot& s = slots_[(h + (uint64_t)i) & (kSlots - 1)];
    if (s.target == -1) return nullptr;
    if (s.h == h && s.len == n && std::memcmp(s.key, k, n) == 0) return &s;
  }
  return nullptr;
}

bool Plan::decode(const uint8_t* p, size_t n, float* row, uint8_t* label, int64_t* stamp) const {
  for (int c = 0; c < width_; ++c) row[c] = NAN;
  *label = 2;
  if (stamp) *stamp = 0;
  const uint8_t* e = p + n;
  p = ws(p, e);
  if (p >= e || *p != '{') return false;
  p = ws(p + 1, e);
  if (p < e && *p == '}') return true;
  char key[sizeof(Slot::key)];
  while (p < e) {
    if (*p != '"') return false;
    ++p;
    // key: canonicalised and hashed on the fly
    size_t kn = 0;
    bool fits = true;
    uint64_t h = kFnv0;
    while (p < e && *p != '"') {
      uint8_t c = *p;
      if (c == '\\') {   // escaped key character: take it literally
        if (++p >= e) return false;
        c = *p;
      }
      ++p;
      if (c == '_') continue;
      if (c >= 'A' && c <= 'Z') c |= 0x20;
      if (kn + 1 < sizeof(key)) key[kn++] = (char)c;
      else fits = false;
      h = fnv_step(h, c);
    }
    if (p >= e) return false;
    p = ws(p + 1, e);
    if (p >= e || *p != ':') return false;
    p = ws(p + 1, e);
    if (p >= e) return false;
    const Slot* s = fits ? find(key, kn, h) : nullptr;
    const int16_t tgt = s ? s->target : (int16_t)-1;
    const uint8_t c0 = *p;
    if (c0 == '"') {
      const uint8_t* a = p + 1;
      const uint8_t* b = str_end(a, e);
      if (b >= e) return false;
      if (tgt == kLabel) {
        *label = feed::label_code(a, (size_t)(b - a));
      } else if (tgt == kStamp) {
        int64_t v;
        if (stamp && parse_i64(a, b, v)) *stamp = v;
      } else if (tgt >= 0) {
        double v;
        row[tgt] = parse_double(a, b, v) ? (float)v : NAN;
      }
      p = b + 1;
    } else if (c0 == '{' || c0 == '[') {
      p = skip_nested(p, e);
    } else if (c0 == 'n' || c0 == 't' || c0 == 'f') {   // null / true / false
      const size_t len = c0 == 'f' ? 5 : 4;
      if ((size_t)(e - p) < len) return false;
      if (tgt == kLabel && c0 != 'n') *label = c0 == 't' ? 1 : 0;
      else if (tgt >= 0) row[tgt] = c0 == 'n' ? NAN : (c0 == 't' ? 1.f : 0.f);
      p += len;
    } else {   // number
      const uint8_t* a = p;
      while (p < e && ((*p >= '0' && *p <= '9') || *p == '-' || *p == '+' || *p == '.' || *p == 'e' || *p == 'E'))
        ++p;
      if (p == a) return false;
      if (tgt == kStamp) {
        int64_t v;
        if (stamp && parse_i64(a, p, v)) *stamp = v;
      } else if (tgt >= 0) {
        double v;
        row[tgt] = parse_double(a, p, v) ? (float)v : NAN;
      }
    }
    p = ws(p, e);
    if (p >= e) return false;
    if (*p == '}') return true;
    if (*p != ',') return false;
    p = ws(p + 1, e);
  }
  return false;
}

}  // namespace jsonrow
}  // namespace sml
