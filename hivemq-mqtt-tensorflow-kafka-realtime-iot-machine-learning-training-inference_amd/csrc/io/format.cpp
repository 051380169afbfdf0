#include "format.h"

#include <algorithm>
#include <charconv>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <vector>

namespace sml {
namespace fmt {
namespace {

// Shortest round-trip decimal digits of v (|v| > 0, finite): v = 0.DIGITS x 10^decpt.
template <typename T>
void shortest(T v, std::string& digits, int& decpt) {
  char b[64];
  const auto r = std::to_chars(b, b + sizeof(b), v, std::chars_format::scientific);
  const char* p = b;
  const char* e = r.ptr;
  if (*p == '-') ++p;
  digits.clear();
  for (; p < e && *p != 'e'; ++p)
    if (*p != '.') digits.push_back(*p);
  int ex = 0;
  std::from_chars(p + 1 + (p[1] == '+'), e, ex);
  decpt = ex + 1;
}

// positional text of 0.DIGITS x 10^decpt: "int.frac" (frac may be empty)
void positional(const std::string& d, int decpt, std::string& ip, std::string& fp) {
  const int n = (int)d.size();
  if (decpt <= 0) {
    ip = "0";
    fp.assign((size_t)(-decpt), '0');
    fp += d;
  } else if (decpt >= n) {
    ip = d;
    ip.append((size_t)(decpt - n), '0');
    fp.clear();
  } else {
    ip = d.substr(0, (size_t)decpt);
    fp = d.substr((size_t)decpt);
  }
}

void trim_zeros(std::string& fp) {
  while (!fp.empty() && fp.back() == '0') fp.pop_back();
}

struct Parts {
  std::string ip, fp, ex;   // int part (with sign), fraction digits, exponent text ("+01")
};

// numpy dragon4_positional(x, precision=8, unique=True, fractional=True, trim='.')
void pos_unique(float x, Parts& o) {
  const bool neg = std::signbit(x);
  if (x == 0.0f) {
    o.ip = neg ? "-0" : "0";
    o.fp.clear();
    return;
  }
  std::string d;
  int decpt;
  shortest<float>(std::fabs(x), d, decpt);
  positional(d, decpt, o.ip, o.fp);
  if (decpt > (int)d.size()) {
    // Dragon4 prints every digit left of the point exactly (52271352., not the
    // shortest-digits 52271350.); such a float is an integer, so %.0f is exact
    char b[64];
    std::snprintf(b, sizeof(b), "%.0f", (double)std::fabs(x));
    o.ip = b;
  } else if (o.fp.size() > 8) {   // cut off at 8 fractional digits, correctly rounded
    char b[80];
    std::snprintf(b, sizeof(b), "%.8f", (double)std::fabs(x));
    const char* dot = std::strchr(b, '.');
    o.ip.assign(b, (size_t)(dot - b));
    o.fp.assign(dot + 1);
    trim_zeros(o.fp);
  }
  if (neg) o.ip.insert(o.ip.begin(), '-');
}

// numpy dragon4_scientific(x, precision=8, unique=True, trim='.')
void sci_unique(float x, Parts& o) {
  const bool neg = std::signbit(x);
  int ex = 0;
  if (x == 0.0f) {
    o.ip = "0";
    o.fp.clear();
  } else {
    std::string d;
    int decpt;
    shortest<float>(std::fabs(x), d, decpt);
    ex = decpt - 1;
    o.ip = d.substr(0, 1);
    o.fp = d.substr(1);
    if (o.fp.size() > 8) {
      char b[80];
      std::snprintf(b, sizeof(b), "%.8e", (double)std::fabs(x));
      const char* dot = std::strchr(b, '.');
      const char* e = std::strchr(b, 'e');
      o.ip.assign(b, (size_t)(dot - b));
      o.fp.assign(dot + 1, (size_t)(e - dot - 1));
      ex = std::atoi(e + 1);
      trim_zeros(o.fp);
    }
  }
  if (neg) o.ip.insert(o.ip.begin(), '-');
  char eb[16];
  std::snprintf(eb, sizeof(eb), "%c%02d", ex < 0 ? '-' : '+', ex < 0 ? -ex : ex);
  o.ex = eb;
}

}  // namespace

void py_float_repr(double v, std::string& out) {
  if (std::isnan(v)) {
    out += "NaN";
    return;
  }
  if (std::isinf(v)) {
    out += v < 0 ? "-Infinity" : "Infinity";
    return;
  }
  if (std::signbit(v)) out.push_back('-');
  if (v == 0.0) {
    out += "0.0";
    return;
  }
  std::string d;
  int decpt;
  shortest<double>(std::fabs(v), d, decpt);
  if (decpt > -4 && decpt <= 16) {
    std::string ip, fp;
    positional(d, decpt, ip, fp);
    out += ip;
    out.push_back('.');
    out += fp.empty() ? "0" : fp;
  } else {
    out.push_back(d[0]);
    if (d.size() > 1) {
      out.push_back('.');
      out.append(d, 1, std::string::npos);
    }
    const int ex = decpt - 1;
    char eb[16];
    std::snprintf(eb, sizeof(eb), "e%c%02d", ex < 0 ? '-' : '+', ex < 0 ? -ex : ex);
    out += eb;
  }
}

void array2string_f32(const float* v, int n, std::string& out) {
  // ---- FloatingFormat.fillFormat ----
  bool any_finite = false, exp_format = false, neginf = false, nonfinite = false;
  float maxv = 0.0f, minv = 0.0f;
  bool have_nz = false;
  for (int i = 0; i < n; ++i) {
    const float x = v[i];
    if (!std::isfinite(x)) {
      nonfinite = true;
      if (std::isinf(x) && x < 0) neginf = true;
      continue;
    }
    any_finite = true;
    if (x != 0.0f) {
      const float a = std::fabs(x);
      if (!have_nz) {
        maxv = minv = a;
        have_nz = true;
      } else {
        maxv = std::max(maxv, a);
        minv = std::min(minv, a);
      }
    }
  }
  // numpy compares the float32 extremes against float32 constants (NEP 50 weak scalars)
  if (have_nz && (maxv >= 1.0e8f || minv < 0.0001f || maxv / minv > 1000.0f)) exp_format = true;
  std::vector<Parts> parts((size_t)n);
  int pad_left = 0, pad_right = 0, precision = 0, exp_size = -1;
  if (any_finite) {
    if (exp_format) {
      int ex_len = 0;
      for (int i = 0; i < n; ++i)
        if (std::isfinite(v[i])) {
          sci_unique(v[i], parts[(size_t)i]);
          precision = std::max(precision, (int)parts[(size_t)i].fp.size());
          pad_left = std::max(pad_left, (int)parts[(size_t)i].ip.size());
          ex_len = std::max(ex_len, (int)parts[(size_t)i].ex.size());
        }
      exp_size = ex_len - 1;
      pad_right = exp_size + 2 + precision;
      // final pass: exactly `precision` digits (unique + min_digits == printf rounding)
      for (int i = 0; i < n; ++i)
        if (std::isfinite(v[i])) {
          char b[96];
          std::snprintf(b, sizeof(b), "%.*e", precision, (double)std::fabs(v[i]));
          const char* dot = std::strchr(b, '.');
          const char* e = std::strchr(b, 'e');
          Parts& p = parts[(size_t)i];
          p.ip.assign(b, (size_t)((dot ? dot : e) - b));
          p.fp = dot ? std::string(dot + 1, (size_t)(e - dot - 1)) : std::string();
          if (std::signbit(v[i])) p.ip.insert(p.ip.begin(), '-');
          const int ex = std::atoi(e + 1);
          char eb[16];
          std::snprintf(eb, sizeof(eb), "%c%0*d", ex < 0 ? '-' : '+', exp_size, ex < 0 ? -ex : ex);
          p.ex = eb;
        }
    } else {
      for (int i = 0; i < n; ++i)
        if (std::isfinite(v[i])) {
          pos_unique(v[i], parts[(size_t)i]);
          pad_left = std::max(pad_left, (int)parts[(size_t)i].ip.size());
          pad_right = std::max(pad_right, (int)parts[(size_t)i].fp.size());
        }
    }
  }
  if (nonfinite) {
    const int offset = pad_right + 1;
    pad_left = std::max({pad_left, 3 - offset, 3 + (neginf ? 1 : 0) - offset});
  }
  // ---- format every element ----
  std::vector<std::string> words((size_t)n);
  for (int i = 0; i < n; ++i) {
    std::string& w = words[(size_t)i];
    const float x = v[i];
    if (!std::isfinite(x)) {
      const char* r = std::isnan(x) ? "nan" : (x < 0 ? "-inf" : "inf");
      const int pad = pad_left + pad_right + 1 - (int)std::strlen(r);
      if (pad > 0) w.assign((size_t)pad, ' ');
      w += r;
      continue;
    }
    const Parts& p = parts[(size_t)i];
    if ((int)p.ip.size() < pad_left) w.assign((size_t)(pad_left - (int)p.ip.size()), ' ');
    w += p.ip;
    w.push_back('.');
    w += p.fp;
    if (exp_format) {
      w.push_back('e');
      w += p.ex;
    } else if ((int)p.fp.size() < pad_right) {
      w.append((size_t)(pad_right - (int)p.fp.size()), ' ');
    }
  }
  // ---- _formatArray, 1-D: linewidth 75, separator ' ', hanging indent ' ' ----
  const size_t elem_width = 75 - 1;
  std::string s, line = " ";
  auto extend = [&](const std::string& word) {
    if (line.size() + word.size() > elem_width && line.size() > 1) {
      size_t e = line.size();
      while (e > 0 && line[e - 1] == ' ') --e;
      s.append(line, 0, e);
      s.push_back('\n');
      line = " ";
    }
    line += word;
  };
  for (int i = 0; i + 1 < n; ++i) {
    extend(words[(size_t)i]);
    line.push_back(' ');
  }
  if (n > 0) extend(words[(size_t)n - 1]);
  s += line;
  out.push_back('[');
  out.append(s, 1, std::string::npos);
  out.push_back(']');
}

void json_string(const uint8_t* p, size_t n, std::string& out) {
  static const char* hex = "0123456789abcdef";
  auto u4 = [&](unsigned c) {
    out += "\\u";
    out.push_back(hex[(c >> 12) & 15]);
    out.push_back(hex[(c >> 8) & 15]);
    out.push_back(hex[(c >> 4) & 15]);
    out.push_back(hex[c & 15]);
  };
  out.push_back('"');
  for (size_t i = 0; i < n;) {
    const uint8_t c = p[i];
    if (c < 0x80) {
      ++i;
      switch (c) {
        case '"': out += "\\\""; break;
        case '\\': out += "\\\\"; break;
        case '\n': out += "\\n"; break;
        case '\r': out += "\\r"; break;
        case '\t': out += "\\t"; break;
        case '\b': out += "\\b"; break;
        case '\f': out += "\\f"; break;
        default:
          if (c < 0x20) u4(c);
          else out.push_back((char)c);
      }
      continue;
    }
    // UTF-8 sequence -> code point (keys are str on the Python side: valid UTF-8)
    unsigned cp = 0;
    int len = c >= 0xF0 ? 4 : c >= 0xE0 ? 3 : 2;
    cp = c & (len == 4 ? 0x07 : len == 3 ? 0x0F : 0x1F);
    for (int k = 1; k < len && i + (size_t)k < n; ++k) cp = (cp << 6) | (p[i + (size_t)k] & 0x3F);
    i += (size_t)len;
    if (cp >= 0x10000) {
      cp -= 0x10000;
      u4(0xD800 + (cp >> 10));
      u4(0xDC00 + (cp & 0x3FF));
    } else {
      u4(cp);
    }
  }
  out.push_back('"');
}

void score_record_json(const uint8_t* key, int64_t key_len, int partition, int64_t offset, float score, bool anomaly,
                       const float* recon, int D, std::string& out) {
  out += "{\"car\": ";
  if (key_len < 0) out += "null";
  else json_string(key, (size_t)key_len, out);
  char b[64];
  std::snprintf(b, sizeof(b), ", \"partition\": %d, \"offset\": %lld, \"score\": ", partition, (long long)offset);
  out += b;
  py_float_repr((double)score, out);
  out += anomaly ? ", \"anomaly\": true" : ", \"anomaly\": false";
  if (recon) {
    out += ", \"reconstruction\": ";
    std::string a;
    array2string_f32(recon, D, a);
    json_string(reinterpret_cast<const uint8_t*>(a.data()), a.size(), out);
  }
  out.push_back('}');
}

}  // namespace fmt
}  // namespace sml
