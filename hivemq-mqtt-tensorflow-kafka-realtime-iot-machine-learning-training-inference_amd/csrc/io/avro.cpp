// Columnar Avro binary codec + Confluent wire framing (see avro.h).
#include "avro.h"

#include <cmath>
#include <cstring>

namespace sml {
namespace avro {

size_t read_varlong(const uint8_t* p, size_t n, int64_t* out) {
  uint64_t v = 0;
  int shift = 0;
  for (size_t i = 0; i < n && i < 10; ++i) {
    const uint8_t b = p[i];
    v |= (uint64_t)(b & 0x7f) << shift;
    if (!(b & 0x80)) {
      *out = (int64_t)((v >> 1) ^ (~(v & 1) + 1));  // zigzag decode
      return i + 1;
    }
    shift += 7;
  }
  return 0;  // truncated / overlong
}

void write_varlong(std::string& out, int64_t v) {
  uint64_t z = ((uint64_t)v << 1) ^ (uint64_t)(v >> 63);  // zigzag encode
  while (z >= 0x80) {
    out.push_back((char)((z & 0x7f) | 0x80));
    z >>= 7;
  }
  out.push_back((char)z);
}

Codec::Codec(std::vector<Field> fields) : fields_(std::move(fields)) {
  col_.assign(fields_.size(), -1);
  for (size_t i = 0; i < fields_.size(); ++i) {
    const Field& f = fields_[i];
    if (f.kind < K_NULL || f.kind > K_FIXED) throw Error("avro: bad field kind for " + f.name);
    if (f.null_branch > 1) throw Error("avro: only 2-branch [null, T] unions are supported (" + f.name + ")");
    if (f.kind == K_FIXED && f.fixed_size <= 0) throw Error("avro: fixed field needs a size (" + f.name + ")");
    if (f.is_numeric()) col_[i] = (int)n_num_++;
    else if (f.is_text()) col_[i] = (int)n_txt_++;
  }
}

namespace {
struct Cursor {
  const uint8_t* p;
  size_t n;
  size_t i = 0;
  bool varlong(int64_t* v) {
    const size_t k = read_varlong(p + i, n - i, v);
    if (!k) return false;
    i += k;
    return true;
  }
  bool bytes(size_t k, const uint8_t** out) {
    if (k > n - i) return false;
    *out = p + i;
    i += k;
    return true;
  }
};
}  // namespace

bool Codec::decode_one(const uint8_t* p, size_t n, float* num_row, double* num64_row, uint8_t* null_row,
                       DecodedBatch& out, size_t row) const {
  Cursor c{p, n};
  for (size_t fi = 0; fi < fields_.size(); ++fi) {
    const Field& f = fields_[fi];
    const int col = col_[fi];
    bool is_null = false;
    if (f.null_branch >= 0) {
      int64_t br;
      if (!c.varlong(&br) || br < 0 || br > 1) return false;
      is_null = (br == f.null_branch);
    }
    if (f.kind == K_NULL) is_null = true;
    if (is_null) {
      if (f.is_numeric()) {
        num_row[col] = NAN;
        if (num64_row) num64_row[col] = NAN;
        null_row[col] = 1;
      } else if (f.is_text()) {
        out.text_null[col][row] = 1;
      }
      continue;
    }
    double v = 0.0;
    const uint8_t* q;
    switch (f.kind) {
      case K_BOOLEAN:
        if (!c.bytes(1, &q)) return false;
        v = q[0] ? 1.0 : 0.0;
        break;
      case K_INT:
      case K_LONG: {
        int64_t x;
        if (!c.varlong(&x)) return false;
        v = (double)x;
        break;
      }
      case K_FLOAT: {
        if (!c.bytes(4, &q)) return false;
        float x;
        std::memcpy(&x, q, 4);
        v = x;
        break;
      }
      case K_DOUBLE: {
        if (!c.bytes(8, &q)) return false;
        std::memcpy(&v, q, 8);
        break;
      }
      case K_STRING:
      case K_BYTES: {
        int64_t len;
        if (!c.varlong(&len) || len < 0 || !c.bytes((size_t)len, &q)) return false;
        out.text[col][row].assign(reinterpret_cast<const char*>(q), (size_t)len);
        continue;
      }
      case K_FIXED:
        if (!c.bytes((size_t)f.fixed_size, &q)) return false;
        out.text[col][row].assign(reinterpret_cast<const char*>(q), (size_t)f.fixed_size);
        continue;
      case K_ENUM: {
        int64_t idx;
        if (!c.varlong(&idx) || idx < 0 || (f.n_symbols && idx >= f.n_symbols)) return false;
        out.text[col][row] = std::to_string(idx);
        continue;
      }
      default:
        return false;
    }
    num_row[col] = (float)v;
    if (num64_row) num64_row[col] = v;
    null_row[col] = 0;
  }
  return c.i == c.n;  // trailing garbage = malformed
}

DecodedBatch Codec::decode(const uint8_t* buf, size_t buf_len, const int64_t* offsets, size_t n, bool framing,
                           bool strict, bool want_f64) const {
  DecodedBatch out;
  out.n = n;
  out.n_numeric = n_num_;
  out.numeric.assign(n * n_num_, NAN);
  if (want_f64) out.numeric64.assign(n * n_num_, NAN);
  out.null_mask.assign(n * n_num_, 1);
  out.text.assign(n_txt_, std::vector<std::string>(n));
  out.text_null.assign(n_txt_, std::vector<uint8_t>(n, 0));
  out.schema_id.assign(n, -1);
  out.ok.assign(n, 0);
  for (size_t r = 0; r < n; ++r) {
    const int64_t a = offsets[r], b = offsets[r + 1];
    if (a < 0 || b < a || (uint64_t)b > buf_len) throw Error("avro: record offsets out of range");
    const uint8_t* p = buf + a;
    size_t len = (size_t)(b - a);
    bool good = true;
    if (framing) {
      if (len < 5 || p[0] != 0) {
        good = false;
      } else {
        out.schema_id[r] = (int32_t)(((uint32_t)p[1] << 24) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 8) | p[4]);
        p += 5;
        len -= 5;
      }
    }
    if (good)
      good = decode_one(p, len, &out.numeric[r * n_num_], want_f64 ? &out.numeric64[r * n_num_] : nullptr,
                        &out.null_mask[r * n_num_], out, r);
    out.ok[r] = good ? 1 : 0;
    if (!good) {
      ++out.n_errors;
      if (strict) throw Error("avro: malformed record at index " + std::to_string(r));
      for (size_t k = 0; k < n_num_; ++k) {
        out.numeric[r * n_num_ + k] = NAN;
        out.null_mask[r * n_num_ + k] = 1;
      }
    }
  }
  return out;
}

void Codec::encode(const double* numeric, const uint8_t* null_mask, const std::vector<std::vector<std::string>>& text,
                   const std::vector<std::vector<uint8_t>>& text_null, size_t n, bool framing, int32_t schema_id,
                   std::string& out, std::vector<int64_t>& offsets) const {
  if (text.size() != n_txt_) throw Error("avro: wrong number of text columns");
  for (const auto& col : text)
    if (col.size() != n) throw Error("avro: text column length mismatch");
  if (offsets.empty()) offsets.push_back((int64_t)out.size());
  for (size_t r = 0; r < n; ++r) {
    if (framing) {
      out.push_back('\0');
      const uint32_t id = (uint32_t)schema_id;
      out.push_back((char)(id >> 24));
      out.push_back((char)(id >> 16));
      out.push_back((char)(id >> 8));
      out.push_back((char)id);
    }
    for (size_t fi = 0; fi < fields_.size(); ++fi) {
      const Field& f = fields_[fi];
      const int col = col_[fi];
      bool is_null = f.kind == K_NULL;
      if (f.is_numeric()) is_null = null_mask && null_mask[r * n_num_ + col];
      else if (f.is_text()) is_null = !text_null.empty() && !text_null[col].empty() && text_null[col][r];
      if (f.null_branch >= 0) {
        write_varlong(out, is_null ? f.null_branch : 1 - f.null_branch);
        if (is_null) continue;
      } else if (is_null && f.kind != K_NULL) {
        throw Error("avro: null value for non-nullable field " + f.name);
      }
      if (f.kind == K_NULL) continue;
      if (f.is_numeric()) {
        const double v = numeric[r * n_num_ + col];
        switch (f.kind) {
          case K_BOOLEAN: out.push_back(v != 0.0 ? 1 : 0); break;
          case K_INT:
          case K_LONG: write_varlong(out, (int64_t)std::llround(v)); break;
          case K_FLOAT: {
            const float x = (float)v;
            out.append(reinterpret_cast<const char*>(&x), 4);
            break;
          }
          case K_DOUBLE: out.append(reinterpret_cast<const char*>(&v), 8); break;
          default: break;
        }
      } else {
        const std::string& s = text[col][r];
        switch (f.kind) {
          case K_STRING:
          case K_BYTES:
            write_varlong(out, (int64_t)s.size());
            out += s;
            break;
          case K_FIXED:
            if ((int)s.size() != f.fixed_size) throw Error("avro: fixed value has wrong size for " + f.name);
            out += s;
            break;
          case K_ENUM:
            write_varlong(out, std::stoll(s));
            break;
          default: break;
        }
      }
    }
    offsets.push_back((int64_t)out.size());
  }
}

}  // namespace avro
}  // namespace sml
