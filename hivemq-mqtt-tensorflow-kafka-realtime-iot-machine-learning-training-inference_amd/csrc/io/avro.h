// Columnar Avro binary codec + Confluent wire framing.
//
// Replaces tensorflow-io's `decode_avro` + the `substr(e, 5, -1)` framing strip
// used by every reference script (AUTOENCODER-TensorFlow-IO-Kafka/cardata-v3.py:49-75):
// a batch of Confluent-framed records (magic 0x00 + 4-byte big-endian schema id +
// Avro body) is decoded in one call straight into row-major float32 feature
// columns (plus a null mask) ready for the pinned-host ring / H2D copy, and
// string columns.  The schema is compiled in Python (JSON) into a flat plan of
// primitive fields, each optionally a ["null", T] union -- the shape of both the
// KSQL record (KsqlDataSourceSchema, nullable UPPERCASE fields) and the
// simulator record (com.hivemq.avro.CarData, plain fields).
#pragma once
#include <cstddef>
#include <cstdint>
#include <stdexcept>
#include <string>
#include <vector>

namespace sml {
namespace avro {

enum Kind : int {
  K_NULL = 0, K_BOOLEAN = 1, K_INT = 2, K_LONG = 3, K_FLOAT = 4, K_DOUBLE = 5,
  K_STRING = 6, K_BYTES = 7, K_ENUM = 8, K_FIXED = 9,
};

struct Field {
  std::string name;
  int kind = K_DOUBLE;
  int null_branch = -1;     // index of "null" in a 2-branch union, -1 = not a union
  int fixed_size = 0;
  int n_symbols = 0;        // enum
  bool is_numeric() const { return kind >= K_BOOLEAN && kind <= K_DOUBLE; }
  bool is_text() const { return kind == K_STRING || kind == K_BYTES || kind == K_FIXED || kind == K_ENUM; }
};

struct Error : std::runtime_error {
  using std::runtime_error::runtime_error;
};

// zigzag varints (Avro int/long; also Kafka record fields)
size_t read_varlong(const uint8_t* p, size_t n, int64_t* out);
void write_varlong(std::string& out, int64_t v);

struct DecodedBatch {
  size_t n = 0;
  size_t n_numeric = 0;
  std::vector<float> numeric;          // [n][n_numeric] row-major
  std::vector<double> numeric64;       // same, double precision (optional)
  std::vector<uint8_t> null_mask;      // [n][n_numeric] 1 = null
  std::vector<std::vector<std::string>> text;   // per text field, n values
  std::vector<std::vector<uint8_t>> text_null;  // per text field, n flags
  std::vector<int32_t> schema_id;      // per record (-1 without framing)
  std::vector<uint8_t> ok;             // per record decode status
  size_t n_errors = 0;
};

class Codec {
 public:
  explicit Codec(std::vector<Field> fields);
  const std::vector<Field>& fields() const { return fields_; }
  size_t n_numeric() const { return n_num_; }
  size_t n_text() const { return n_txt_; }

  // Decode `n` records laid out back to back in `buf` (record i spans
  // [offsets[i], offsets[i+1])).  framing: expect/strip the 5-byte Confluent
  // header.  strict: throw on the first malformed record, else flag it in `ok`.
  DecodedBatch decode(const uint8_t* buf, size_t buf_len, const int64_t* offsets, size_t n, bool framing,
                      bool strict, bool want_f64) const;

  // Encode rows (numeric [n][n_numeric] doubles, null mask, text columns) back to
  // Avro (+ optional Confluent header with `schema_id`), appending to `out` and
  // pushing record end offsets into `offsets`.
  void encode(const double* numeric, const uint8_t* null_mask, const std::vector<std::vector<std::string>>& text,
              const std::vector<std::vector<uint8_t>>& text_null, size_t n, bool framing, int32_t schema_id,
              std::string& out, std::vector<int64_t>& offsets) const;

 private:
  std::vector<Field> fields_;
  std::vector<int> col_;           // field -> column within its category (numeric / text), -1 for null
  size_t n_num_ = 0, n_txt_ = 0;
  bool decode_one(const uint8_t* p, size_t n, float* num_row, double* num64_row, uint8_t* null_row,
                  DecodedBatch& out, size_t row) const;
};

}  // namespace avro
}  // namespace sml
