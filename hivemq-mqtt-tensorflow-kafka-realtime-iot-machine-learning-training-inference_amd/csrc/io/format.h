// Result-record formatting in C++ (no Python object per event).
//
// The reference's predict job writes every reconstruction as `np.array2string(output)`
// (AUTOENCODER-TensorFlow-IO-Kafka/cardata-v3.py:241-246); the streaming scorer writes a
// JSON record per event built with `json.dumps` (cli/serve.py).  Both are reproduced
// byte for byte here so the low-latency loop (scoreloop.h) never enters Python:
//
//   * py_float_repr     -- Python's repr(float): shortest round-trip digits, fixed
//                          notation for 1e-4 <= |x| < 1e16, else d.ddde+XX;
//   * array2string_f32  -- numpy's default array2string of a 1-D float32 array
//                          (floatmode 'maxprec', precision 8, linewidth 75, shortest
//                          float32 digits, common padding, exponent mode when the
//                          non-zero magnitudes span > 1e3 or reach < 1e-4 / >= 1e8);
//   * json_string       -- json.dumps string escaping (ensure_ascii: \uXXXX, surrogate
//                          pairs for non-BMP code points).
#pragma once
#include <cstddef>
#include <cstdint>
#include <string>

namespace sml {
namespace fmt {

void py_float_repr(double v, std::string& out);
void array2string_f32(const float* v, int n, std::string& out);
void json_string(const uint8_t* p, size_t n, std::string& out);

// {"car": <key|null>, "partition": P, "offset": O, "score": S, "anomaly": true|false
//  [, "reconstruction": "<array2string(recon)>"]}   (json.dumps field order / spacing)
void score_record_json(const uint8_t* key, int64_t key_len, int partition, int64_t offset, float score, bool anomaly,
                       const float* recon, int D, std::string& out);

}  // namespace fmt
}  // namespace sml
