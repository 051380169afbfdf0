// Flat JSON car-event records -> projected float rows, in one pass, no allocation.
//
// The MQTT->Kafka bridge writes each device PUBLISH payload unchanged to the Kafka topic
// `sensor-data` (infrastructure/hivemq/kafka-config.yaml:20-29): one JSON object per event
// with the 18 sensor fields + `failure_occurred`, which KSQL declares as the stream
// SENSOR_DATA_S (infrastructure/confluent/01_installConfluentPlatform.sh:235) before
// re-encoding it as Avro (:242).  This decoder reads those records directly: the low-latency
// scorer can follow `sensor-data` itself (no KSQL hop on the per-event path), and the KSQL
// JSON -> Avro job (data/ksql.py) parses whole fetches here instead of json.loads per record.
//
// Keys are matched after canonicalisation -- ASCII lower case with every '_' dropped -- so
// the KSQL UPPERCASE columns, the simulator's snake_case (`tire_pressure11`), the CSV form
// (`tire_pressure_1_1`) and camelCase all name the same column.  Values: JSON numbers,
// numbers inside strings, null (-> NaN); the label is a "true"/"false" string (code 1 / 0,
// anything else 2, the feed's label codes); nested objects / arrays are skipped.
#pragma once
#include <cstddef>
#include <cstdint>
#include <string>
#include <utility>
#include <vector>

namespace sml {
namespace jsonrow {

class Plan {
 public:
  // columns: (key, output column); label_key / stamp_key: "" = none.  Keys are
  // canonicalised here (callers may pass any spelling).
  Plan(const std::vector<std::pair<std::string, int>>& columns, const std::string& label_key,
       const std::string& stamp_key);
  int width() const { return width_; }
  // One record.  Missing columns are NaN, a missing label is code 2, a missing stamp 0.
  // Returns false for a record that is not a JSON object (row contents then undefined).
  bool decode(const uint8_t* p, size_t n, float* row, uint8_t* label, int64_t* stamp) const;

 private:
  static constexpr int kSlots = 128;                  // open addressing, load <= 1/4
  struct Slot {
    uint64_t h = 0;
    uint8_t len = 0;
    char key[40] = {0};
    int16_t target = -1;                              // column, kLabel or kStamp
  };
  static constexpr int16_t kLabel = -2, kStamp = -3;
  Slot slots_[kSlots];
  int width_ = 0;
  void add(const std::string& key, int16_t target);
  const Slot* find(const char* k, size_t n, uint64_t h) const;
};

// canonical form of a key (lower case, no '_'); exposed for tests
std::string canonical(const std::string& key);

}  // namespace jsonrow
}  // namespace sml
