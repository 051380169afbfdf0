// Host-code sanitizer harness: the untrusted-input parsers and the
// threaded broker/client are the risky native parts, so they are exercised here
// under -fsanitize=address,undefined (mode "fuzz") and -fsanitize=thread (mode
// "threads"), as a plain C++ program (no Python, no GPU).  Built and run by
// tests/test_sanitizers.py.
//
//   fuzz:     round-trips valid inputs, then feeds thousands of mutated / truncated
//             Avro records, Kafka record batches and HDF5 images to the decoders;
//             every malformed input must end in a clean exception, never UB.
//   threads:  one in-process broker, several producer and consumer threads on
//             separate client connections, concurrent appends / fetches / commits;
//             then the MQTT broker (epoll I/O threads) with its Kafka bridge under
//             concurrent publishers, a shared-subscription group and the simulator.
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <random>
#include <string>
#include <thread>
#include <vector>

#include "../io/avro.h"
#include "../io/h5.h"
#include "../io/kafka.h"
#include "../io/mqtt.h"

using namespace sml;

namespace {

int failures = 0;
#define CHECK(cond)                                                        \
  do {                                                                     \
    if (!(cond)) {                                                         \
      std::fprintf(stderr, "CHECK failed %s:%d: %s\n", __FILE__, __LINE__, #cond); \
      ++failures;                                                          \
    }                                                                      \
  } while (0)

std::vector<avro::Field> ksql_like_fields() {
  std::vector<avro::Field> f;
  for (int i = 0; i < 13; ++i) f.push_back({"F" + std::to_string(i), avro::K_DOUBLE, 0, 0, 0});
  for (int i = 0; i < 5; ++i) f.push_back({"I" + std::to_string(i), avro::K_INT, 0, 0, 0});
  f.push_back({"FAILURE_OCCURRED", avro::K_STRING, 0, 0, 0});
  f.push_back({"plain", avro::K_LONG, -1, 0, 0});
  return f;
}

void mutate(std::string& s, std::mt19937_64& rng) {
  if (s.empty()) return;
  const int kind = rng() % 4;
  if (kind == 0) {
    s[rng() % s.size()] = (char)(rng() & 0xff);
  } else if (kind == 1) {
    s.resize(rng() % s.size());
  } else if (kind == 2) {
    const size_t p = rng() % s.size();
    s.insert(p, 1 + rng() % 8, (char)(rng() & 0xff));
  } else {
    for (int i = 0; i < 4; ++i) s[rng() % s.size()] ^= (char)(1 << (rng() % 8));
  }
}

void fuzz_avro(std::mt19937_64& rng) {
  avro::Codec codec(ksql_like_fields());
  const size_t n = 64;
  std::vector<double> num(n * codec.n_numeric());
  std::vector<uint8_t> nulls(n * codec.n_numeric());
  for (size_t i = 0; i < num.size(); ++i) {
    const bool is_int = (i % codec.n_numeric()) >= 13;   // INT / LONG columns carry integers
    num[i] = is_int ? (double)((int64_t)(rng() % 20000) - 1000) : (double)(rng() % 20000) / 7.0 - 1000.0;
    const bool nullable = (i % codec.n_numeric()) != codec.n_numeric() - 1;   // "plain" is not a union
    nulls[i] = nullable && (rng() % 10) == 0;
  }
  std::vector<std::vector<std::string>> text(codec.n_text(), std::vector<std::string>(n));
  std::vector<std::vector<uint8_t>> tnull(codec.n_text(), std::vector<uint8_t>(n, 0));
  for (size_t i = 0; i < n; ++i) text[0][i] = (i % 3) ? "false" : "true";
  std::string buf;
  std::vector<int64_t> offs{0};
  codec.encode(num.data(), nulls.data(), text, tnull, n, true, 7, buf, offs);
  auto dec = codec.decode(reinterpret_cast<const uint8_t*>(buf.data()), buf.size(), offs.data(), n, true, true,
                          true);
  CHECK(dec.n == n && dec.n_errors == 0);
  for (size_t i = 0; i < num.size(); ++i)
    if (!nulls[i]) CHECK(dec.numeric64[i] == num[i]);
  int rejected = 0;
  for (int it = 0; it < 4000; ++it) {
    std::string m = buf;
    mutate(m, rng);
    std::vector<int64_t> mo = offs;
    for (auto& o : mo) o = std::min<int64_t>(o, (int64_t)m.size());
    try {
      auto d = codec.decode(reinterpret_cast<const uint8_t*>(m.data()), m.size(), mo.data(), n, true, false, false);
      rejected += (int)d.n_errors;
    } catch (const std::exception&) {
      ++rejected;
    }
    try {   // strict mode must throw, not crash
      codec.decode(reinterpret_cast<const uint8_t*>(m.data()), m.size(), mo.data(), n, true, true, false);
    } catch (const std::exception&) {
    }
  }
  CHECK(rejected > 0);
  std::printf("avro: ok (%d malformed records rejected)\n", rejected);
}

void fuzz_kafka_batches(std::mt19937_64& rng) {
  std::vector<kafka::Record> recs;
  for (int i = 0; i < 50; ++i) {
    kafka::Record r;
    r.timestamp = 1000 + i;
    r.value = std::string(1 + rng() % 200, (char)('a' + i % 26));
    if (i % 2) {
      r.key = "car-" + std::to_string(i);
      r.key_null = false;
    }
    recs.push_back(r);
  }
  std::string batch = kafka::encode_record_batch(100, recs);
  kafka::FetchResult fr;
  kafka::decode_record_batches(reinterpret_cast<const uint8_t*>(batch.data()), batch.size(), 0, fr);
  CHECK(fr.size() == recs.size());
  for (size_t i = 0; i < fr.size(); ++i) CHECK(fr.offsets[i] == (int64_t)(100 + i));
  int errs = 0;
  for (int it = 0; it < 4000; ++it) {
    std::string m = batch;
    mutate(m, rng);
    kafka::FetchResult out;
    try {
      kafka::decode_record_batches(reinterpret_cast<const uint8_t*>(m.data()), m.size(), 0, out);
    } catch (const std::exception&) {
      ++errs;
    }
    CHECK(out.value_offsets.size() == out.offsets.size() + 1);
  }
  std::printf("kafka batches: ok (%d rejected)\n", errs);
}

void fuzz_h5(std::mt19937_64& rng) {
  h5::Node root;
  h5::Value title;
  title.kind = h5::Value::VLEN_STRING;
  title.strings = {"{\"class_name\": \"Model\"}"};
  root.attrs.push_back({"model_config", title});
  h5::Node grp;
  h5::Node ds;
  ds.is_group = false;
  ds.value.kind = h5::Value::NUMERIC;
  ds.value.dtype = 'f';
  ds.value.itemsize = 4;
  ds.value.shape = {18, 14};
  ds.value.data.assign(18 * 14 * 4, '\x01');
  grp.children.push_back({"kernel:0", ds});
  root.children.push_back({"dense", grp});
  const std::string img = h5::write_bytes(root);
  h5::Node back = h5::read_bytes(img);
  CHECK(back.children.size() == 1 && back.children[0].second.children.size() == 1);
  int errs = 0;
  for (int it = 0; it < 3000; ++it) {
    std::string m = img;
    mutate(m, rng);
    try {
      h5::read_bytes(m);
    } catch (const std::exception&) {
      ++errs;
    }
  }
  std::printf("h5: ok (%d rejected)\n", errs);
}


void fuzz_mqtt(std::mt19937_64& rng) {
  // valid packets first, then mutations through the framing parser and PUBLISH decoder
  std::vector<std::string> seeds;
  for (int v : {4, 5})
    for (int q = 0; q < 3; ++q) {
      mqtt::Message m;
      m.topic = "vehicles/sensor/data/electric-vehicle-0000" + std::to_string(q);
      m.payload = std::string(40 + 300 * q, 'x');
      m.qos = q;
      m.packet_id = (uint16_t)(q + 1);
      seeds.push_back(mqtt::encode_publish(m, v));
      seeds.push_back(mqtt::encode_connect("c" + std::to_string(q), v, 60, q != 1, q ? "u" : "", q ? "p" : ""));
      seeds.push_back(mqtt::encode_subscribe((uint16_t)(q + 9), {{"a/+/#", q}, {"$share/g/b", 1}}, v));
    }
  int errs = 0, parsed = 0;
  for (int it = 0; it < 20000; ++it) {
    std::string b = seeds[rng() % seeds.size()];
    if (it % 10) mutate(b, rng);
    try {
      mqtt::Packet pk;
      const size_t used = mqtt::parse_packet(reinterpret_cast<const uint8_t*>(b.data()), b.size(), pk);
      CHECK(used <= b.size());
      if (used && pk.type == mqtt::PUBLISH) {
        mqtt::Message m = mqtt::decode_publish(pk, (it & 1) ? 5 : 4);
        CHECK(m.topic.size() + m.payload.size() <= pk.body.size());
      }
      if (used) ++parsed;
    } catch (const std::exception&) {
      ++errs;
    }
  }
  for (int it = 0; it < 5000; ++it) {  // topic matcher on random filters/topics
    std::string f, t;
    const char alpha[] = "ab/+#$";
    for (int k = rng() % 8; k > 0; --k) f.push_back(alpha[rng() % 6]);
    for (int k = rng() % 8; k > 0; --k) t.push_back(alpha[rng() % 3]);
    if (mqtt::valid_filter(f)) (void)mqtt::topic_matches(f, t);
  }
  std::printf("mqtt: ok (%d parsed, %d rejected)\n", parsed, errs);
}

void threads_broker() {
  kafka::BrokerConfig bc;
  bc.sasl_username = "test";
  bc.sasl_password = "test123";
  kafka::Broker broker(bc);
  broker.create_topic("t", 4);
  kafka::ClientConfig cc;
  cc.sasl_mechanism = "PLAIN";
  cc.sasl_username = "test";
  cc.sasl_password = "test123";
  const std::string addr = "127.0.0.1:" + std::to_string(broker.port());
  std::atomic<int> produced{0}, consumed{0}, errors{0};
  std::vector<std::thread> th;
  for (int p = 0; p < 4; ++p) {
    th.emplace_back([&, p] {
      try {
        kafka::Client c(addr, cc);
        for (int i = 0; i < 50; ++i) {
          std::vector<kafka::Record> rs(20);
          for (auto& r : rs) r.value = "v" + std::to_string(p) + "-" + std::to_string(i);
          c.produce("t", p, rs, 1);
          produced += 20;
        }
      } catch (const std::exception& e) {
        std::fprintf(stderr, "producer: %s\n", e.what());
        ++errors;
      }
    });
  }
  for (int q = 0; q < 4; ++q) {
    th.emplace_back([&, q] {
      try {
        kafka::Client c(addr, cc);
        int64_t off = 0;
        int idle = 0;
        while (idle < 200) {
          auto fr = c.fetch("t", q, off, 1 << 16, 5);
          if (fr.size() == 0) {
            ++idle;
            continue;
          }
          idle = 0;
          consumed += (int)fr.size();
          off = fr.offsets.back() + 1;
          c.commit("g", "t", q, off);
          if (off >= 1000) break;
        }
      } catch (const std::exception& e) {
        std::fprintf(stderr, "consumer: %s\n", e.what());
        ++errors;
      }
    });
  }
  for (auto& t : th) t.join();
  broker.stop();
  CHECK(errors == 0);
  CHECK(produced == 4000);
  CHECK(consumed == 4000);
  std::printf("threads: ok (produced %d, consumed %d)\n", produced.load(), consumed.load());
}


void threads_mqtt() {
  kafka::BrokerConfig kbc;
  kafka::Broker kb(kbc);
  kb.create_topic("sensor-data", 4);
  mqtt::BrokerConfig mc;
  mc.kafka_bootstrap = "127.0.0.1:" + std::to_string(kb.port());
  mc.mappings.push_back({"sensor-data", {"vehicles/sensor/data/#"}, "sensor-data"});
  mqtt::Broker broker(mc);
  std::atomic<int> got{0}, errors{0};
  std::atomic<bool> done{false};
  std::vector<std::thread> th;
  for (int c = 0; c < 3; ++c) {  // shared-subscription consumers
    th.emplace_back([&, c] {
      try {
        mqtt::Client cl;
        cl.connect("127.0.0.1", broker.port(), "consumer-" + std::to_string(c), 5);
        cl.subscribe({{"$share/consumers/vehicles/sensor/data/#", 1}});
        mqtt::Message m;
        while (!done || cl.receive(m, 200)) {
          if (cl.receive(m, 50)) ++got;
        }
        cl.disconnect();
      } catch (const std::exception& e) {
        std::fprintf(stderr, "mqtt consumer: %s\n", e.what());
        ++errors;
      }
    });
  }
  std::this_thread::sleep_for(std::chrono::milliseconds(100));
  mqtt::SimConfig sc;
  sc.port = broker.port();
  sc.clients = 40;
  sc.messages_per_client = 10;
  sc.interval_s = 0.002;
  sc.qos = 1;
  sc.threads = 4;
  const auto st = mqtt::simulate(sc);
  CHECK(st.published == 400 && st.acked == 400 && st.connect_failed == 0);
  CHECK(broker.flush(10000));
  std::this_thread::sleep_for(std::chrono::milliseconds(300));
  done = true;
  for (auto& t : th) t.join();
  int64_t in_kafka = 0;
  for (int p = 0; p < 4; ++p) in_kafka += kb.end_offset("sensor-data", p);
  broker.stop();
  kb.stop();
  CHECK(errors == 0);
  CHECK(in_kafka == 400);
  CHECK(got == 400);
  std::printf("threads mqtt: ok (kafka %lld, shared consumers %d)\n", (long long)in_kafka, got.load());
}

}  // namespace

int main(int argc, char** argv) {
  const std::string mode = argc > 1 ? argv[1] : "fuzz";
  std::mt19937_64 rng(12345);
  if (mode == "fuzz") {
    fuzz_avro(rng);
    fuzz_kafka_batches(rng);
    fuzz_h5(rng);
    fuzz_mqtt(rng);
  } else if (mode == "threads") {
    threads_broker();
    threads_mqtt();
  } else {
    std::fprintf(stderr, "usage: %s fuzz|threads\n", argv[0]);
    return 2;
  }
  if (failures) {
    std::fprintf(stderr, "%d checks failed\n", failures);
    return 1;
  }
  std::printf("PASS %s\n", mode.c_str());
  return 0;
}
