// MQTT 3.1.1 / 5 broker with a Kafka bridge, an MQTT client, and a device-fleet
// simulator: the ingestion front of the reference architecture.
//
// Reference layers replaced:
//  * HiveMQ cluster (`infrastructure/hivemq/hivemq-crd.yaml:10-13`, maxQos 2) and its
//    Kafka extension, whose topic mapping forwards `vehicles/sensor/data/#` to the
//    Kafka topic `sensor-data` (`infrastructure/hivemq/kafka-config.yaml:20-29`; the
//    Kafka record key is the MQTT topic, the value the PUBLISH payload);
//  * the HiveMQ device simulator (`infrastructure/test-generator/scenario.xml`:
//    100 000 MQTT 5 clients `electric-vehicle-NNNNN`, each publishing car-sensor
//    payloads to `vehicles/sensor/data/<client>` at 1 msg / 10 s, QoS 0; the
//    evaluation scenario 25 clients, QoS 1, 1 msg / 5 s).
//
// Protocol subset: CONNECT/CONNACK (username/password, clean start, keep-alive,
// v5 properties parsed and skipped), PUBLISH QoS 0/1/2 with PUBACK / PUBREC /
// PUBREL / PUBCOMP, retained messages, SUBSCRIBE/SUBACK and UNSUBSCRIBE/UNSUBACK
// with `+` / `#` wildcards and `$share/<group>/<filter>` shared subscriptions
// (round-robin inside a group, as the scenario's 6 shared consumers use),
// PINGREQ/PINGRESP, DISCONNECT, client take-over on a duplicate client id.
#pragma once
#include <atomic>
#include <condition_variable>
#include <cstdint>
#include <deque>
#include <map>
#include <memory>
#include <mutex>
#include <stdexcept>
#include <string>
#include <thread>
#include <utility>
#include <vector>

#include "kafka.h"

namespace sml {
namespace mqtt {

struct Error : std::runtime_error {
  explicit Error(const std::string& m) : std::runtime_error(m) {}
};

enum PacketType : uint8_t {
  CONNECT = 1, CONNACK = 2, PUBLISH = 3, PUBACK = 4, PUBREC = 5, PUBREL = 6, PUBCOMP = 7,
  SUBSCRIBE = 8, SUBACK = 9, UNSUBSCRIBE = 10, UNSUBACK = 11, PINGREQ = 12, PINGRESP = 13,
  DISCONNECT = 14, AUTH = 15
};

// ---- codec ------------------------------------------------------------------
struct Packet {
  uint8_t type = 0;
  uint8_t flags = 0;   // low nibble of the fixed header
  std::string body;    // variable header + payload
};

void put_varint(std::string& s, uint32_t v);
// Parses one packet from [p, p+n); returns bytes consumed (0 = incomplete).
size_t parse_packet(const uint8_t* p, size_t n, Packet& out);
std::string frame(uint8_t type, uint8_t flags, const std::string& body);

struct Message {
  std::string topic;
  std::string payload;
  int qos = 0;
  bool retain = false;
  bool dup = false;
  uint16_t packet_id = 0;
};

std::string encode_connect(const std::string& client_id, int version, uint16_t keepalive, bool clean,
                           const std::string& username, const std::string& password);
std::string encode_publish(const Message& m, int version);
Message decode_publish(const Packet& pk, int version);
std::string encode_subscribe(uint16_t packet_id, const std::vector<std::pair<std::string, int>>& filters, int version);

// MQTT topic filter matching (sec. 4.7): `+` one level, `#` the rest (incl. the
// parent level); wildcards never match topics beginning with `$` at level one.
bool topic_matches(const std::string& filter, const std::string& topic);
bool valid_filter(const std::string& filter);

// Kafka's default partitioner (murmur2 of the key, positive, mod partitions).
uint32_t murmur2(const std::string& key);
int kafka_partition(const std::string& key, int partitions);

// ---- broker -----------------------------------------------------------------
struct TopicMapping {
  std::string id;                    // e.g. "sensor-data"
  std::vector<std::string> filters;  // e.g. {"vehicles/sensor/data/#"}
  std::string kafka_topic;           // e.g. "sensor-data"
};

struct BrokerConfig {
  int port = 0;                      // 0 = ephemeral (127.0.0.1); 1883 in the reference
  std::string username, password;    // empty = anonymous allowed
  int max_qos = 2;                   // hivemq-crd.yaml:13
  std::string kafka_bootstrap;       // "host:port" of the Kafka cluster; empty = no bridge
  kafka::ClientConfig kafka;
  std::vector<TopicMapping> mappings;
  int bridge_batch = 1024;           // records per partition record batch of a Produce request
  int bridge_linger_ms = 2;
  size_t bridge_queue_max = 1 << 20; // back-pressure bound (records)
};

// Byte cap of one bridged record batch: under a Kafka broker's default message.max.bytes (1 MB)
constexpr size_t kBridgeBatchBytes = 900u * 1024u;

struct BrokerStats {
  uint64_t incoming_publish = 0;     // com_hivemq_messages_incoming_publish_count
  uint64_t outgoing_publish = 0;
  uint64_t connections_current = 0;  // com_hivemq_networking_connections_current
  uint64_t connections_total = 0;
  uint64_t retained = 0;
  uint64_t kafka_sent = 0;           // kafka_extension_..._send_count (all mappings)
  uint64_t kafka_failed = 0;
  uint64_t kafka_queued = 0;
};

class Broker {
 public:
  explicit Broker(BrokerConfig cfg);
  ~Broker();
  int port() const { return port_; }
  void stop();
  // in-process publish (same routing as a client PUBLISH)
  void publish(const Message& m);
  BrokerStats stats();
  std::map<std::string, uint64_t> mapping_counts();  // per mapping id
  // block until every bridged record so far is acknowledged by Kafka (or timeout)
  bool flush(int timeout_ms);

  struct Session;

 private:
  struct Sub {
    std::string filter;
    int qos;
    std::string share_group;  // empty = normal
  };
  struct SharedGroup {
    std::vector<std::string> members;  // client ids
    size_t next = 0;
  };
  struct BridgeRec {
    int mapping;
    std::string key, value;
    int64_t ts;
  };

  BrokerConfig cfg_;
  int listen_fd_ = -1;
  int port_ = 0;
  std::atomic<bool> running_{false};
  std::thread accept_thread_;
  std::mutex mu_;  // sessions, subscriptions, retained
  std::map<std::string, std::shared_ptr<Session>> sessions_;
  std::map<std::string, std::vector<Sub>> subs_;  // client id -> subscriptions
  std::map<std::pair<std::string, std::string>, SharedGroup> shared_;  // (group, filter)
  std::map<std::string, Message> retained_;
  std::vector<std::thread> workers_;
  std::vector<int> fds_;

  std::atomic<uint64_t> in_pub_{0}, out_pub_{0}, conn_cur_{0}, conn_tot_{0}, kafka_sent_{0}, kafka_failed_{0};
  std::vector<std::unique_ptr<std::atomic<uint64_t>>> map_counts_;

  // bridge
  std::mutex bq_mu_;
  std::condition_variable bq_cv_, bq_done_cv_;
  std::deque<BridgeRec> bq_;
  uint64_t b_enq_ = 0, b_done_ = 0;
  std::thread bridge_thread_;

  void accept_loop();
  void serve(int fd);
  void route(const Message& m, const std::string& from_client);
  void deliver(const std::shared_ptr<Session>& s, Message m, int sub_qos);
  void bridge_loop();
};

// ---- client -----------------------------------------------------------------
class Client {
 public:
  Client() = default;
  ~Client();
  // returns the CONNACK reason / return code (0 = accepted); throws on transport errors
  // source_ip: bind the socket to this local address first ("" = the kernel's choice); a
  // fleet beyond the ~28k ephemeral ports of one (source, destination) pair spreads its
  // connections over several loopback sources (127.0.0.x)
  int connect(const std::string& host, int port, const std::string& client_id, int version = 5,
              uint16_t keepalive = 60, bool clean = true, const std::string& username = "",
              const std::string& password = "", int timeout_ms = 5000, const std::string& source_ip = "");
  // QoS 1/2 block until the handshake completes (PUBACK / PUBCOMP)
  void publish(const std::string& topic, const std::string& payload, int qos = 0, bool retain = false);
  std::vector<int> subscribe(const std::vector<std::pair<std::string, int>>& filters);
  void unsubscribe(const std::vector<std::string>& filters);
  // next application message (acks QoS 1/2 deliveries); false on timeout
  bool receive(Message& out, int timeout_ms);
  bool ping(int timeout_ms = 2000);
  void disconnect();
  bool connected() const { return fd_ >= 0; }
  bool session_present() const { return session_present_; }

 private:
  int fd_ = -1;
  int version_ = 5;
  uint16_t next_id_ = 1;
  bool session_present_ = false;
  std::string rx_;
  std::deque<Message> inbox_;
  std::mutex mu_;
  uint16_t alloc_id();
  bool read_packet(Packet& pk, int timeout_ms);
  void send_raw(const std::string& s);
  void handle_incoming(const Packet& pk);  // PUBLISH / PUBREL received while waiting
};

// ---- device simulator ----------------------------------------------------------
// Payload: one JSON object per PUBLISH with the 18 car-sensor fields of the KSQL
// stream SENSOR_DATA_S plus `failure_occurred` (01_installConfluentPlatform.sh:235).
struct SimConfig {
  std::string host = "127.0.0.1";
  int port = 1883;
  std::string client_prefix = "electric-vehicle-";  // clientIdPattern electric-vehicle-[0-9]{5}
  int id_digits = 5;
  int id_offset = 0;
  std::string topic_prefix = "vehicles/sensor/data/";  // topic = prefix + client id
  int clients = 25;
  int messages_per_client = 40;
  double interval_s = 5.0;     // rate "1/5s"
  double ramp_s = 0.0;         // connect ramp-up spread
  int qos = 0;
  int version = 5;
  int threads = 4;
  uint64_t seed = 0;
  double failure_rate = 0.01;  // P(failure_occurred = "true") per event
  std::string username, password;
  // Paced mode (fleet benchmarks): every client connects first; publishing starts for all
  // clients at once -- at start_at_unix (wall clock, shared by several simulator processes)
  // or, if 0, when this process's last client is connected -- and client i's message k is
  // due at start + interval * (i + 0.5) / clients + k * interval, so the fleet offers a
  // steady clients / interval messages per second.
  bool paced = false;
  double start_at_unix = 0.0;
  bool stamp_ns = false;             // add "sent_ns" (CLOCK_MONOTONIC ns at send) to each payload
  std::vector<std::string> source_ips;   // client i binds source_ips[i % n] (empty: kernel's choice)
  // per-feature generator ranges (18 entries, SENSOR_DATA_S column order)
  std::vector<double> lo, hi;
  std::vector<int> is_int;
};

struct SimStats {
  uint64_t connected = 0;
  uint64_t connect_failed = 0;
  uint64_t published = 0;
  uint64_t acked = 0;
  uint64_t publish_failed = 0;
  double elapsed_s = 0.0;
  double connect_s = 0.0;            // first connect -> last client connected
  double publish_s = 0.0;            // first publish -> last publish
  double max_lag_ms = 0.0;           // paced: worst send delay behind schedule
  uint64_t late_10ms = 0;            // paced: sends more than 10 ms behind schedule
};

SimStats simulate(const SimConfig& cfg, std::atomic<bool>* stop = nullptr);
std::string car_payload_json(const SimConfig& cfg, uint64_t car, uint64_t seq, int64_t ts_ms, int64_t sent_ns = -1);

}  // namespace mqtt
}  // namespace sml
