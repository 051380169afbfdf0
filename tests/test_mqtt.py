"""MQTT broker + Kafka bridge + client + device simulator (csrc/io/mqtt.cpp).

Mirrors the reference's ingestion layers: the HiveMQ device simulator
(infrastructure/test-generator/scenario*.xml), the HiveMQ broker with its Kafka
extension (infrastructure/hivemq/kafka-config.yaml) and KSQL's JSON -> Avro ->
PARTITION BY CAR streams (infrastructure/confluent/01_installConfluentPlatform.sh:235-256).
Everything runs over real sockets on 127.0.0.1.
"""
import json
import os
import subprocess
import sys
import time

import numpy as np
import pytest

from streamml.kafka import KafkaDataset, fake_broker
from streamml.mqtt import (MqttBroker, MqttClient, Scenario, TopicMapping, car_payload, kafka_partition,
                           load_topic_mappings, simulate, topic_matches)
from streamml.ops import load_io

REF = "/root/reference/infrastructure"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _ref(path):
    p = os.path.join(REF, path)
    if not os.path.exists(p):
        pytest.skip("reference tree not mounted")
    return p


# ---- codec --------------------------------------------------------------------------
def test_murmur2_matches_kafka_partitioner():
    # vectors from Kafka's UtilsTest.testMurmur2 (signed Java ints)
    io = load_io()
    for key, want in [("21", -973932308), ("foobar", -790332482), ("a-little-bit-long-string", -985981536),
                      ("a-little-bit-longer-string", -1486304829),
                      ("lkjh234lh9fiuh90y23oiuhsafujhadof229phr9h19h89h8", -58897971), ("abc", 479470107)]:
        assert io.murmur2(key) == want & 0xFFFFFFFF
    assert kafka_partition("foobar", 10) == ((-790332482 & 0x7FFFFFFF) % 10)


@pytest.mark.parametrize("flt,topic,ok", [
    ("vehicles/sensor/data/#", "vehicles/sensor/data/electric-vehicle-00001", True),
    ("vehicles/sensor/data/#", "vehicles/sensor/data", True),        # '#' includes the parent level
    ("vehicles/sensor/data/#", "vehicles/sensor/datax/a", False),
    ("vehicles/+/data/+", "vehicles/sensor/data/car", True),
    ("vehicles/+/data/+", "vehicles/sensor/data/car/x", False),
    ("+/+", "/a", True),
    ("#", "$SYS/broker", False),                                        # $-topics excluded from wildcards
    ("$SYS/#", "$SYS/broker", True),
    ("a/b", "a/b", True),
    ("a/b", "a/b/", False),
])
def test_topic_matching(flt, topic, ok):
    assert topic_matches(flt, topic) is ok


def test_publish_codec_roundtrip():
    io = load_io()
    for version in (4, 5):
        for qos in (0, 1, 2):
            raw = io.mqtt_encode_publish("vehicles/sensor/data/c1", b"\x00\x01payload", qos, qos == 2, 77, version)
            d = io.mqtt_parse_packet(raw + b"extra", version)
            assert d["type"] == 3 and d["size"] == len(raw)
            assert d["topic"] == "vehicles/sensor/data/c1" and d["payload"] == b"\x00\x01payload"
            assert d["qos"] == qos and d["retain"] == (qos == 2)
            assert d["packet_id"] == (77 if qos else 0)
    big = b"x" * 300_000   # 3-byte remaining length
    raw = io.mqtt_encode_publish("t", big, 0, False, 0, 5)
    assert io.mqtt_parse_packet(raw[:-1], 5) is None               # incomplete
    assert io.mqtt_parse_packet(raw, 5)["payload"] == big


# ---- broker / client ---------------------------------------------------------------
@pytest.fixture
def broker():
    b = MqttBroker()
    yield b
    b.stop()


def _client(b, cid, version=5, **kw):
    c = MqttClient()
    assert c.connect("127.0.0.1", b.port, cid, version=version, **kw) == 0
    return c


@pytest.mark.parametrize("version", [4, 5])
def test_qos_levels_and_wildcards(broker, version):
    sub = _client(broker, "sub", version)
    assert sub.subscribe(("vehicles/sensor/data/+", 2)) == [2]
    pub = _client(broker, "pub", version)
    for q in (0, 1, 2):
        pub.publish("vehicles/sensor/data/car-7", f"m{q}".encode(), qos=q)
    got = [sub.receive(2.0) for _ in range(3)]
    assert [(g[0], g[1], g[2]) for g in got] == [("vehicles/sensor/data/car-7", f"m{q}".encode(), q)
                                                 for q in (0, 1, 2)]
    pub.publish("other/topic", b"x")
    assert sub.receive(0.3) is None
    assert sub.ping()
    sub.unsubscribe("vehicles/sensor/data/+")
    pub.publish("vehicles/sensor/data/car-7", b"after", qos=1)
    assert sub.receive(0.3) is None
    sub.disconnect()
    pub.disconnect()


def test_max_qos_downgrade_and_retained():
    b = MqttBroker(max_qos=1)
    try:
        pub = _client(b, "p")
        pub.publish("cars/1/state", b"parked", qos=2, retain=True)   # QoS 2 handshake, stored at QoS 1
        pub.publish("cars/2/state", b"driving", qos=0, retain=True)
        pub.publish("cars/2/state", b"", qos=0, retain=True)         # empty retained payload clears it
        late = _client(b, "late")
        assert late.subscribe(("cars/+/state", 2)) == [1]             # granted QoS capped at max_qos
        m = late.receive(2.0)
        assert m == ("cars/1/state", b"parked", 1, True)
        assert late.receive(0.3) is None
        assert b.stats()["retained"] == 1
    finally:
        b.stop()


def test_shared_subscription_round_robin(broker):
    # scenario.xml: six consumers share $share/consumers/vehicles/sensor/data/#
    members = [_client(broker, f"consumer-{i}") for i in range(3)]
    for m in members:
        m.subscribe(("$share/consumers/vehicles/sensor/data/#", 1))
    pub = _client(broker, "car")
    for k in range(30):
        pub.publish(f"vehicles/sensor/data/electric-vehicle-{k:05d}", str(k).encode(), qos=1)
    counts = []
    seen = set()
    for m in members:
        n = 0
        while True:
            r = m.receive(0.5)
            if r is None:
                break
            seen.add(int(r[1]))
            n += 1
        counts.append(n)
    assert sorted(seen) == list(range(30))          # every message to exactly one member
    assert counts == [10, 10, 10]


def test_auth_and_takeover():
    b = MqttBroker(username="test", password="test123")
    try:
        bad = MqttClient()
        assert bad.connect("127.0.0.1", b.port, "x", version=5, username="test", password="nope") == 0x86
        assert bad.connect("127.0.0.1", b.port, "y", version=4, username="test", password="nope") == 4
        c1 = _client(b, "car-1", username="test", password="test123")
        c2 = _client(b, "car-1", username="test", password="test123")   # same id takes over
        time.sleep(0.2)
        with pytest.raises(RuntimeError):
            c1.ping(1.0)
        assert c2.ping()
        assert b.stats()["connections_current"] == 1
    finally:
        b.stop()


# ---- bridge ------------------------------------------------------------------------
def test_reference_kafka_extension_config_parses():
    maps, cluster = load_topic_mappings(_ref("hivemq/kafka-config.yaml"))
    assert [(m.id, m.filters, m.kafka_topic) for m in maps] == [("sensor-data", ["vehicles/sensor/data/#"],
                                                                 "sensor-data")]
    assert cluster["bootstrap"] == "kafka.operator.svc.cluster.local:9071"
    assert (cluster["username"], cluster["password"]) == ("test", "test123")


def test_bridge_to_kafka_keys_and_partitions():
    kb = fake_broker("mqtt-bridge-test")
    kb.create_topic("sensor-data", 10)   # 01_installConfluentPlatform.sh:180: 10 partitions
    with MqttBroker(kafka="fake://mqtt-bridge-test") as b:
        pub = _client(b, "fleet")
        topics = [f"vehicles/sensor/data/electric-vehicle-{i:05d}" for i in range(40)]
        for i, t in enumerate(topics):
            pub.publish(t, json.dumps({"i": i}).encode(), qos=1)
        pub.publish("not/mapped", b"ignored", qos=1)
        assert b.flush(10.0)
        st = b.stats()
        assert st["kafka_sent"] == 40 and st["kafka_failed"] == 0 and st["incoming_publish"] == 41
        assert b.mapping_counts() == {"sensor-data": 40}
    got = {}
    for p in range(10):
        for off, key, val in kb.read("sensor-data", p, 0):
            key = key.decode()
            assert kafka_partition(key, 10) == p          # Kafka default partitioner on the MQTT topic
            got[key] = json.loads(val)["i"]
    assert got == {t: i for i, t in enumerate(topics)}


def test_bridge_batches_fit_message_max_bytes():
    """A burst of ~600-byte car payloads to a one-partition topic (the auto-created default):
    the bridge cuts each partition's share of a drained queue into record batches under the
    broker's message.max.bytes (1 MB here, as Kafka's default) -- none refused, none dropped."""
    from streamml.kafka import FakeBroker
    kb = FakeBroker(message_max_bytes=1048588)
    kb.create_topic("sensor-data", 1)
    n = 6000
    payload = b"x" * 600
    with MqttBroker(kafka=kb.address) as b:
        pub = _client(b, "burst")
        for i in range(n):
            pub.publish(f"vehicles/sensor/data/electric-vehicle-{i % 50:05d}", payload, qos=0)
        deadline = time.time() + 20.0   # QoS 0: flush() covers what the broker has received so far
        while b.stats()["incoming_publish"] < n and time.time() < deadline:
            time.sleep(0.01)
        assert b.flush(20.0)
        st = b.stats()
        assert st["kafka_failed"] == 0 and st["kafka_sent"] == n, st
    assert kb.end_offset("sensor-data", 0) == n


def test_broker_refuses_oversized_batches_client_splits():
    """The in-process broker's message.max.bytes check (MESSAGE_TOO_LARGE, nothing appended),
    and the client's record sets: one produce call of 1.8 MB goes out as several batches."""
    from streamml.kafka import FakeBroker, KafkaClient
    kb = FakeBroker(message_max_bytes=1048588)
    kb.create_topic("t", 1)
    c = KafkaClient(kb.address)
    c.produce("t", 0, [b"v" * 600] * 3000)
    assert kb.end_offset("t", 0) == 3000
    small = FakeBroker(message_max_bytes=10_000)
    small.create_topic("t", 1)
    with pytest.raises(Exception, match="10"):
        KafkaClient(small.address).produce("t", 0, [b"v" * 600] * 100)
    assert small.end_offset("t", 0) == 0
    kb.stop()
    small.stop()


# ---- simulator ---------------------------------------------------------------------
def test_reference_scenarios_parse():
    full = Scenario.from_xml(_ref("test-generator/scenario.xml"))
    assert (full.clients, full.messages_per_client, full.interval_s, full.qos, full.version) == (100000, 3000, 10.0,
                                                                                                0, 5)
    assert full.client_prefix == "electric-vehicle-" and full.id_digits == 5
    assert full.topic_prefix == "vehicles/sensor/data/" and full.ramp_s == 20.0
    assert full.rate_per_s == pytest.approx(10000.0)          # 10 000 msg/s
    ev = Scenario.from_xml(_ref("test-generator/scenario_evaluation.xml"))
    assert (ev.clients, ev.messages_per_client, ev.interval_s, ev.qos) == (25, 40, 5.0, 1)


def test_payload_is_ksql_sensor_json():
    from streamml.data.cardata import FEATURES, canonical
    rec = json.loads(car_payload(42, 3, ts_ms=1234))
    assert {canonical(k) for k in rec if k not in ("failure_occurred", "timestamp")} == set(FEATURES)
    assert rec["failure_occurred"] in ("true", "false")
    assert rec["control_unit_firmware"] in (1000, 2000)
    assert isinstance(rec["tire_pressure11"], int)
    assert car_payload(42, 3, ts_ms=1234) == car_payload(42, 3, ts_ms=1234)   # deterministic per (car, seq)


def test_devsim_to_kafka_to_ksql_avro_to_training():
    """device simulator -> MQTT -> Kafka 'sensor-data' (JSON) -> KSQL Avro + REKEY ->
    per-car 5-min counts and an autoencoder epoch over the Avro stream (CPU)."""
    from streamml.data.avro import AvroCodec
    from streamml.data.ksql import run_events_per_window, run_json_to_avro
    name = "mqtt-e2e"
    kb = fake_broker(name)
    kb.create_topic("sensor-data", 10)
    kb.create_topic("SENSOR_DATA_S_AVRO", 1)
    kb.create_topic("SENSOR_DATA_S_AVRO_REKEY", 10)
    sc = Scenario.from_xml(_ref("test-generator/scenario_evaluation.xml")).scaled(messages=8, interval_s=0.01,
                                                                                 ramp_s=0.05)
    with MqttBroker(kafka=f"fake://{name}") as b:
        st = simulate(sc, "127.0.0.1", b.port, threads=5, failure_rate=0.2)
        assert st["connected"] == 25 and st["published"] == 200 and st["acked"] == 200   # QoS 1
        assert b.flush(10.0)
        assert b.stats()["kafka_sent"] == 200
    counts = run_json_to_avro(f"fake://{name}")
    assert counts == {"read": 200, "written": 200, "rekeyed": 200, "bad": 0}
    codec = AvroCodec("ksql-cardata-v1")
    rows, labels = [], []
    for bt in KafkaDataset(["SENSOR_DATA_S_AVRO:0:0"], servers=f"fake://{name}", codec=codec):
        rows.append(bt["numeric"])
        labels += list(bt["text"]["FAILURE_OCCURRED"])
    x = np.concatenate(rows)
    assert x.shape == (200, len(codec.numeric_fields)) and np.isfinite(x).all()
    assert set(labels) <= {b"true", b"false", "true", "false"}
    assert 0 < sum(1 for v in labels if v in (b"true", "true")) < 200
    n = run_events_per_window(f"fake://{name}", "SENSOR_DATA_S_AVRO_REKEY", "SENSOR_DATA_EVENTS_PER_5MIN_T")
    tot = 0
    for _, key, val in kb.read("SENSOR_DATA_EVENTS_PER_5MIN_T", 0, 0):
        tot += json.loads(val)["EVENT_COUNT"]
        assert json.loads(val)["CAR"].startswith("vehicles/sensor/data/electric-vehicle-")
    assert tot == 200 and n >= 25
    # train the reference autoencoder on the normal events of the Avro stream (CPU plumbing path)
    from streamml.data import stream as dst
    from streamml.models.autoencoder import Autoencoder
    normal = [c.x for c in dst.kafka(f"fake://{name}", ["SENSOR_DATA_S_AVRO:0:0"], schema="ksql-cardata-v1")
              .filter_normal()]
    xs = np.concatenate(normal).astype(np.float32)
    assert 0 < len(xs) < 200 and xs.shape[1] == 18
    ae = Autoencoder(device="cpu", input_normalizer="cardata")
    ae.compile()
    hist = ae.fit(xs, xs, epochs=2, batch_size=32, verbose=0)
    losses = hist.history["loss"] if hasattr(hist, "history") else hist["loss"]
    assert np.isfinite(losses).all()


def test_cli_devsim_and_broker(tmp_path):
    env = dict(os.environ, PYTHONPATH=ROOT)
    port = None
    srv = subprocess.Popen([sys.executable, "-m", "streamml.cli", "mqtt-broker", "--port", "0", "--kafka",
                            "fake://cli", "--duration", "20"], stdout=subprocess.PIPE, stderr=subprocess.STDOUT,
                           text=True, env=env, cwd=ROOT)
    try:
        for line in srv.stdout:
            if line.startswith("MQTT broker listening"):
                port = int(line.split()[3])
                break
        assert port
        r = subprocess.run([sys.executable, "-m", "streamml.cli", "devsim", "run", "-s",
                            _ref("test-generator/scenario.xml"), "--broker", f"127.0.0.1:{port}", "--clients", "50",
                            "--messages", "3", "--interval", "0.01", "--ramp", "0.05"],
                           capture_output=True, text=True, timeout=120, env=env, cwd=ROOT)
        assert r.returncode == 0, r.stdout + r.stderr
        st = json.loads(r.stdout.strip().splitlines()[-1])
        assert st["published"] == 150 and st["connected"] == 50
    finally:
        srv.terminate()
        out = srv.communicate(timeout=30)[0]
    final = json.loads([ln for ln in out.splitlines() if ln.startswith("{")][-1])
    assert final["incoming_publish"] == 150 and final["kafka_sent"] == 150


def test_prometheus_exposes_hivemq_and_devsim_metrics():
    from streamml.obs.metrics import REGISTRY
    with MqttBroker(kafka="fake://mqtt-metrics") as b:
        sc = Scenario().scaled(clients=5, messages=2, interval_s=0.001)
        simulate(sc, "127.0.0.1", b.port, threads=2)
        assert b.flush(5.0)
        text = REGISTRY.exposition()
        lab = f'{{broker="{b.port}"}}'
        assert f"com_hivemq_messages_incoming_publish_count{lab} 10" in text
        assert f"kafka_extension_topic_mapping_sensor_data_send_count{lab} 10" in text
        assert "agent_publish_successful_count" in text
    assert f'broker="{b.port}"' not in REGISTRY.exposition()      # stopped brokers leave the scrape
