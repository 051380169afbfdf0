"""MQTT ingestion: broker with a Kafka bridge, client, and the device-fleet simulator.

The reference's device -> model path starts with MQTT:
HiveMQ device-simulator agents publish car-sensor payloads to
``vehicles/sensor/data/electric-vehicle-NNNNN`` (``infrastructure/test-generator/scenario.xml``),
a 5-node HiveMQ cluster (``infrastructure/hivemq/hivemq-crd.yaml:10-13``) forwards every
topic under ``vehicles/sensor/data/#`` to the Kafka topic ``sensor-data`` through its Kafka
extension (``infrastructure/hivemq/kafka-config.yaml:20-29``), and KSQL turns the JSON
records into the Avro streams the training scripts read
(``infrastructure/confluent/01_installConfluentPlatform.sh:231-256``).

Here all of it is native C++ (``csrc/io/mqtt.cpp``): an epoll MQTT 3.1.1/5 broker whose
bridge produces to any Kafka-protocol broker with the Kafka default (murmur2) partitioner
keyed by the MQTT topic, a blocking client, and a multi-threaded fleet simulator.  The
reference configuration files are read directly: :func:`load_topic_mappings` parses the
HiveMQ ``kafka-configuration`` XML (or the ConfigMap YAML that wraps it) and
:class:`Scenario` parses the device-simulator scenario XML.
"""
from __future__ import annotations

import re
import xml.etree.ElementTree as ET
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence, Tuple

from ..ops._ext import load_io

SENSOR_TOPIC_FILTER = "vehicles/sensor/data/#"     # kafka-config.yaml:26
SENSOR_KAFKA_TOPIC = "sensor-data"                 # kafka-config.yaml:28


def _io():
    return load_io()


def topic_matches(filter_: str, topic: str) -> bool:
    """MQTT topic-filter matching (``+`` one level, ``#`` the rest, ``$`` topics excluded)."""
    return _io().mqtt_topic_matches(filter_, topic)


def kafka_partition(key, partitions: int) -> int:
    """Kafka's default partitioner (murmur2 of the key bytes) -- what the bridge uses."""
    if isinstance(key, (bytes, bytearray)):
        key = key.decode("latin-1")
    return _io().kafka_partition(key, int(partitions))


@dataclass
class TopicMapping:
    """One HiveMQ Kafka-extension ``<topic-mapping>``: MQTT filters -> a Kafka topic."""

    id: str
    filters: List[str]
    kafka_topic: str


def load_topic_mappings(path_or_text: str) -> Tuple[List[TopicMapping], Dict[str, str]]:
    """Parse the HiveMQ Kafka-extension configuration.

    Accepts the bare ``<kafka-configuration>`` XML or the Kubernetes ConfigMap YAML
    that carries it (``kafka-config.yaml``).  Returns the topic mappings and the
    first cluster's connection settings (``bootstrap``, ``username``, ``password``).
    """
    text = path_or_text
    if "<" not in path_or_text and "\n" not in path_or_text:
        with open(path_or_text) as fh:
            text = fh.read()
    if "<kafka-configuration" not in text:
        raise ValueError("no <kafka-configuration> element found")
    if not text.lstrip().startswith("<"):
        import yaml  # ConfigMap: data['kafka-configuration.xml']
        doc = yaml.safe_load(text)
        text = doc["data"]["kafka-configuration.xml"]
    root = ET.fromstring(text)
    cluster: Dict[str, str] = {}
    for c in root.iter("kafka-cluster"):
        cluster["id"] = (c.findtext("id") or "").strip()
        cluster["bootstrap"] = (c.findtext("bootstrap-servers") or "").strip()
        plain = c.find("authentication/plain")
        if plain is not None:
            cluster["username"] = (plain.findtext("username") or "").strip()
            cluster["password"] = (plain.findtext("password") or "").strip()
        break
    maps = []
    for tm in root.iter("topic-mapping"):
        filters = [(f.text or "").strip() for f in tm.iter("mqtt-topic-filter")]
        maps.append(TopicMapping((tm.findtext("id") or "").strip(), filters, (tm.findtext("kafka-topic") or "").strip()))
    return maps, cluster


class MqttBroker:
    """MQTT 3.1.1/5 broker (QoS 0-2, retained, shared subscriptions) with a Kafka bridge.

    ``kafka`` is a bootstrap list, ``fake://name`` (in-process Kafka broker) or None
    (no bridge).  ``mappings`` defaults to the reference's single mapping
    ``vehicles/sensor/data/# -> sensor-data``.
    """

    def __init__(self, port: int = 0, kafka: Optional[str] = None,
                 mappings: Optional[Sequence[TopicMapping]] = None, username: str = "", password: str = "",
                 max_qos: int = 2, kafka_config: Optional[Sequence[str]] = None, bridge_batch: int = 1024,
                 bridge_linger_ms: int = 2, metrics: bool = True):
        from ..kafka.client import parse_config, resolve_servers
        if mappings is None:
            mappings = [TopicMapping(SENSOR_KAFKA_TOPIC, [SENSOR_TOPIC_FILTER], SENSOR_KAFKA_TOPIC)]
        self.mappings = list(mappings)
        kcfg = parse_config(kafka_config)
        mech = ""
        if kcfg.get("security.protocol", "plaintext").lower() == "sasl_plaintext":
            mech = kcfg.get("sasl.mechanisms", kcfg.get("sasl.mechanism", "PLAIN")).upper()
        boot = resolve_servers(kafka) if kafka else ""
        self._b = _io().MqttBroker(port, username, password, max_qos, boot,
                                   [(m.id, list(m.filters), m.kafka_topic) for m in self.mappings], mech,
                                   kcfg.get("sasl.username", ""), kcfg.get("sasl.password", ""), bridge_batch,
                                   bridge_linger_ms)
        self._metrics_key = None
        if metrics:
            self._register_metrics()

    def _register_metrics(self) -> None:
        """Expose the broker's counters under the HiveMQ / Kafka-extension metric names the
        reference's Grafana dashboard queries (infrastructure/hivemq/hivemq.json)."""
        import weakref
        from ..obs.metrics import REGISTRY
        ref = weakref.ref(self)
        port = self.port

        def collect():
            b = ref()
            if b is None:
                return []
            st = b._b.stats()
            lab = {"broker": str(port)}
            out = [("com_hivemq_messages_incoming_publish_count", "counter", st["incoming_publish"], lab),
                   ("com_hivemq_messages_outgoing_publish_count", "counter", st["outgoing_publish"], lab),
                   ("com_hivemq_networking_connections_current", "gauge", st["connections_current"], lab),
                   ("com_hivemq_networking_connections_total_count", "counter", st["connections_total"], lab),
                   ("com_hivemq_messages_retained_current", "gauge", st["retained"], lab),
                   ("kafka_extension_total_success_count", "counter", st["kafka_sent"], lab),
                   ("kafka_extension_total_failure_count", "counter", st["kafka_failed"], lab),
                   ("kafka_extension_queue_current", "gauge", st["kafka_queued"], lab)]
            for mid, n in b._b.mapping_counts().items():
                name = "kafka_extension_topic_mapping_" + re.sub(r"[^a-zA-Z0-9_]", "_", mid) + "_send_count"
                out.append((name, "counter", n, lab))
            return out

        self._metrics_key = f"mqtt-broker-{port}-{id(self)}"
        REGISTRY.add_collector(self._metrics_key, collect)

    @property
    def port(self) -> int:
        return self._b.port

    @property
    def address(self) -> str:
        return f"127.0.0.1:{self.port}"

    def publish(self, topic: str, payload: bytes, qos: int = 0, retain: bool = False) -> None:
        self._b.publish(topic, bytes(payload), qos, retain)

    def stats(self) -> Dict[str, int]:
        """HiveMQ-style counters (incoming publishes, connections, Kafka send count, ...)."""
        return self._b.stats()

    def mapping_counts(self) -> Dict[str, int]:
        """Records produced per topic mapping (``kafka_extension_topic_mapping_<id>_send_count``)."""
        return self._b.mapping_counts()

    def flush(self, timeout_s: float = 10.0) -> bool:
        return self._b.flush(int(timeout_s * 1000))

    def stop(self) -> None:
        self._b.stop()
        if self._metrics_key:
            from ..obs.metrics import REGISTRY
            REGISTRY.remove_collector(self._metrics_key)
            self._metrics_key = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.stop()


class MqttClient:
    """Blocking MQTT client (v3.1.1 = 4, v5 = 5)."""

    def __init__(self):
        self._c = _io().MqttClient()

    def connect(self, host: str, port: int, client_id: str, version: int = 5, keepalive: int = 60,
                clean: bool = True, username: str = "", password: str = "", timeout_s: float = 5.0) -> int:
        return self._c.connect(host, int(port), client_id, version, keepalive, clean, username, password,
                               int(timeout_s * 1000))

    def publish(self, topic: str, payload: bytes, qos: int = 0, retain: bool = False) -> None:
        self._c.publish(topic, bytes(payload), qos, retain)

    def subscribe(self, *filters: Tuple[str, int]) -> List[int]:
        return self._c.subscribe([(f, int(q)) for f, q in filters])

    def unsubscribe(self, *filters: str) -> None:
        self._c.unsubscribe(list(filters))

    def receive(self, timeout_s: float = 1.0):
        """``(topic, payload, qos, retain)`` or None on timeout."""
        return self._c.receive(int(timeout_s * 1000))

    def ping(self, timeout_s: float = 2.0) -> bool:
        return self._c.ping(int(timeout_s * 1000))

    def disconnect(self) -> None:
        self._c.disconnect()

    @property
    def connected(self) -> bool:
        return self._c.connected

    @property
    def session_present(self) -> bool:
        return self._c.session_present


# ---- device simulator -------------------------------------------------------------
_DURATION = re.compile(r"^\s*(\d+(?:\.\d+)?)\s*(ms|s|m|h)?\s*$")


def _seconds(text: str) -> float:
    m = _DURATION.match(text or "0")
    if not m:
        raise ValueError(f"bad duration {text!r}")
    v = float(m.group(1))
    return v * {"ms": 1e-3, "s": 1.0, "m": 60.0, "h": 3600.0}[m.group(2) or "s"]


def _rate_interval(rate: str) -> float:
    """scenario rate ``"1/10s"`` (messages per duration) -> seconds between messages."""
    n, _, per = rate.partition("/")
    return _seconds(per or "1s") / max(float(n), 1e-9)


def _pattern_prefix(pattern: str) -> Tuple[str, int]:
    """``electric-vehicle-[0-9]{5}`` -> (``electric-vehicle-``, 5)."""
    m = re.match(r"^(.*?)\[0-9\]\{(\d+)\}$", pattern)
    if not m:
        raise ValueError(f"unsupported id pattern {pattern!r} (expected <prefix>[0-9]{{N}})")
    return m.group(1), int(m.group(2))


@dataclass
class Scenario:
    """The publishing part of a HiveMQ device-simulator scenario (``scenario.xml``)."""

    clients: int = 25
    client_prefix: str = "electric-vehicle-"
    id_digits: int = 5
    topic_prefix: str = "vehicles/sensor/data/"
    messages_per_client: int = 40
    interval_s: float = 5.0
    ramp_s: float = 0.0
    qos: int = 1
    version: int = 5
    broker: Tuple[str, int] = ("127.0.0.1", 1883)
    payload: str = "com.hivemq.CarDataPayloadGenerator"
    extra: Dict[str, str] = field(default_factory=dict)

    @classmethod
    def from_xml(cls, path_or_text: str) -> "Scenario":
        text = path_or_text
        if "<" not in path_or_text:
            with open(path_or_text) as fh:
                text = fh.read()
        root = ET.fromstring(text)
        sc = cls()
        b = root.find("brokers/broker")
        if b is not None:
            sc.broker = ((b.findtext("address") or "127.0.0.1").strip(), int(b.findtext("port") or 1883))
        groups = {g.get("id"): g for g in root.iter("clientGroup")}
        topics = {t.get("id"): t for t in root.iter("topicGroup")}
        pub = None
        for lc in root.iter("lifeCycle"):
            if lc.find("publish") is not None:
                pub = lc
                break
        if pub is None:
            raise ValueError("scenario has no publishing lifeCycle")
        g = groups[pub.get("clientGroup")]
        sc.clients = int(g.findtext("count") or 1)
        sc.version = 5 if (g.findtext("mqttVersion") or "5").strip() == "5" else 4
        sc.client_prefix, sc.id_digits = _pattern_prefix((g.findtext("clientIdPattern") or "").strip())
        p = pub.find("publish")
        tg = topics[p.get("topicGroup")]
        tprefix, tdigits = _pattern_prefix((tg.findtext("topicNamePattern") or "").strip())
        if not tprefix.endswith(sc.client_prefix):
            raise ValueError("topic pattern must end with the client id pattern (one topic per car)")
        sc.topic_prefix = tprefix[: len(tprefix) - len(sc.client_prefix)]
        sc.messages_per_client = int(p.get("count", "1"))
        sc.interval_s = _rate_interval(p.get("rate", "1/1s"))
        sc.qos = int(p.get("qos", "0"))
        sc.payload = p.get("payloadGeneratorType", sc.payload)
        ramp = pub.find("rampUp")
        sc.ramp_s = _seconds(ramp.get("duration", "0s")) if ramp is not None else 0.0
        return sc

    def scaled(self, clients: Optional[int] = None, messages: Optional[int] = None,
               interval_s: Optional[float] = None, ramp_s: Optional[float] = None) -> "Scenario":
        """A smaller / faster copy (e.g. 100 000 cars -> a few hundred for a test run)."""
        import copy
        s = copy.deepcopy(self)
        if clients is not None:
            s.clients = int(clients)
        if messages is not None:
            s.messages_per_client = int(messages)
        if interval_s is not None:
            s.interval_s = float(interval_s)
        if ramp_s is not None:
            s.ramp_s = float(ramp_s)
        return s

    @property
    def events(self) -> int:
        return self.clients * self.messages_per_client

    @property
    def rate_per_s(self) -> float:
        return self.clients / self.interval_s


def raise_nofile_limit() -> int:
    """Raise this process's descriptor limit to its hard limit (a simulator agent or broker
    node holds one socket per connected car); returns the new soft limit."""
    import resource
    soft, hard = resource.getrlimit(resource.RLIMIT_NOFILE)
    if hard == resource.RLIM_INFINITY:
        hard = 1 << 20
    if soft < hard:
        try:
            resource.setrlimit(resource.RLIMIT_NOFILE, (hard, hard))
            soft = hard
        except (ValueError, OSError):
            pass
    return int(soft)


def simulate(scenario: Scenario, host: Optional[str] = None, port: Optional[int] = None, threads: int = 4,
             seed: int = 0, failure_rate: float = 0.01, username: str = "", password: str = "",
             id_offset: int = 0, paced: bool = False, start_at_unix: float = 0.0, stamp_ns: bool = False,
             source_ips: Sequence[str] = ()) -> Dict[str, float]:
    """Run the fleet: connect every client, publish ``messages_per_client`` car payloads each.

    Payloads are JSON objects with the 18 sensor fields + ``failure_occurred`` of the KSQL
    stream ``SENSOR_DATA_S``; each car has a stable operating point plus per-event noise
    drawn inside the ranges of :data:`streamml.data.cardata.SYNTH_RANGES`.  ``id_offset``
    numbers this process's cars from there (several simulator agents share one fleet).

    ``paced``: all clients connect first, then publish on a fixed schedule from one start
    (``start_at_unix``, shared by several agent processes) so the fleet offers a steady
    ``clients / interval_s`` msg/s; the stats report the connect time and how far sends fell
    behind schedule.  ``stamp_ns`` adds the CLOCK_MONOTONIC send time (``sent_ns``) to each
    payload for publish -> result latency.  ``source_ips`` spreads the clients' sockets over
    several loopback source addresses (beyond ~28k connections to one broker port).
    """
    from ..data.cardata import FEATURES, INT_FEATURES, SYNTH_RANGES
    raise_nofile_limit()
    cfg = {
        "host": host or scenario.broker[0], "port": int(port or scenario.broker[1]),
        "client_prefix": scenario.client_prefix, "id_digits": scenario.id_digits, "id_offset": int(id_offset),
        "topic_prefix": scenario.topic_prefix, "clients": scenario.clients,
        "messages_per_client": scenario.messages_per_client, "interval_s": scenario.interval_s,
        "ramp_s": scenario.ramp_s, "qos": scenario.qos, "version": scenario.version, "threads": threads,
        "seed": seed, "failure_rate": failure_rate, "username": username, "password": password,
        "lo": [float(SYNTH_RANGES[f][0]) for f in FEATURES], "hi": [float(SYNTH_RANGES[f][1]) for f in FEATURES],
        "is_int": [1 if f in INT_FEATURES else 0 for f in FEATURES],
        "paced": bool(paced), "start_at_unix": float(start_at_unix), "stamp_ns": bool(stamp_ns),
        "source_ips": [str(a) for a in source_ips],
    }
    st = _io().mqtt_simulate(cfg)
    # device-simulator agent counters (infrastructure/test-generator/devsim.json)
    from ..obs.metrics import REGISTRY
    for name, v in (("agent_connect_successful_count", st["connected"]),
                    ("agent_connect_failed_count", st["connect_failed"]),
                    ("agent_publish_outgoing_count", st["published"] + st["publish_failed"]),
                    ("agent_publish_successful_count", st["published"]),
                    ("agent_publish_error_count", st["publish_failed"])):
        REGISTRY.counter(name, "device simulator (streamml.mqtt.simulate)").inc(float(v))
    return st


def car_payload(car: int, seq: int, ts_ms: int = 0, seed: int = 0, failure_rate: float = 0.01) -> bytes:
    """One simulator payload (JSON bytes), for tests and custom feeders."""
    from ..data.cardata import FEATURES, INT_FEATURES, SYNTH_RANGES
    return _io().mqtt_car_payload({"seed": seed, "failure_rate": failure_rate,
                                   "lo": [float(SYNTH_RANGES[f][0]) for f in FEATURES],
                                   "hi": [float(SYNTH_RANGES[f][1]) for f in FEATURES],
                                   "is_int": [1 if f in INT_FEATURES else 0 for f in FEATURES]},
                                  int(car), int(seq), int(ts_ms))
