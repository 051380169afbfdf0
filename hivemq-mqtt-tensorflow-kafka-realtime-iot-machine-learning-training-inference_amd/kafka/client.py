"""Native Kafka client / in-process broker wrappers and config parsing."""
from __future__ import annotations

import threading
from typing import Dict, List, Optional, Sequence, Tuple

from ..ops._ext import load_io


def _io():
    return load_io()


class KafkaError(RuntimeError):
    pass


OFFSET_OUT_OF_RANGE = 1   # Kafka protocol error code


def error_code(exc: BaseException) -> int:
    """The Kafka protocol error code a native client error carries (``-1`` when none)."""
    return int(getattr(exc, "code", -1))


def offset_reset_policy(config) -> str:
    """``auto.offset.reset`` from librdkafka-style config: ``earliest`` (default here: a consumer
    whose position was deleted by retention loses the fewest records), ``latest``, or ``none``
    (raise).  librdkafka's aliases smallest / beginning / largest / end / error are accepted."""
    cfg = config if isinstance(config, dict) else parse_config(config)
    v = cfg.get("auto.offset.reset", "earliest").lower()
    alias = {"smallest": "earliest", "beginning": "earliest", "largest": "latest", "end": "latest",
             "error": "none"}
    v = alias.get(v, v)
    if v not in ("earliest", "latest", "none"):
        raise ValueError(f"bad auto.offset.reset {v!r}")
    return v


def parse_config(config: Optional[Sequence[str]]) -> Dict[str, str]:
    """librdkafka ``key=value`` strings (cardata-v3.py:7-15) -> dict."""
    out: Dict[str, str] = {}
    for item in config or []:
        if "=" not in item:
            raise ValueError(f"bad config entry {item!r} (expected key=value)")
        k, v = item.split("=", 1)
        out[k.strip()] = v.strip()
    return out


def parse_topic_spec(spec: str) -> Tuple[str, int, int]:
    """``"topic:partition:offset"`` (tfio convention) -> (topic, partition, offset).
    ``"topic:*:offset"`` names every partition of the topic (partition -1, expanded from the
    broker's metadata by :func:`streamml.kafka.assign.expand_specs`)."""
    parts = spec.split(":")
    topic = parts[0]
    if len(parts) > 1 and parts[1] == "*":
        partition = -1
    else:
        partition = int(parts[1]) if len(parts) > 1 and parts[1] != "" else 0
    offset = int(parts[2]) if len(parts) > 2 and parts[2] != "" else 0
    return topic, partition, offset


class FakeBroker:
    """In-process partitioned append-only log serving the Kafka protocol on 127.0.0.1."""

    def __init__(self, port: int = 0, sasl_username: str = "", sasl_password: str = "",
                 retention_records: int = -1, message_max_bytes: int = 1048588, retention_ms: int = -1,
                 retention_bytes: int = -1, retention_check_ms: int = 1000):
        """``message_max_bytes``: a produced record batch over it is refused (MESSAGE_TOO_LARGE,
        nothing appended), as a Kafka broker's ``message.max.bytes`` default; <= 0 = no cap.
        ``retention_ms`` / ``retention_bytes``: the topics' default retention.ms / retention.bytes
        (-1 = unbounded), enforced every ``retention_check_ms`` by deleting whole log segments
        (the reference's topics: retention.ms=100000, 01_installConfluentPlatform.sh:180, 183)."""
        self._b = _io().KafkaBroker(port, sasl_username, sasl_password, retention_records, message_max_bytes,
                                    retention_ms, retention_bytes, retention_check_ms)

    @property
    def port(self) -> int:
        return self._b.port

    @property
    def address(self) -> str:
        return f"127.0.0.1:{self.port}"

    def create_topic(self, name: str, partitions: int = 1, retention_ms: Optional[int] = None,
                     retention_bytes: Optional[int] = None) -> None:
        """``kafka-topics --create --partitions N [--config retention.ms=..]``: None keeps the
        broker default, -1 = unbounded."""
        self._b.create_topic(name, partitions, -2 if retention_ms is None else int(retention_ms),
                             -2 if retention_bytes is None else int(retention_bytes))

    def enforce_retention(self) -> int:
        """Run one retention pass now (the background check does the same); segments deleted."""
        return self._b.enforce_retention()

    @property
    def deleted_segments(self) -> int:
        return self._b.deleted_segments

    @property
    def deleted_records(self) -> int:
        return self._b.deleted_records

    def log_bytes(self) -> int:
        """Encoded bytes the log holds over all topics."""
        return self._b.log_bytes()

    def log_segments(self) -> int:
        return self._b.log_segments()

    def append(self, topic: str, partition: int, values: Sequence[bytes], keys=None, timestamps=None) -> int:
        return self._b.append(topic, partition, list(values), None if keys is None else list(keys),
                              None if timestamps is None else [int(t) for t in timestamps])

    def append_buffer(self, topic: str, partition: int, buf: bytes, offsets, timestamp: int = 0) -> int:
        import numpy as np
        return self._b.append_buffer(topic, partition, buf, np.ascontiguousarray(offsets, dtype=np.int64), timestamp)

    def end_offset(self, topic: str, partition: int = 0) -> int:
        return self._b.end_offset(topic, partition)

    def start_offset(self, topic: str, partition: int = 0) -> int:
        return self._b.start_offset(topic, partition)

    def read(self, topic: str, partition: int = 0, offset: int = 0, max_records: int = 1 << 30):
        return self._b.read(topic, partition, offset, max_records)

    def set_faults(self, fail_every: int = 0, delay_ms: int = 0) -> None:
        self._b.set_faults(fail_every, delay_ms)

    def set_thread_cpus(self, cpus) -> None:
        """Pin the connection threads accepted from now on to ``cpus`` (empty: unpinned)."""
        self._b.set_thread_cpus([int(c) for c in cpus])

    def set_spin_us(self, us: int) -> None:
        """Low-latency mode: connection threads and empty long polls busy-wait ``us`` first."""
        self._b.set_spin_us(int(us))

    def record_append_times(self, on: bool = True) -> None:
        """Record each appended record's steady-clock time (LogAppendTime, ns)."""
        self._b.record_append_times(bool(on))

    def append_times(self, topic: str, partition: int, start: int, count: int):
        """int64 [count]: append time (ns, the process steady clock) of each offset (-1 = none)."""
        return self._b.append_times(topic, int(partition), int(start), int(count))

    @property
    def fetch_count(self) -> int:
        return self._b.fetch_count

    @property
    def injected_failures(self) -> int:
        return self._b.injected_failures

    def stop(self) -> None:
        self._b.stop()


_FAKES: Dict[str, FakeBroker] = {}
_FAKES_LOCK = threading.Lock()


def fake_broker(name: str = "default", **kw) -> FakeBroker:
    """Process-wide named in-process broker (created on first use)."""
    with _FAKES_LOCK:
        b = _FAKES.get(name)
        if b is None:
            b = FakeBroker(**kw)
            _FAKES[name] = b
        return b


def resolve_servers(servers: str) -> str:
    if servers.startswith("fake://"):
        name = servers[len("fake://"):] or "default"
        return fake_broker(name).address
    return servers


class KafkaClient:
    """Thin wrapper over the native client; SASL/PLAIN taken from librdkafka-style config."""

    def __init__(self, servers: str, config: Optional[Sequence[str]] = None, client_id: str = "streamml",
                 timeout_ms: int = 30000):
        cfg = parse_config(config)
        proto = cfg.get("security.protocol", "plaintext").lower()
        mech = ""
        if proto in ("sasl_plaintext", "sasl_ssl"):
            if proto == "sasl_ssl":
                raise KafkaError("TLS is not supported by the native client")
            mech = cfg.get("sasl.mechanisms", cfg.get("sasl.mechanism", "PLAIN")).upper()
            if mech != "PLAIN":
                raise KafkaError(f"SASL mechanism {mech} not supported (PLAIN only)")
        self.servers = resolve_servers(servers)
        self._c = _io().KafkaClient(self.servers, cfg.get("client.id", client_id), mech,
                                    cfg.get("sasl.username", ""), cfg.get("sasl.password", ""),
                                    int(cfg.get("socket.timeout.ms", timeout_ms)))

    @property
    def native(self):
        return self._c

    def partitions(self) -> Dict[str, int]:
        return self._c.partitions()

    def earliest(self, topic: str, partition: int = 0) -> int:
        return self._c.list_offset(topic, partition, -2)

    def latest(self, topic: str, partition: int = 0) -> int:
        return self._c.list_offset(topic, partition, -1)

    def fetch(self, topic: str, partition: int, offset: int, max_bytes: int = 1 << 20, max_wait_ms: int = 100):
        return self._c.fetch(topic, partition, offset, max_bytes, max_wait_ms)

    def fetch_decode(self, codec, topic: str, partition: int, offset: int, max_bytes: int = 1 << 20,
                     max_wait_ms: int = 100, framing: bool = True, with_text: bool = True, str_keys: bool = False):
        """Fetch + Avro decode in C++ (GIL released).  ``with_text=False`` skips building
        per-record bytes objects for text columns (their label codes are always in
        ``text_codes``); ``str_keys`` returns record keys as ``str``."""
        return self._c.fetch_decode(codec.native, topic, partition, offset, max_bytes, max_wait_ms, framing,
                                    with_text, str_keys)

    def produce(self, topic: str, partition: int, values: Sequence[bytes], keys=None, timestamps=None,
                acks: int = 1) -> int:
        return self._c.produce(topic, partition, list(values), None if keys is None else list(keys),
                               None if timestamps is None else [int(t) for t in timestamps], acks)

    def commit(self, group: str, topic: str, partition: int, offset: int) -> None:
        self._c.commit(group, topic, partition, offset)

    def committed(self, group: str, topic: str, partition: int) -> int:
        return self._c.committed(group, topic, partition)

    @property
    def bytes_received(self) -> int:
        return self._c.bytes_received
