"""Low-latency streaming scorer (``csrc/io/scoreloop.cpp``): ``serve --low-latency``.

One C++ thread per replica runs Kafka long-poll fetch -> Avro decode -> persistent GPU
scorer (:class:`streamml.ops.serve.ScoringServer`, no launch per event) -> result-record
formatting (byte-identical to ``cli/serve.py``'s ``json.dumps`` / ``np.array2string``)
-> one produce per fetch -> offset commit.  No Python runs per event or per batch.
Reference: AUTOENCODER-TensorFlow-IO-Kafka/cardata-v3.py:235-279 (predict + output
callback), which batches events and formats every output in Python.
"""
from __future__ import annotations

from typing import Optional, Sequence

import numpy as np

from ..ops._ext import load_io
from .client import KafkaClient
from .feed import _auth


def feature_fields(schema: str = "cardata-v1"):
    """(codec, schema field index of every model feature, in model column order)."""
    from ..data.avro import AvroCodec
    from ..data.cardata import FEATURES, canonical
    codec = AvroCodec(schema)
    names = [f.name for f in codec.fields]
    idx = []
    for name in FEATURES:
        match = [f for f in codec.numeric_fields if canonical(f) == name]
        if not match:
            raise ValueError(f"schema has no field for feature {name}")
        idx.append(names.index(match[0]))
    return codec, idx


def json_columns():
    """(key, model column) of every car feature for JSON source records (the C++ decoder
    canonicalises keys: KSQL UPPERCASE, the simulator's snake_case and camelCase all match)."""
    from ..data.cardata import FEATURES
    return [(name, i) for i, name in enumerate(FEATURES)]


class LowLatencyScorer:
    """``scorer``: a :class:`~streamml.ops.serve.ScoringServer`, a
    :class:`~streamml.ops.serve.LSTMScoringServer` (keyed: each record key -- the car -- gets
    a device slot holding its window, mapped in C++ on first sight), or anything with a
    ``c_api()`` returning an ``SmlScorerApi`` table address (``_io.EchoScorer`` in CPU
    tests).  Keep the scorer alive while the loop runs.  ``spin_us`` > 0 busy-polls each
    broker response that long before blocking (a blocked recv costs a thread wake-up).

    ``source_format="json"`` follows JSON car events -- the MQTT bridge's ``sensor-data``
    topic, KSQL's SENSOR_DATA_S -- instead of Confluent Avro; ``json_stamp`` names a numeric
    field copied into the latency records (the device simulator's ``sent_ns``)."""

    def __init__(self, servers: str, topic: str, result_topic: str, partitions: Sequence[int], scorer,
                 schema: str = "cardata-v1", group: Optional[str] = None, starts: Optional[Sequence[int]] = None,
                 result_partitions: Optional[Sequence[int]] = None, emit_recon: bool = False,
                 config: Optional[Sequence[str]] = None, max_batch: int = 4096, max_bytes: int = 1 << 20,
                 max_wait_ms: int = 100, commit_interval_s: float = 0.0, record_latency: bool = False,
                 framing: bool = True, spin_us: int = 0, source_format: str = "avro", json_stamp: str = "",
                 hash_ranges: Optional[Sequence] = None):
        """``hash_ranges``: one ``(lo, hi)`` key-hash share per partition (kafka/assign.py
        ``key_shares``); records whose key hashes outside it are another replica's cars
        (skipped, counted as ``foreign``)."""
        client = KafkaClient(servers, config)
        self.partitions = [int(p) for p in partitions]
        if starts is None:   # committed offset of the group, else the log start
            starts = []
            for p in self.partitions:
                s = client.committed(group, topic, p) if group else -1
                starts.append(s if s >= 0 else client.earliest(topic, p))
        if source_format not in ("avro", "json"):
            raise ValueError(f"source_format must be 'avro' or 'json', not {source_format!r}")
        if result_partitions is None:
            nres = max(1, client.partitions().get(result_topic, 1))
            result_partitions = [p % nres for p in self.partitions]
        codec, fields = feature_fields(schema)
        self._scorer = scorer
        cid, mech, user, pw, tmo = _auth(config)
        api = scorer.c_api() if hasattr(scorer, "c_api") else scorer._s.c_api()
        from .client import offset_reset_policy
        # auto.offset.reset for a position deleted by retention while the loop runs (the
        # result's reset_skipped counts the records jumped over)
        reset = {"earliest": 0, "latest": 1, "none": 2}[offset_reset_policy(config)]
        self._loop = load_io().ScoreLoop(client.servers, cid, mech, user, pw, tmo,
                                         [fs.as_tuple() for fs in codec.fields], topic, result_topic, group or "",
                                         self.partitions, [int(s) for s in starts],
                                         [int(r) for r in result_partitions], fields, framing, bool(emit_recon),
                                         int(max_batch), int(max_bytes), int(max_wait_ms), float(commit_interval_s),
                                         bool(record_latency), int(api), int(spin_us),
                                         json_columns() if source_format == "json" else [], str(json_stamp),
                                         [(int(lo), int(hi)) for lo, hi in (hash_ranges or [])], reset)

    def run(self, max_events: int = 0, idle_timeout_s: Optional[float] = None) -> dict:
        """Blocking (GIL released): until ``stop()``, ``max_events`` or ``idle_timeout_s``
        without records.  Returns per-stage counters and seconds."""
        return dict(self._loop.run(int(max_events), -1.0 if idle_timeout_s is None else float(idle_timeout_s)))

    def stop(self) -> None:
        self._loop.stop()

    def positions(self):
        return list(self._loop.positions())

    def latency_bytes(self) -> int:
        """Bytes held by the latency records so far (safe to read while ``run`` is going)."""
        return int(self._loop.latency_bytes())

    def latency_records(self) -> np.ndarray:
        """[n, 7] int64: (partition, offset, steady-clock ns the result became visible (produce
        ack), of the fetch response that carried the event, of its score, of its formatted
        record, the record's ``json_stamp`` field or 0) -- the same clock as the broker's
        append times."""
        return self._loop.latency_records()


def paced_produce(servers: str, topic: str, partition: int, values: bytes, offsets, keys=None,
                  qps: float = 10000.0, spin_us: int = 0) -> np.ndarray:
    """Append records one produce request each at ``qps`` (C++, GIL released); returns
    the steady-clock send time (ns) of every record (same clock as latency_records)."""
    from .client import resolve_servers
    return load_io().paced_produce(resolve_servers(servers), topic, int(partition), values,
                                   [int(o) for o in offsets], keys, float(qps), int(spin_us))
