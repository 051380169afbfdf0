"""The reference's KSQL preprocessing as a small columnar stream processor.

01_installConfluentPlatform.sh:231-256 defines, in order:

1. ``SENSOR_DATA_S``            -- JSON records of the 19 car fields on topic ``sensor-data``;
2. ``SENSOR_DATA_S_AVRO``       -- the same re-encoded as Avro (``VALUE_FORMAT='AVRO'``);
3. ``SENSOR_DATA_S_AVRO_REKEY`` -- ``SELECT ROWKEY as CAR, * ... PARTITION BY CAR``;
4. ``SENSOR_DATA_EVENTS_PER_5MIN_T`` -- ``SELECT car, count(*) as event_count ...
   WINDOW TUMBLING (SIZE 5 MINUTE) GROUP BY car``.

Steps 1-3 run as :func:`run_json_to_avro` on the JSON records the MQTT->Kafka bridge
writes to ``sensor-data`` (``streamml.mqtt``): parse, re-encode as Confluent-framed Avro
(KSQL's nullable ``KsqlDataSourceSchema``), keep the Kafka key (the MQTT topic = ROWKEY)
and partition the REKEY stream by it with Kafka's murmur2 partitioner.  Synthetic
sources skip the JSON stage (``data.produce`` writes the Avro streams directly).  Step 4
is :class:`TumblingCounter`, a
vectorised (numpy ``unique``) per-key tumbling-window count; :func:`run_events_per_window`
drives it as a Kafka-to-Kafka job whose output records are keyed
``<car>@<window_start_ms>`` with JSON values, the shape KSQL's windowed table
emits.
"""
from __future__ import annotations

import json
from typing import Dict, Iterable, List, Optional, Sequence, Tuple

import numpy as np


class TumblingCounter:
    """count(*) GROUP BY key over tumbling windows of ``window_ms``; windows close on watermark."""

    def __init__(self, window_ms: int = 5 * 60 * 1000, grace_ms: int = 0):
        self.window_ms = int(window_ms)
        self.grace_ms = int(grace_ms)
        self.counts: Dict[Tuple[str, int], int] = {}
        self.watermark = -1

    def update(self, keys: Sequence, timestamps_ms: np.ndarray) -> None:
        ts = np.asarray(timestamps_ms, dtype=np.int64)
        if len(ts) == 0:
            return
        ks = np.asarray([k.decode() if isinstance(k, (bytes, bytearray)) else str(k) for k in keys], dtype=object)
        win = (ts // self.window_ms) * self.window_ms
        # one unique() over integer (key, window) codes instead of a Python loop per event
        kuniq, kinv = np.unique(ks.astype(str), return_inverse=True)
        wuniq, winv = np.unique(win, return_inverse=True)
        code = kinv.astype(np.int64) * len(wuniq) + winv
        cu, cnt = np.unique(code, return_counts=True)
        for cc, n in zip(cu.tolist(), cnt.tolist()):
            key = (str(kuniq[cc // len(wuniq)]), int(wuniq[cc % len(wuniq)]))
            self.counts[key] = self.counts.get(key, 0) + int(n)
        self.watermark = max(self.watermark, int(ts.max()))

    def closed(self) -> List[Tuple[str, int, int]]:
        """Pop windows that ended before the watermark (minus grace): [(key, window_start, count)]."""
        limit = self.watermark - self.grace_ms
        out = [(k, w, c) for (k, w), c in self.counts.items() if w + self.window_ms <= limit]
        for k, w, _ in out:
            del self.counts[(k, w)]
        return sorted(out, key=lambda r: (r[1], r[0]))

    def table(self) -> Dict[Tuple[str, int], int]:
        return dict(self.counts)


def events_per_window(chunks: Iterable, window_s: int = 300) -> Dict[Tuple[str, int], int]:
    """Offline form: ``{(car, window_start_ms): count}`` over a Stream of chunks with keys + meta timestamps."""
    tc = TumblingCounter(window_s * 1000)
    for c in chunks:
        ts = c.meta.get("timestamp")
        if ts is None or c.keys is None:
            raise ValueError("chunks need keys and meta['timestamp'] (ms)")
        tc.update(c.keys, np.asarray(ts))
    return tc.table()


def run_events_per_window(servers: str, source_topic: str, target_topic: str, window_s: int = 300,
                          config=None, partitions: Optional[int] = None, eof: bool = True,
                          grace_s: Optional[int] = None) -> int:
    """Consume ``source_topic`` (all partitions), count per car per tumbling window, produce
    the closed windows (all windows at eof) to ``target_topic``; returns records produced.
    Partitions are read round-robin, so windows close one ``grace_s`` (default one
    window) after the watermark passes them."""
    from ..kafka import KafkaClient, KafkaDataset
    cl = KafkaClient(servers, config)
    nparts = partitions or cl.partitions().get(source_topic, 1)
    specs = [f"{source_topic}:{p}:0" for p in range(nparts)]
    tc = TumblingCounter(window_s * 1000, (window_s if grace_s is None else grace_s) * 1000)
    produced = 0

    def emit(rows):
        nonlocal produced
        if not rows:
            return
        vals = [json.dumps({"CAR": k, "WINDOW_START": w, "WINDOW_END": w + tc.window_ms, "EVENT_COUNT": c}).encode()
                for k, w, c in rows]
        keys = [f"{k}@{w}".encode() for k, w, _ in rows]
        cl.produce(target_topic, 0, vals, keys)
        produced += len(vals)

    for b in KafkaDataset(specs, servers=servers, eof=eof, config_global=config):
        tc.update(b["keys"], np.asarray(b["timestamps"], dtype=np.int64))
        emit(tc.closed())
    emit(sorted(((k, w, c) for (k, w), c in tc.counts.items()), key=lambda r: (r[1], r[0])))
    tc.counts.clear()
    return produced


def _parse_json_rows(values: bytes, voffs):
    """JSON car events (SENSOR_DATA_S columns) -> raw feature rows [n, 18] + label codes.

    Field names are matched through :func:`streamml.data.cardata.canonical` (KSQL
    upper-case, snake_case and camelCase all map).  Missing numeric fields become
    NaN (KSQL nulls); unparsable records are skipped and counted."""
    from .cardata import FEATURES, LABEL, canonical
    from .stream import LABEL_FALSE, LABEL_MISSING, LABEL_TRUE
    n = len(voffs) - 1
    x = np.full((n, len(FEATURES)), np.nan, dtype=np.float64)
    lab = np.full(n, LABEL_MISSING, dtype=np.uint8)
    ok = np.ones(n, dtype=bool)
    col = {f: i for i, f in enumerate(FEATURES)}
    bad = 0
    for i in range(n):
        try:
            rec = json.loads(values[voffs[i]:voffs[i + 1]])
        except ValueError:
            ok[i] = False
            bad += 1
            continue
        for k, v in rec.items():
            c = canonical(k)
            if c == LABEL:
                lab[i] = LABEL_TRUE if str(v).lower() == "true" else (LABEL_FALSE if str(v).lower() == "false"
                                                                    else LABEL_MISSING)
            elif c in col and v is not None:
                x[i, col[c]] = float(v)
    return x[ok], lab[ok], bad, ok


def run_json_to_avro(servers: str, source_topic: str = "sensor-data", target_topic: str = "SENSOR_DATA_S_AVRO",
                     rekey_topic: Optional[str] = "SENSOR_DATA_S_AVRO_REKEY", schema: str = "ksql-cardata-v1",
                     config=None, eof: bool = True, target_partitions: int = 1,
                     rekey_partitions: Optional[int] = None, idle_timeout_s: Optional[float] = None) -> dict:
    """KSQL steps 1-3 (01_installConfluentPlatform.sh:235-249) as one streaming job.

    ``SENSOR_DATA_S`` (JSON on ``source_topic``) -> ``SENSOR_DATA_S_AVRO`` (Avro, partition
    ``target_partitions`` spread by key) and ``SENSOR_DATA_S_AVRO_REKEY`` (same records,
    ``PARTITION BY CAR`` where CAR = ROWKEY = the MQTT topic the bridge used as key).
    Record timestamps are carried over.  Returns counts."""
    from ..kafka import KafkaClient, KafkaDataset
    from ..mqtt import kafka_partition
    from .avro import AvroCodec
    from .produce import encode_chunk
    cl = KafkaClient(servers, config)
    parts = cl.partitions()
    nsrc = parts.get(source_topic, 1)
    codec = AvroCodec(schema)
    npart_t = max(1, int(target_partitions))
    npart_r = int(rekey_partitions or parts.get(rekey_topic, npart_t) if rekey_topic else 1)
    stats = {"read": 0, "written": 0, "rekeyed": 0, "bad": 0}
    specs = [f"{source_topic}:{p}:0" for p in range(nsrc)]
    for b in KafkaDataset(specs, servers=servers, eof=eof, config_global=config, idle_timeout_s=idle_timeout_s):
        voffs = np.asarray(b["value_offsets"], dtype=np.int64)
        x, lab, bad, ok = _parse_json_rows(b["values"], voffs)
        stats["read"] += len(voffs) - 1
        stats["bad"] += bad
        if len(x) == 0:
            continue
        keys = [k for k, good in zip(b["keys"], ok) if good]
        ts = np.asarray(b["timestamps"], dtype=np.int64)[ok]
        buf, offs = encode_chunk(codec, x, lab, framing=True)
        vals = [buf[offs[i]:offs[i + 1]] for i in range(len(offs) - 1)]
        for topic, npart, counter in ((target_topic, npart_t, "written"), (rekey_topic, npart_r, "rekeyed")):
            if not topic:
                continue
            pidx = np.array([kafka_partition(k, npart) for k in keys]) if npart > 1 else np.zeros(len(keys), int)
            for p in range(npart):
                idx = np.nonzero(pidx == p)[0]
                if len(idx):
                    cl.produce(topic, p, [vals[i] for i in idx], [keys[i] for i in idx], ts[idx])
            stats[counter] += len(vals)
    return stats
