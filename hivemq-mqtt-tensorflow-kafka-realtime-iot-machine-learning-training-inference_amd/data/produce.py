"""Producers: any :class:`~streamml.data.stream.Stream` -> Confluent-framed Avro on Kafka.

Replaces the reference's test feeders: the kafka-python CSV
producer (autoencoder-anomaly-detection/Sensor-Kafka-Producer-From-CSV.py:5-15),
``kafka-avro-console-producer`` of JSON lines (LSTM-.../cardata-v1.sh:6) and the
KSQL JSON->Avro conversion (01_installConfluentPlatform.sh:242).  Records are
keyed by car id and routed with Kafka's default partitioner (murmur2 of the key,
as KSQL ``PARTITION BY CAR`` does, :249) when the topic has several partitions.
"""
from __future__ import annotations

from typing import Optional, Sequence

import numpy as np

from .avro import AvroCodec
from .cardata import FEATURES, LABEL, canonical
from .stream import LABEL_FALSE, LABEL_TRUE, Stream


def _label_text(codes: np.ndarray):
    return ["false" if c == LABEL_FALSE else ("true" if c == LABEL_TRUE else "") for c in codes]


def encode_chunk(codec: AvroCodec, x: np.ndarray, label: np.ndarray, framing: bool = True, schema_id: int = 1):
    """Raw feature rows -> (buffer, offsets) in the codec's schema field order."""
    n = len(x)
    num = np.zeros((n, len(codec.numeric_fields)), dtype=np.float64)
    for j, fname in enumerate(codec.numeric_fields):
        c = canonical(fname)
        if c in FEATURES:
            num[:, j] = x[:, FEATURES.index(c)]
    text = {}
    text_null = {}
    for fname in codec.text_fields:
        if canonical(fname) == LABEL:
            text[fname] = _label_text(label)
            text_null[fname] = (label > LABEL_TRUE).astype(np.uint8)
    return codec.encode(num, text, text_null=text_null or None, framing=framing, schema_id=schema_id)


def produce(stream: Stream, servers: str, topic: str, schema="cardata-v1", partitions: Optional[int] = None,
            partition: int = 0, schema_id: int = 1, framing: bool = True,
            config: Optional[Sequence[str]] = None, create: bool = True) -> int:
    """Encode and produce every chunk of ``stream``; returns the record count."""
    from ..kafka import KafkaClient, fake_broker

    codec = AvroCodec(schema)
    if servers.startswith("fake://") and create:
        b = fake_broker(servers[len("fake://"):] or "default")
        b.create_topic(topic, partitions or (partition + 1))
    client = KafkaClient(servers, config)
    nparts = partitions or client.partitions().get(topic, 1)
    total = 0
    for c in stream:
        buf, offs = encode_chunk(codec, c.x, c.label, framing, schema_id)
        vals = [buf[offs[i]:offs[i + 1]] for i in range(len(offs) - 1)]
        keys = c.keys
        if keys is None and "device" in c.meta:   # the simulator's MQTT client id is the record key
            keys = [f"electric-vehicle-{int(d):05d}" for d in c.meta["device"]]
        keys = None if keys is None else [k.encode() if isinstance(k, str) else k for k in keys]
        ts = c.meta.get("timestamp")
        # Kafka timestamps are epoch milliseconds; the car events carry epoch seconds
        ts = None if ts is None else (np.asarray(ts, dtype=np.int64) * (1000 if np.max(ts) < 1e11 else 1))
        if keys is not None and nparts > 1:
            from ..mqtt import kafka_partition
            parts = np.array([kafka_partition(k, nparts) for k in keys])
            for p in range(nparts):
                idx = np.nonzero(parts == p)[0]
                if len(idx):
                    client.produce(topic, p, [vals[i] for i in idx], [keys[i] for i in idx],
                                   None if ts is None else ts[idx])
        else:
            step = 8192
            for s in range(0, len(vals), step):
                client.produce(topic, partition, vals[s:s + step], None if keys is None else keys[s:s + step],
                               None if ts is None else ts[s:s + step])
        total += len(vals)
    return total
