"""Kafka Connect sink equivalents: the digital-twin document store and the Avro data lake.

The reference runs two Kafka Connect sinks next to the ML path:

* ``MongoSinkConnector`` on ``sensor-data`` -- JSON values, ``StringConverter`` keys hoisted
  into ``_id`` by ``HoistField$Key``, one document per car in the ``sensor-data``
  collection of the ``confluent-kafka-digital-twin`` database
  (``infrastructure/kafka-connect/mongodb/mongodb-connector-configmap.yaml:6-22``);
* ``GcsSinkConnector`` on ``SENSOR_DATA_S_AVRO`` -- Avro object-container files, default
  partitioner, ``flush.size`` records per file, bucket ``car-demo-sensor-data-avro``
  (``infrastructure/kafka-connect/gcs/README.md:21-43``).

:func:`run_sink` consumes the configured topics (all partitions, committed consumer-group
offsets so a restarted sink resumes) and writes

* :class:`DocumentStore` -- a local document collection with upsert-by-``_id`` (the
  MongoDB sink's replace-one write model), persisted as JSON lines;
* :class:`AvroLake` -- Avro Object Container Files laid out as Confluent's storage
  connectors name them (``topics/<topic>/partition=<p>/<topic>+<p>+<start offset>.avro``)
  in a local directory or a ``gs://`` bucket (via :mod:`streamml.utils.model_store`).

:func:`read_avro_file` reads such files back (e.g. to train offline from the lake).
The connector JSON is read in the reference's own format (bare or ConfigMap-wrapped).
"""
from __future__ import annotations

import io
import json
import os
from typing import Dict, Iterator, List, Optional, Sequence, Tuple

AVRO_MAGIC = b"Obj\x01"


# ---- config ---------------------------------------------------------------------------
def load_connector_config(path_or_text: str) -> Dict[str, str]:
    """Connector JSON (``{"name":..., "config": {...}}`` or a bare config dict), or the
    Kubernetes ConfigMap that carries it -> flat config dict (``name`` included)."""
    text = path_or_text
    if not path_or_text.lstrip().startswith(("{", "apiVersion")) and os.path.exists(path_or_text):
        with open(path_or_text) as fh:
            text = fh.read()
    if text.lstrip().startswith("apiVersion") or "\nkind:" in text:
        import yaml
        doc = yaml.safe_load(text)
        text = next(iter(doc["data"].values()))
    doc = json.loads(text)
    cfg = dict(doc.get("config", doc))
    if "name" in doc:
        cfg.setdefault("name", doc["name"])
    return {k: (v if isinstance(v, str) else json.dumps(v) if isinstance(v, (dict, list)) else str(v).lower()
                if isinstance(v, bool) else str(v)) for k, v in cfg.items()}


# ---- Avro object container files ------------------------------------------------------
def _zigzag_long(v: int) -> bytes:
    v = (v << 1) ^ (v >> 63)
    out = bytearray()
    while True:
        b = v & 0x7F
        v >>= 7
        if v:
            out.append(b | 0x80)
        else:
            out.append(b)
            return bytes(out)


def _read_long(buf: io.BytesIO) -> int:
    shift, acc = 0, 0
    while True:
        b = buf.read(1)
        if not b:
            raise EOFError("truncated Avro long")
        acc |= (b[0] & 0x7F) << shift
        if not b[0] & 0x80:
            return (acc >> 1) ^ -(acc & 1)
        shift += 7


def _avro_bytes(b: bytes) -> bytes:
    return _zigzag_long(len(b)) + b


def write_avro_file(fh, schema_json: str, records: Sequence[bytes], sync: Optional[bytes] = None) -> None:
    """One Object Container File (codec ``null``, one block) holding already-encoded records."""
    sync = sync or os.urandom(16)
    meta = {b"avro.schema": schema_json.encode(), b"avro.codec": b"null"}
    fh.write(AVRO_MAGIC)
    fh.write(_zigzag_long(len(meta)))
    for k, v in meta.items():
        fh.write(_avro_bytes(k) + _avro_bytes(v))
    fh.write(_zigzag_long(0))
    fh.write(sync)
    if records:
        body = b"".join(records)
        fh.write(_zigzag_long(len(records)) + _zigzag_long(len(body)) + body + sync)


def read_avro_file(data: bytes) -> Tuple[str, List[bytes], int]:
    """-> (schema JSON, concatenated-record blocks, record count).  Verifies sync markers."""
    buf = io.BytesIO(data)
    if buf.read(4) != AVRO_MAGIC:
        raise ValueError("not an Avro object container file")
    meta = {}
    while True:
        n = _read_long(buf)
        if n == 0:
            break
        if n < 0:
            _read_long(buf)
            n = -n
        for _ in range(n):
            k = buf.read(_read_long(buf))
            meta[k] = buf.read(_read_long(buf))
    sync = buf.read(16)
    if meta.get(b"avro.codec", b"null") != b"null":
        raise ValueError("only the null codec is supported")
    blocks, total = [], 0
    while buf.tell() < len(data):
        cnt = _read_long(buf)
        size = _read_long(buf)
        blocks.append(buf.read(size))
        if buf.read(16) != sync:
            raise ValueError("Avro sync marker mismatch")
        total += cnt
    return meta[b"avro.schema"].decode(), blocks, total


# ---- sinks ----------------------------------------------------------------------------
class DocumentStore:
    """Document collection with upsert by ``_id`` (MongoDB sink, replace-one write model)."""

    def __init__(self, root: str, database: str, collection: str):
        self.path = os.path.join(root, database, collection + ".jsonl")
        os.makedirs(os.path.dirname(self.path), exist_ok=True)
        self.docs: Dict[str, dict] = {}
        if os.path.exists(self.path):
            with open(self.path) as fh:
                for line in fh:
                    d = json.loads(line)
                    self.docs[str(d["_id"])] = d

    def upsert(self, doc: dict) -> None:
        self.docs[str(doc["_id"])] = doc

    def flush(self) -> None:
        tmp = self.path + ".tmp"
        with open(tmp, "w") as fh:
            for d in self.docs.values():
                fh.write(json.dumps(d) + "\n")
        os.replace(tmp, self.path)

    def find(self, _id: str) -> Optional[dict]:
        return self.docs.get(str(_id))

    def __len__(self) -> int:
        return len(self.docs)


class AvroLake:
    """Rolling Avro container files per topic-partition (Confluent storage-connector layout)."""

    def __init__(self, url: str, schema_json: str, flush_size: int = 3):
        self.url = url.rstrip("/")
        self.schema_json = schema_json
        self.flush_size = max(1, int(flush_size))
        self.pending: Dict[Tuple[str, int], Tuple[int, List[bytes]]] = {}
        self.files: List[str] = []

    def _put(self, rel: str, data: bytes) -> str:
        if self.url.startswith("gs://"):
            from ..utils.model_store import open_store
            bucket, _, prefix = self.url[5:].partition("/")
            store = open_store(bucket, "gs://")
            import tempfile
            with tempfile.NamedTemporaryFile(delete=False) as tf:
                tf.write(data)
            try:
                store.upload(tf.name, (prefix + "/" if prefix else "") + rel)
            finally:
                os.unlink(tf.name)
            return f"{self.url}/{rel}"
        root = self.url[7:] if self.url.startswith("file://") else self.url
        path = os.path.join(root, rel)
        os.makedirs(os.path.dirname(path), exist_ok=True)
        with open(path + ".tmp", "wb") as fh:
            fh.write(data)
        os.replace(path + ".tmp", path)
        return path

    def add(self, topic: str, partition: int, offset: int, record: bytes) -> None:
        start, recs = self.pending.get((topic, partition), (offset, []))
        recs.append(record)
        self.pending[(topic, partition)] = (start, recs)
        if len(recs) >= self.flush_size:
            self._roll(topic, partition)

    def _roll(self, topic: str, partition: int) -> None:
        start, recs = self.pending.pop((topic, partition), (0, []))
        if not recs:
            return
        bio = io.BytesIO()
        write_avro_file(bio, self.schema_json, recs)
        rel = f"topics/{topic}/partition={partition}/{topic}+{partition}+{start:010d}.avro"
        self.files.append(self._put(rel, bio.getvalue()))

    def flush_all(self) -> None:
        """Write partial files (the connector keeps them open until flush.size; at eof we close)."""
        for topic, partition in list(self.pending):
            self._roll(topic, partition)


def _strip_framing(v: bytes) -> bytes:
    """Confluent wire format (magic 0 + 4-byte schema id) -> bare Avro record."""
    if len(v) >= 5 and v[0] == 0:
        return v[5:]
    raise ValueError("record without Confluent framing (magic byte 0)")


def run_sink(config: Dict[str, str], servers: str, store_root: str = "./connect-sink", eof: bool = True,
             kafka_config: Optional[Sequence[str]] = None, schema: str = "ksql-cardata-v1",
             idle_timeout_s: Optional[float] = None) -> Dict[str, int]:
    """Run one sink connector over ``config['topics']`` until the partitions' ends (``eof``)
    or ``idle_timeout_s`` without data; resumes from the committed ``connect-<name>`` offsets."""
    from ..kafka import KafkaClient, KafkaDataset
    cls = config.get("connector.class", "")
    topics = [t.strip() for t in config.get("topics", "").split(",") if t.strip()]
    if not topics:
        raise ValueError("connector config has no 'topics'")
    group = "connect-" + config.get("name", "sink")
    cl = KafkaClient(servers, kafka_config)
    parts = cl.partitions()
    specs = [f"{t}:{p}:0" for t in topics for p in range(parts.get(t, 1))]
    stats = {"records": 0, "documents": 0, "files": 0, "skipped": 0}
    if cls.endswith("MongoSinkConnector"):
        hoist = config.get("transforms.WrapKey.field", "_id") if "WrapKey" in config.get("transforms", "") else None
        store = DocumentStore(store_root, config.get("database", "db"), config.get("collection", topics[0]))
        for b in KafkaDataset(specs, servers=servers, group=group, eof=eof, config_global=kafka_config,
                              commit=True, resume=True, idle_timeout_s=idle_timeout_s):
            vals, voffs = b["values"], b["value_offsets"]
            for i, key in enumerate(b["keys"]):
                try:
                    doc = json.loads(vals[voffs[i]:voffs[i + 1]])
                except ValueError:
                    stats["skipped"] += 1
                    continue
                if not isinstance(doc, dict):
                    doc = {"value": doc}
                if hoist:
                    doc[hoist] = key.decode(errors="replace")
                doc.setdefault("_id", f"{b['topic']}-{b['partition']}-{int(b['offsets'][i])}")
                store.upsert(doc)
                stats["records"] += 1
            store.flush()
        stats["documents"] = len(store)
    elif cls.endswith("GcsSinkConnector") or cls.endswith("S3SinkConnector") or cls.endswith("StorageSinkConnector"):
        from ..data.avro import load_schema
        bucket = config.get("gcs.bucket.name") or config.get("s3.bucket.name") or "bucket"
        url = store_root if "://" in store_root else os.path.join(store_root, bucket)
        lake = AvroLake(url, json.dumps(load_schema(schema)), int(config.get("flush.size", "3")))
        for b in KafkaDataset(specs, servers=servers, group=group, eof=eof, config_global=kafka_config,
                              commit=True, resume=True, idle_timeout_s=idle_timeout_s):
            vals, voffs = b["values"], b["value_offsets"]
            for i in range(len(b["offsets"])):
                try:
                    rec = _strip_framing(vals[voffs[i]:voffs[i + 1]])
                except ValueError:
                    stats["skipped"] += 1
                    continue
                lake.add(b["topic"], b["partition"], int(b["offsets"][i]), rec)
                stats["records"] += 1
        lake.flush_all()
        stats["files"] = len(lake.files)
    else:
        raise ValueError(f"unsupported connector.class {cls!r} (MongoSinkConnector, GcsSinkConnector)")
    return stats


def record_offsets(body: bytes, n: int, fields) -> List[int]:
    """Boundaries of ``n`` back-to-back binary records of a flat record schema (container
    blocks carry no per-record lengths): walks union indices, varints and lengths."""
    b = io.BytesIO(body)
    offs = [0]
    for _ in range(n):
        for f in fields:
            if f.nullable and _read_long(b) == f.null_branch:
                continue
            k = f.kind
            if k in ("int", "long", "enum"):
                _read_long(b)
            elif k == "boolean":
                b.read(1)
            elif k == "float":
                b.read(4)
            elif k == "double":
                b.read(8)
            elif k in ("string", "bytes"):
                b.read(_read_long(b))
            elif k == "fixed":
                b.read(f.fixed_size)
        offs.append(b.tell())
    if offs[-1] > len(body):
        raise ValueError("records run past the block")
    return offs


def iter_lake_records(root: str, schema: str = "ksql-cardata-v1") -> Iterator[Tuple[str, dict]]:
    """Decode every record of every ``.avro`` file under ``root`` -> (path, decoded batch dict)."""
    import glob
    import numpy as np
    from ..data.avro import AvroCodec
    codec = AvroCodec(schema)
    for path in sorted(glob.glob(os.path.join(root, "**", "*.avro"), recursive=True)):
        with open(path, "rb") as fh:
            _, blocks, n = read_avro_file(fh.read())
        body = b"".join(blocks)
        offs = np.asarray(record_offsets(body, n, codec.fields), dtype=np.int64)
        yield path, codec.decode((body, offs), framing=False)
