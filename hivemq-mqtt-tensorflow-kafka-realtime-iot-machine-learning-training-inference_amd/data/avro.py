"""Avro schema compilation + the columnar C++ codec (``streamml._io.AvroCodec``).

Equivalent of ``kafka_io.decode_avro(e, schema=..., dtype=[...])`` after the
Confluent framing strip ``tf.strings.substr(e, 5, -1)``
(AUTOENCODER-TensorFlow-IO-Kafka/cardata-v3.py:49-75): one call decodes a whole
batch of framed records into a float32 feature matrix (schema order), a null
mask and text columns.  Output dtype handling differs from the reference on
purpose: the reference decodes doubles as float64 (v3) or float32 (v1,
cardata-v1.py:16-37); we always produce float32 features (+ optional float64)
because that is what the device consumes.
"""
from __future__ import annotations

import json
import os
from dataclasses import dataclass
from typing import Dict, List, Optional, Sequence, Tuple, Union

import numpy as np

from ..ops._ext import load_io

KINDS = {"null": 0, "boolean": 1, "int": 2, "long": 3, "float": 4, "double": 5, "string": 6, "bytes": 7,
         "enum": 8, "fixed": 9}

SCHEMA_DIR = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "schemas")
BUNDLED = {
    "cardata-v1": "ksql-cardata-v1.avsc",        # KSQL nullable UPPERCASE record (what the scripts decode)
    "ksql-cardata-v1": "ksql-cardata-v1.avsc",
    "cardata-v1-source": "cardata-v1.avsc",      # com.hivemq.avro.CarData (simulator)
    "cardata-v1-compact": "cardata-v1-compact.avsc",
}


@dataclass
class FieldSpec:
    name: str
    kind: str
    nullable: bool
    null_branch: int = -1
    fixed_size: int = 0
    symbols: Tuple[str, ...] = ()

    def as_tuple(self):
        return (self.name, KINDS[self.kind], self.null_branch, self.fixed_size, len(self.symbols))


def load_schema(schema: Union[str, dict]) -> dict:
    """Accepts a parsed schema, JSON text, a bundled name or a path."""
    if isinstance(schema, dict):
        return schema
    s = schema.strip()
    if s.startswith("{"):
        return json.loads(s)
    path = os.path.join(SCHEMA_DIR, BUNDLED[s]) if s in BUNDLED else s
    with open(path) as f:
        return json.load(f)


def compile_schema(schema: Union[str, dict]) -> List[FieldSpec]:
    """Flatten a record schema of primitive / [null, T] fields into codec specs."""
    sch = load_schema(schema)
    if sch.get("type") != "record":
        raise ValueError("top-level Avro schema must be a record")
    out: List[FieldSpec] = []
    for f in sch["fields"]:
        t = f["type"]
        nullable, null_branch = False, -1
        if isinstance(t, list):
            if len(t) != 2 or "null" not in t:
                raise ValueError(f"field {f['name']}: only [null, T] unions are supported")
            null_branch = t.index("null")
            t = t[1 - null_branch]
            nullable = True
        fixed, symbols = 0, ()
        if isinstance(t, dict):
            kind = t["type"]
            if kind == "enum":
                symbols = tuple(t["symbols"])
            elif kind == "fixed":
                fixed = int(t["size"])
            elif kind not in KINDS:
                raise ValueError(f"field {f['name']}: complex type {kind!r} not supported")
            t = kind
        if t not in KINDS:
            raise ValueError(f"field {f['name']}: unsupported type {t!r}")
        out.append(FieldSpec(f["name"], t, nullable, null_branch, fixed, symbols))
    return out


class AvroCodec:
    """Batch decoder/encoder bound to one record schema."""

    def __init__(self, schema: Union[str, dict]):
        self.fields = compile_schema(schema)
        self._c = load_io().AvroCodec([f.as_tuple() for f in self.fields])
        self.numeric_fields = [f.name for f in self.fields if 1 <= KINDS[f.kind] <= 5]
        self.text_fields = [f.name for f in self.fields if KINDS[f.kind] >= 6]

    @property
    def native(self):
        return self._c

    def decode(self, records: Union[Sequence[bytes], Tuple[bytes, np.ndarray]], framing: bool = True,
               strict: bool = False, want_f64: bool = False) -> Dict[str, object]:
        """Decode a list of framed records (or a ``(buffer, offsets)`` pair)."""
        if isinstance(records, tuple) and len(records) == 2 and isinstance(records[0], (bytes, bytearray)):
            buf, offs = records
        else:
            buf = b"".join(records)
            offs = np.zeros(len(records) + 1, dtype=np.int64)
            np.cumsum([len(r) for r in records], out=offs[1:])
        out = self._c.decode(bytes(buf), np.ascontiguousarray(offs, dtype=np.int64), framing, strict, want_f64)
        out["text"] = {name: col for name, col in zip(self.text_fields, out["text"])}
        out["text_null"] = {name: col for name, col in zip(self.text_fields, out["text_null"])}
        return out

    def encode(self, numeric: np.ndarray, text: Optional[Dict[str, Sequence]] = None,
               null_mask: Optional[np.ndarray] = None, text_null: Optional[Dict[str, np.ndarray]] = None,
               framing: bool = True, schema_id: int = 1) -> Tuple[bytes, np.ndarray]:
        numeric = np.asarray(numeric, dtype=np.float64)
        n = numeric.shape[0]
        cols = []
        for name in self.text_fields:
            vals = (text or {}).get(name, [""] * n)
            cols.append([v.encode() if isinstance(v, str) else bytes(v) for v in vals])
        tn = None
        if text_null is not None:
            tn = [np.asarray(text_null.get(name, np.zeros(n, np.uint8)), dtype=np.uint8) for name in self.text_fields]
        nm = None if null_mask is None else np.asarray(null_mask, dtype=np.uint8)
        return self._c.encode(numeric, nm, cols, tn, framing, schema_id)

    def split(self, buf: bytes, offsets: np.ndarray) -> List[bytes]:
        return [buf[offsets[i]:offsets[i + 1]] for i in range(len(offsets) - 1)]


def frame(payload: bytes, schema_id: int) -> bytes:
    """Confluent wire format: magic 0x00 + 4-byte big-endian schema id + Avro body."""
    return b"\x00" + int(schema_id).to_bytes(4, "big") + payload


def unframe(msg: bytes) -> Tuple[int, bytes]:
    if len(msg) < 5 or msg[0] != 0:
        raise ValueError("not a Confluent-framed message")
    return int.from_bytes(msg[1:5], "big"), msg[5:]
