"""TensorBoard-compatible event files (no TensorFlow dependency).

The reference logs through ``tf.keras.callbacks.TensorBoard`` (notebook
Python-Tensorflow-2.0-Keras-...ipynb:866; confluent-tensorflow-io-kafka.py:54-55):
``logs/train`` and ``logs/validation`` event files with ``epoch_loss`` /
``epoch_accuracy`` scalars (decoded tags).  This writer emits the
same framing -- u64 length, masked CRC-32C of the length, the serialized
``tensorflow.Event`` protobuf, masked CRC-32C of the payload -- with a
hand-rolled protobuf encoder for the few fields needed, plus a reader used by
tests and tooling.
"""
from __future__ import annotations

import os
import socket
import struct
import time
from typing import Iterator, List, Optional, Tuple

from ..ops._ext import load_io


def _crc(data: bytes) -> int:
    return load_io().crc32c(data)


def masked_crc(data: bytes) -> int:
    c = _crc(data)
    return ((((c >> 15) | (c << 17)) & 0xFFFFFFFF) + 0xA282EAD8) & 0xFFFFFFFF


def _varint(v: int) -> bytes:
    out = bytearray()
    v &= (1 << 64) - 1
    while v >= 0x80:
        out.append((v & 0x7F) | 0x80)
        v >>= 7
    out.append(v)
    return bytes(out)


def _field(num: int, wire: int, payload: bytes) -> bytes:
    return _varint((num << 3) | wire) + payload


def _len_field(num: int, data: bytes) -> bytes:
    return _field(num, 2, _varint(len(data)) + data)


def encode_event(wall_time: float, step: int = 0, file_version: Optional[str] = None,
                 scalars: Optional[List[Tuple[str, float]]] = None) -> bytes:
    ev = _field(1, 1, struct.pack("<d", wall_time))
    if step:
        ev += _field(2, 0, _varint(step))
    if file_version is not None:
        ev += _len_field(3, file_version.encode())
    if scalars:
        summ = b""
        for tag, val in scalars:
            v = _len_field(1, tag.encode()) + _field(2, 5, struct.pack("<f", float(val)))
            summ += _len_field(1, v)
        ev += _len_field(5, summ)
    return ev


def frame_record(data: bytes) -> bytes:
    hdr = struct.pack("<Q", len(data))
    return hdr + struct.pack("<I", masked_crc(hdr)) + data + struct.pack("<I", masked_crc(data))


class EventFileWriter:
    """``events.out.tfevents.<time>.<host>.v2`` writer with scalar summaries."""

    def __init__(self, logdir: str, suffix: str = ".v2"):
        os.makedirs(logdir, exist_ok=True)
        name = f"events.out.tfevents.{int(time.time())}.{socket.gethostname()}.{os.getpid()}{suffix}"
        self.path = os.path.join(logdir, name)
        self._f = open(self.path, "wb")
        self._f.write(frame_record(encode_event(time.time(), file_version="brain.Event:2")))
        self._f.flush()

    def scalar(self, tag: str, value: float, step: int) -> None:
        self._f.write(frame_record(encode_event(time.time(), step, scalars=[(tag, value)])))

    def scalars(self, values: dict, step: int) -> None:
        self._f.write(frame_record(encode_event(time.time(), step, scalars=list(values.items()))))

    def flush(self) -> None:
        self._f.flush()

    def close(self) -> None:
        if not self._f.closed:
            self._f.close()


# ---------------------------------------------------------------------------
# reader (tests / tooling; also decodes the reference's own logs/*.v2 files)
# ---------------------------------------------------------------------------
def _read_varint(b: bytes, i: int) -> Tuple[int, int]:
    v, s = 0, 0
    while True:
        c = b[i]
        i += 1
        v |= (c & 0x7F) << s
        if not c & 0x80:
            return v, i
        s += 7


def _parse(b: bytes) -> Iterator[Tuple[int, int, object]]:
    i = 0
    while i < len(b):
        key, i = _read_varint(b, i)
        num, wire = key >> 3, key & 7
        if wire == 0:
            v, i = _read_varint(b, i)
        elif wire == 1:
            v = b[i:i + 8]
            i += 8
        elif wire == 5:
            v = b[i:i + 4]
            i += 4
        elif wire == 2:
            n, i = _read_varint(b, i)
            v = b[i:i + n]
            i += n
        else:
            raise ValueError(f"unsupported wire type {wire}")
        yield num, wire, v


def read_records(path: str, verify: bool = True) -> Iterator[bytes]:
    with open(path, "rb") as f:
        data = f.read()
    i = 0
    while i + 12 <= len(data):
        (n,) = struct.unpack_from("<Q", data, i)
        if verify and struct.unpack_from("<I", data, i + 8)[0] != masked_crc(data[i:i + 8]):
            raise ValueError("tfevents: length CRC mismatch")
        rec = data[i + 12:i + 12 + n]
        if verify and struct.unpack_from("<I", data, i + 12 + n)[0] != masked_crc(rec):
            raise ValueError("tfevents: data CRC mismatch")
        yield rec
        i += 12 + n + 4


def read_scalars(path: str) -> List[Tuple[int, float, str, float]]:
    """[(step, wall_time, tag, value)] for simple_value and scalar tensor summaries."""
    out = []
    for rec in read_records(path):
        wall, step, summ = 0.0, 0, None
        for num, wire, v in _parse(rec):
            if num == 1 and wire == 1:
                wall = struct.unpack("<d", v)[0]
            elif num == 2 and wire == 0:
                step = v
            elif num == 5 and wire == 2:
                summ = v
        if summ is None:
            continue
        for num, wire, val in _parse(summ):
            if num != 1:
                continue
            tag, sv = None, None
            for n2, w2, x in _parse(val):
                if n2 == 1:
                    tag = x.decode(errors="replace")
                elif n2 == 2 and w2 == 5:
                    sv = struct.unpack("<f", x)[0]
                elif n2 == 8 and w2 == 2:   # TensorProto (TF2 scalar summaries)
                    for n3, w3, y in _parse(x):
                        if n3 == 5 and w3 == 5:              # float_val (unpacked)
                            sv = struct.unpack("<f", y)[0]
                        elif n3 == 5 and w3 == 2 and len(y) >= 4:   # packed float_val
                            sv = struct.unpack("<f", y[:4])[0]
                        elif n3 == 4 and w3 == 2 and len(y) >= 4:   # tensor_content
                            sv = struct.unpack("<f", y[:4])[0]
            if tag is not None and sv is not None:
                out.append((step, wall, tag, sv))
    return out
