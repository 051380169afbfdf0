"""TensorBoard-compatible event files (no TensorFlow dependency).

The reference logs through ``tf.keras.callbacks.TensorBoard`` (notebook
Python-Tensorflow-2.0-Keras-...ipynb:866; confluent-tensorflow-io-kafka.py:54-55):
``logs/train`` and ``logs/validation`` event files with ``epoch_loss`` /
``epoch_accuracy`` scalars, a ``keras`` model-config summary, and (``histogram_freq``,
``write_images``) per-weight histograms and images (decoded tags).
This writer emits the same framing -- u64 length, masked CRC-32C of the length, the
serialized ``tensorflow.Event`` protobuf, masked CRC-32C of the payload -- with a
hand-rolled protobuf encoder for the fields needed (``Summary.Value`` simple_value /
image / histo / tensor + metadata), plus a reader used by tests and tooling.
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


def _dbl(num: int, v: float) -> bytes:
    return _field(num, 1, struct.pack("<d", float(v)))


def _packed_doubles(num: int, vals) -> bytes:
    return _len_field(num, b"".join(struct.pack("<d", float(x)) for x in vals))


def histogram_proto(values, bins: int = 30) -> bytes:
    """``tensorflow.HistogramProto`` of ``values``: min, max, num, sum, sum of squares and
    ``bins`` equal-width buckets (the right edge of each in ``bucket_limit``) -- the TF2
    ``tf.summary.histogram`` bucketing (30 buckets over [min, max])."""
    import numpy as np
    v = np.asarray(values, dtype=np.float64).ravel()
    v = v[np.isfinite(v)]
    if v.size == 0:
        return _dbl(1, 0.0) + _dbl(2, 0.0) + _dbl(3, 0.0) + _dbl(4, 0.0) + _dbl(5, 0.0)
    lo, hi = float(v.min()), float(v.max())
    if hi == lo:
        limits, counts = [hi], [float(v.size)]
    else:
        counts, edges = np.histogram(v, bins=bins, range=(lo, hi))
        limits = list(edges[1:])
        counts = [float(c) for c in counts]
    return (_dbl(1, lo) + _dbl(2, hi) + _dbl(3, float(v.size)) + _dbl(4, float(v.sum())) +
            _dbl(5, float((v * v).sum())) + _packed_doubles(6, limits) + _packed_doubles(7, counts))


def png_gray(img) -> bytes:
    """8-bit grayscale PNG of a 2-D array (min..max -> 0..255), stdlib zlib only."""
    import zlib

    import numpy as np
    a = np.asarray(img, dtype=np.float64)
    lo, hi = (float(a.min()), float(a.max())) if a.size else (0.0, 0.0)
    q = np.zeros(a.shape, np.uint8) if hi <= lo else np.round((a - lo) / (hi - lo) * 255.0).astype(np.uint8)
    h, w = q.shape
    raw = b"".join(b"\x00" + q[r].tobytes() for r in range(h))

    def chunk(kind: bytes, data: bytes) -> bytes:
        return struct.pack(">I", len(data)) + kind + data + struct.pack(">I", zlib.crc32(kind + data) & 0xFFFFFFFF)

    return (b"\x89PNG\r\n\x1a\n" + chunk(b"IHDR", struct.pack(">IIBBBBB", w, h, 8, 0, 0, 0, 0)) +
            chunk(b"IDAT", zlib.compress(raw)) + chunk(b"IEND", b""))


def encode_value_event(wall_time: float, step: int, value: bytes) -> bytes:
    """An Event carrying one pre-encoded ``Summary.Value``."""
    ev = _field(1, 1, struct.pack("<d", wall_time))
    if step:
        ev += _field(2, 0, _varint(step))
    return ev + _len_field(5, _len_field(1, value))


def histo_value(tag: str, values) -> bytes:
    return _len_field(1, tag.encode()) + _len_field(5, histogram_proto(values))


def image_value(tag: str, img) -> bytes:
    import numpy as np
    a = np.atleast_2d(np.asarray(img))
    im = (_field(1, 0, _varint(a.shape[0])) + _field(2, 0, _varint(a.shape[1])) + _field(3, 0, _varint(1)) +
          _len_field(4, png_gray(a)))
    return _len_field(1, tag.encode()) + _len_field(4, im)


def text_tensor_value(tag: str, text: str, plugin: str, content: bytes = b"") -> bytes:
    """A scalar DT_STRING tensor summary with plugin metadata (the ``keras`` model summary
    TF2's TensorBoard callback writes: plugin ``graph_keras_model``, text = model JSON)."""
    meta = _len_field(1, _len_field(1, plugin.encode()) + (_len_field(2, content) if content else b""))
    tensor = _field(1, 0, _varint(7)) + _len_field(2, b"") + _len_field(8, text.encode())
    return _len_field(1, tag.encode()) + _len_field(8, tensor) + _len_field(9, meta)   # field order as TF writes


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

    def histogram(self, tag: str, values, step: int) -> None:
        self._f.write(frame_record(encode_value_event(time.time(), step, histo_value(tag, values))))

    def image(self, tag: str, img, step: int) -> None:
        self._f.write(frame_record(encode_value_event(time.time(), step, image_value(tag, img))))

    def text_tensor(self, tag: str, text: str, step: int, plugin: str, content: bytes = b"") -> None:
        self._f.write(frame_record(encode_value_event(time.time(), step, text_tensor_value(tag, text, plugin, content))))

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


def read_values(path: str) -> List[Tuple[int, str, str, object]]:
    """[(step, tag, kind, payload)] of every summary value: kind ``scalar`` (float),
    ``histo`` (dict: min, max, num, sum, sum_squares, bucket_limit, bucket), ``image``
    (dict: height, width, png bytes), ``tensor`` (dict: plugin, strings)."""
    out = []
    for rec in read_records(path):
        step, summ = 0, None
        for num, wire, v in _parse(rec):
            if num == 2 and wire == 0:
                step = v
            elif num == 5 and wire == 2:
                summ = v
        if summ is None:
            continue
        for num, _, val in _parse(summ):
            if num != 1:
                continue
            tag, kind, pay, plugin = None, None, None, None
            for n2, w2, x in _parse(val):
                if n2 == 1:
                    tag = x.decode(errors="replace")
                elif n2 == 2 and w2 == 5:
                    kind, pay = "scalar", struct.unpack("<f", x)[0]
                elif n2 == 5:
                    h = {"bucket_limit": [], "bucket": []}
                    for n3, w3, y in _parse(x):
                        if w3 == 1:
                            h[{1: "min", 2: "max", 3: "num", 4: "sum", 5: "sum_squares"}[n3]] = struct.unpack("<d", y)[0]
                        elif w3 == 2:
                            h["bucket_limit" if n3 == 6 else "bucket"] = list(struct.unpack(f"<{len(y) // 8}d", y))
                    kind, pay = "histo", h
                elif n2 == 4:
                    im = {}
                    for n3, _w3, y in _parse(x):
                        im[{1: "height", 2: "width", 3: "colorspace", 4: "png"}[n3]] = y
                    kind, pay = "image", im
                elif n2 == 9:
                    for n3, _w3, y in _parse(x):
                        if n3 == 1:
                            for n4, _w4, z in _parse(y):
                                if n4 == 1:
                                    plugin = z.decode()
                elif n2 == 8:
                    strs = [y for n3, _w3, y in _parse(x) if n3 == 8]
                    kind, pay = "tensor", {"strings": strs}
            if kind == "tensor":
                pay["plugin"] = plugin
            if tag is not None and kind is not None:
                out.append((step, tag, kind, pay))
    return out


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
