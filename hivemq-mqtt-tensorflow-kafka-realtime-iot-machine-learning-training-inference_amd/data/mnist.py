"""MNIST over Kafka: raw-byte records, IDX files and a synthetic stand-in.

Reference producer (python-scripts/tensorflow-kafka-mnist-ONLY-producer.py:9-16,
confluent-tensorflow-io-kafka.py:9-18): every training image is sent as its raw
784 ``uint8`` bytes to topic ``xx`` and its label as one raw byte to topic
``yy``.  The consumer (tensorflow-kafka-mnist.py:22-36) reads both partitions,
``decode_raw`` -> reshape ``[28, 28]`` -> ``convert_image_dtype(float32)`` (= /255)
and zips them by position.

Here both topics are fetched in bulk and decoded with one ``np.frombuffer`` per
fetch (fixed-length records, no per-message Python).  The /255 scale is applied
on the device by the model, so the H2D copy moves ``uint8`` (4x fewer bytes).

There is no network, so ``tf.keras.datasets.mnist.load_data()`` is replaced by
:func:`load_idx` (for IDX files a user already has) and :func:`synthetic_mnist`
(class-conditional 28x28 digit-like blobs; learnable, not real MNIST).
"""
from __future__ import annotations

import gzip
import os
import struct
from typing import Iterator, Optional, Tuple

import numpy as np

IMAGE_BYTES = 28 * 28


def synthetic_mnist(n: int, seed: int = 0, noise: float = 0.15) -> Tuple[np.ndarray, np.ndarray]:
    """``n`` uint8 images [n, 28, 28] + uint8 labels, 10 separable stroke-pattern classes."""
    rng = np.random.default_rng(seed)
    proto_rng = np.random.default_rng(12345)   # the class prototypes are fixed across seeds
    yy, xx = np.mgrid[0:28, 0:28].astype(np.float32)
    protos = np.zeros((10, 28, 28), np.float32)
    for c in range(10):
        for _ in range(3):  # three gaussian strokes per class
            cy, cx = proto_rng.uniform(6, 22, 2)
            sy, sx = proto_rng.uniform(1.5, 5.0, 2)
            protos[c] += np.exp(-((yy - cy) ** 2 / (2 * sy * sy) + (xx - cx) ** 2 / (2 * sx * sx)))
        protos[c] /= protos[c].max()
    labels = rng.integers(0, 10, size=n).astype(np.uint8)
    shift = rng.integers(-2, 3, size=(n, 2))
    imgs = protos[labels]
    out = np.empty((n, 28, 28), np.uint8)
    for s in range(0, n, 8192):   # bounded temporaries
        e = min(n, s + 8192)
        blk = imgs[s:e].copy()
        for dy in range(-2, 3):
            for dx in range(-2, 3):
                m = (shift[s:e, 0] == dy) & (shift[s:e, 1] == dx)
                if m.any():
                    blk[m] = np.roll(blk[m], (dy, dx), axis=(1, 2))
        blk = blk * rng.uniform(0.7, 1.0, size=(e - s, 1, 1)) + noise * rng.random(blk.shape, dtype=np.float32)
        out[s:e] = np.clip(blk * 255.0, 0, 255).astype(np.uint8)
    return out, labels


def load_idx(path: str) -> np.ndarray:
    """Read an IDX file (``train-images-idx3-ubyte[.gz]`` / labels ``idx1``)."""
    opener = gzip.open if path.endswith(".gz") else open
    with opener(path, "rb") as f:
        data = f.read()
    if len(data) < 4 or data[0] != 0 or data[1] != 0:
        raise ValueError(f"{path}: not an IDX file")
    dtype_code, ndim = data[2], data[3]
    dtypes = {0x08: np.uint8, 0x09: np.int8, 0x0B: ">i2", 0x0C: ">i4", 0x0D: ">f4", 0x0E: ">f8"}
    if dtype_code not in dtypes:
        raise ValueError(f"{path}: unknown IDX dtype 0x{dtype_code:02x}")
    dims = struct.unpack(">" + "I" * ndim, data[4:4 + 4 * ndim])
    arr = np.frombuffer(data, dtype=dtypes[dtype_code], offset=4 + 4 * ndim)
    if arr.size != int(np.prod(dims)):
        raise ValueError(f"{path}: truncated ({arr.size} of {int(np.prod(dims))} elements)")
    return arr.reshape(dims)


def write_idx(path: str, arr: np.ndarray) -> None:
    arr = np.ascontiguousarray(arr)
    codes = {np.dtype(np.uint8): 0x08, np.dtype(np.int8): 0x09}
    if arr.dtype not in codes:
        raise ValueError("write_idx supports uint8 / int8")
    head = bytes([0, 0, codes[arr.dtype], arr.ndim]) + struct.pack(">" + "I" * arr.ndim, *arr.shape)
    opener = gzip.open if path.endswith(".gz") else open
    with opener(path, "wb") as f:
        f.write(head + arr.tobytes())


def load_mnist(directory: Optional[str] = None, seed: int = 0, n_synthetic: int = 60000):
    """``(x_train, y_train), (x_test, y_test)`` from IDX files if present, else synthetic."""
    if directory:
        def find(stem):
            for suf in ("", ".gz"):
                p = os.path.join(directory, stem + suf)
                if os.path.exists(p):
                    return p
            return None
        names = ["train-images-idx3-ubyte", "train-labels-idx1-ubyte", "t10k-images-idx3-ubyte",
                 "t10k-labels-idx1-ubyte"]
        paths = [find(n) for n in names]
        if all(paths):
            a, b, c, d = (load_idx(p) for p in paths)
            return (a, b), (c, d)
    xtr, ytr = synthetic_mnist(n_synthetic, seed)
    xte, yte = synthetic_mnist(max(n_synthetic // 6, 1), seed + 1)
    return (xtr, ytr), (xte, yte)


def produce_mnist(servers: str, x: np.ndarray, y: np.ndarray, topic_x: str = "xx", topic_y: str = "yy",
                  config=None, partition: int = 0, chunk: int = 4096) -> int:
    """Reference producer: raw image bytes -> ``xx``, raw label byte -> ``yy`` (same order)."""
    from ..kafka import KafkaClient, fake_broker

    if servers.startswith("fake://"):
        b = fake_broker(servers[len("fake://"):] or "default")
        b.create_topic(topic_x, partition + 1)
        b.create_topic(topic_y, partition + 1)
    cl = KafkaClient(servers, config)
    x = np.ascontiguousarray(x, dtype=np.uint8).reshape(len(x), -1)
    y = np.ascontiguousarray(y, dtype=np.uint8).reshape(len(y), -1)
    for s in range(0, len(x), chunk):
        e = min(len(x), s + chunk)
        cl.produce(topic_x, partition, [x[i].tobytes() for i in range(s, e)])
        cl.produce(topic_y, partition, [y[i].tobytes() for i in range(s, e)])
    return len(x)


def _fixed_records(batch: dict, size: int) -> np.ndarray:
    vo = np.asarray(batch["value_offsets"], dtype=np.int64)
    lens = np.diff(vo)
    if len(lens) and (lens != size).any():
        raise ValueError(f"expected fixed {size}-byte records, got lengths {sorted(set(lens.tolist()))[:5]}")
    buf = batch["values"]
    buf = np.frombuffer(buf, dtype=np.uint8) if not isinstance(buf, np.ndarray) else buf.view(np.uint8)
    return buf[:len(lens) * size].reshape(len(lens), size)


def kafka_mnist(servers: str, topic_x: str = "xx:0", topic_y: str = "yy:0", config=None, group_x: str = "xx",
                group_y: str = "yy", eof: bool = True, chunk: int = 8 << 20) -> Iterator[Tuple[np.ndarray, np.ndarray]]:
    """Yield aligned ``(images uint8 [n, 28, 28], labels uint8 [n])`` chunks read from ``xx`` / ``yy``."""
    from ..kafka import KafkaDataset

    dx = iter(KafkaDataset([topic_x], servers=servers, group=group_x, eof=eof, config_global=config,
                           max_bytes=chunk))
    dy = iter(KafkaDataset([topic_y], servers=servers, group=group_y, eof=eof, config_global=config))
    xbuf = np.zeros((0, IMAGE_BYTES), np.uint8)
    ybuf = np.zeros((0,), np.uint8)
    while True:
        # refill the shorter side; once it is exhausted no further pair can form (zip semantics)
        if len(xbuf) <= len(ybuf):
            b = next(dx, None)
            if b is None:
                return
            xbuf = np.concatenate([xbuf, _fixed_records(b, IMAGE_BYTES)])
        else:
            b = next(dy, None)
            if b is None:
                return
            ybuf = np.concatenate([ybuf, _fixed_records(b, 1)[:, 0]])
        n = min(len(xbuf), len(ybuf))
        if n:
            yield xbuf[:n].reshape(n, 28, 28), ybuf[:n].copy()
            xbuf, ybuf = xbuf[n:], ybuf[n:]
