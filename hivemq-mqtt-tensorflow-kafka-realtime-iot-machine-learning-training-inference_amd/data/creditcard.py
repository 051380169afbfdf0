"""Credit-card fraud data (the D = 30 autoencoder of autoencoder-anomaly-detection/).

Reference pipeline:

* producer (Sensor-Kafka-Producer-From-CSV.py:5-15): every line of Kaggle's
  ``creditcard.csv`` (header skipped) is sent verbatim to topic ``creditcard``;
* consumer (Sensor-Kafka-Consumer-and-TensorFlow-Model-Training.py:33-44):
  ``KafkaDataset(['creditcard:0'], group='creditcard', eof=True).batch(32)``,
  ``decode_csv`` with 30 float columns + the quoted string ``Class`` column,
  x = the 30 numbers, y = ``to_number(Class)``;
* notebook preprocessing (Python-Tensorflow-2.0-Keras-Fraud-Detection-Autoencoder.ipynb):
  ``StandardScaler`` on Time and Amount, ``train_test_split(test_size=0.2,
  random_state=314)``, train on ``Class == 0`` only, score = reconstruction MSE,
  ``threshold_fixed = 5``.

The Kaggle file is not available offline; :func:`synthetic_creditcard` generates
data of the same shape (Time, V1..V28 PCA-like components, Amount, Class with a
0.172 % fraud rate) where fraud rows are shifted in a few components, so the
anomaly-detection path has signal.  :func:`parse_csv_lines` is the vectorised
``decode_csv`` (one numpy parse per fetched batch, no per-line Python).
"""
from __future__ import annotations

from typing import Iterator, List, Optional, Tuple

import numpy as np

COLUMNS = ["Time"] + [f"V{i}" for i in range(1, 29)] + ["Amount", "Class"]
NUM_FEATURES = 30
FRAUD_RATE = 492 / 284807


def synthetic_creditcard(n: int, seed: int = 0, fraud_rate: float = FRAUD_RATE) -> Tuple[np.ndarray, np.ndarray]:
    """(x [n, 30] float64: Time, V1..V28, Amount; y [n] int Class)."""
    rng = np.random.default_rng(seed)
    y = (rng.random(n) < fraud_rate).astype(np.int64)
    t = np.sort(rng.uniform(0, 172792, n))
    v = rng.standard_normal((n, 28)) * np.linspace(1.9, 0.3, 28)   # decreasing PCA variances
    shift = np.zeros(28)
    shift[[0, 2, 3, 9, 11, 13, 16]] = [-3.0, -5.0, 4.0, -5.0, -6.0, -7.0, -6.0]
    v[y == 1] = v[y == 1] * 1.8 + shift
    amount = np.round(rng.lognormal(3.0, 1.4, n), 2)
    x = np.column_stack([t, v, amount])
    return x, y


def to_csv_lines(x: np.ndarray, y: np.ndarray) -> List[bytes]:
    """Kaggle formatting: numbers then ``"0"`` / ``"1"`` (quoted Class)."""
    out = []
    for row, c in zip(x, y):
        out.append((",".join(repr(float(v)) for v in row) + f',"{int(c)}"').encode())
    return out


def header_line() -> bytes:
    return ",".join(f'"{c}"' for c in COLUMNS).encode()


def parse_csv_lines(buf: bytes, offsets: Optional[np.ndarray] = None) -> Tuple[np.ndarray, np.ndarray]:
    """Concatenated CSV records -> (x [n, 30] float64, y [n] int64) in one vectorised parse.

    ``buf`` holds the records back to back (a Kafka fetch) with record boundaries
    ``offsets`` (len n+1), or newline-separated text when ``offsets`` is None.
    """
    if offsets is not None:
        offs = np.asarray(offsets, dtype=np.int64)
        parts = [buf[offs[i]:offs[i + 1]] for i in range(len(offs) - 1)]
        text = b"\n".join(parts)
        n = len(parts)
    else:
        text = buf.strip(b"\n")
        n = text.count(b"\n") + 1 if text else 0
    if n == 0:
        return np.zeros((0, NUM_FEATURES)), np.zeros(0, np.int64)
    flat = np.array(text.replace(b'"', b"").replace(b"\n", b",").split(b","), dtype=np.float64)
    if flat.size != n * (NUM_FEATURES + 1):
        raise ValueError(f"expected {NUM_FEATURES + 1} columns per record, got {flat.size / n:.2f}")
    arr = flat.reshape(n, NUM_FEATURES + 1)
    return arr[:, :NUM_FEATURES].copy(), arr[:, NUM_FEATURES].astype(np.int64)


def load_csv(path: str) -> Tuple[np.ndarray, np.ndarray]:
    with open(path, "rb") as f:
        data = f.read()
    first_nl = data.find(b"\n")
    if first_nl >= 0 and data[:first_nl].lstrip().startswith(b'"Time"'):
        data = data[first_nl + 1:]
    return parse_csv_lines(data)


def produce_creditcard(servers: str, x: np.ndarray, y: np.ndarray, topic: str = "creditcard", config=None,
                       chunk: int = 8192) -> int:
    from ..kafka import KafkaClient, fake_broker
    if servers.startswith("fake://"):
        fake_broker(servers[len("fake://"):] or "default").create_topic(topic, 1)
    cl = KafkaClient(servers, config)
    lines = to_csv_lines(x, y)
    for s in range(0, len(lines), chunk):
        cl.produce(topic, 0, lines[s:s + chunk])
    return len(lines)


def kafka_creditcard(servers: str, topic: str = "creditcard:0", group: str = "creditcard", config=None,
                     eof: bool = True) -> Iterator[Tuple[np.ndarray, np.ndarray]]:
    from ..kafka import KafkaDataset
    for b in KafkaDataset([topic], servers=servers, group=group, eof=eof, config_global=config):
        yield parse_csv_lines(b["values"], b["value_offsets"])


def standardize_time_amount(x: np.ndarray, scaler_time=None, scaler_amount=None):
    """Notebook prep: StandardScaler on Time (col 0) and Amount (col 29); returns (x', scalers)."""
    from ..utils.evaluation import StandardScaler
    x = np.array(x, dtype=np.float64, copy=True)
    st = scaler_time or StandardScaler().fit(x[:, :1])
    sa = scaler_amount or StandardScaler().fit(x[:, 29:30])
    x[:, :1] = st.transform(x[:, :1])
    x[:, 29:30] = sa.transform(x[:, 29:30])
    return x, (st, sa)
