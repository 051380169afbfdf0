"""Columnar streaming datasets: sources + tf.data-style transforms.

The reference builds its input with tf.data ops over one decoded record at a
time (cardata-v3.py:197-218):

    kafka_dataset -> map(normalize_fn) -> filter(y == "false") -> map(x)
    -> zip((x, x)) -> batch(B) -> take(100)

and for the LSTM (LSTM-.../cardata-v2.py:199-206) ``window(look_back, shift=1)``
+ ``skip(look_back)`` + ``zip`` + ``batch(1)`` + ``take(1000)``.

Here every stage works on *columnar chunks* (:class:`Chunk`: raw feature matrix
[n, 18] float32 in :data:`FEATURES` order + label codes + keys), so the per-row
Python cost disappears.  Normalisation is deliberately NOT a host stage on the
GPU path: the train / score kernels apply ``normalize_fn`` as a fused affine map
on load; :meth:`Stream.normalize` exists for the CPU path and for oracles.
"""
from __future__ import annotations

import json
from dataclasses import dataclass, field
from typing import Callable, Iterable, Iterator, List, Optional, Sequence

import numpy as np

from .cardata import FEATURES, LABEL, NUM_FEATURES, SyntheticCarSource, canonical, load_csv, normalize_np

LABEL_FALSE, LABEL_TRUE, LABEL_MISSING = 0, 1, 2


def label_codes(values: Sequence, null: Optional[np.ndarray] = None) -> np.ndarray:
    """``failure_occurred`` strings -> 0 ("false") / 1 ("true") / 2 (missing / other)."""
    out = np.full(len(values), LABEL_MISSING, dtype=np.uint8)
    for i, v in enumerate(values):
        s = v.decode() if isinstance(v, (bytes, bytearray)) else (v if isinstance(v, str) else "")
        s = s.strip().lower()
        if s == "false":
            out[i] = LABEL_FALSE
        elif s == "true":
            out[i] = LABEL_TRUE
    if null is not None:
        out[np.asarray(null, dtype=bool)] = LABEL_MISSING
    return out


@dataclass
class Chunk:
    x: np.ndarray                                    # [n, 18] float32 raw features
    label: np.ndarray                                # [n] uint8 codes
    keys: Optional[List] = None                      # record keys (car id) if known
    offsets: Optional[np.ndarray] = None             # source offsets (Kafka) if known
    meta: dict = field(default_factory=dict)

    def __len__(self) -> int:
        return int(self.x.shape[0])

    def select(self, mask_or_idx) -> "Chunk":
        keys = None
        if self.keys is not None:
            if isinstance(mask_or_idx, slice):
                keys = self.keys[mask_or_idx]
            else:
                sel = np.asarray(mask_or_idx)
                idx = np.nonzero(sel)[0] if sel.dtype == bool else sel
                keys = [self.keys[i] for i in idx]
        return Chunk(self.x[mask_or_idx], self.label[mask_or_idx], keys,
                     None if self.offsets is None else self.offsets[mask_or_idx], dict(self.meta))

    @staticmethod
    def concat(chunks: Sequence["Chunk"]) -> "Chunk":
        keys = None
        if chunks and all(c.keys is not None for c in chunks):
            keys = [k for c in chunks for k in c.keys]
        offs = None
        if chunks and all(c.offsets is not None for c in chunks):
            offs = np.concatenate([c.offsets for c in chunks])
        return Chunk(np.concatenate([c.x for c in chunks]), np.concatenate([c.label for c in chunks]), keys, offs)


class Stream:
    """A lazy, re-iterable chain of chunk transforms (each ``iter`` restarts the source)."""

    # (rank, world) when this stream yields only one data-parallel rank's share of its
    # source (``kafka(shard=...)``); transforms keep it, ``fit`` trains on it unsharded
    shard = None

    def __init__(self, factory: Callable[[], Iterator[Chunk]], shard=None):
        self._factory = factory
        self.shard = shard

    def __iter__(self) -> Iterator[Chunk]:
        return self._factory()

    def _derive(self, factory: Callable[[], Iterator[Chunk]]) -> "Stream":
        return Stream(factory, self.shard)

    # --- transforms ---------------------------------------------------------
    def map(self, fn: Callable[[Chunk], Chunk]) -> "Stream":
        return self._derive(lambda: (fn(c) for c in self))

    def filter_label(self, keep: int = LABEL_FALSE, device: bool = False) -> "Stream":
        """``filter(lambda x, y: y == "false")`` (cardata-v3.py:212).

        ``device=True`` marks the filter as deferrable: host iteration still filters
        here, but a GPU consumer (``DeviceLoader`` via ``Autoencoder.fit``) ships the
        unfiltered rows + labels and compacts them with the K8 HIP kernel instead."""
        def gen():
            for c in self:
                m = c.label == keep
                if m.any():
                    yield c.select(m)
        out = self._derive(gen)
        if device:
            out.device_filter = (self, int(keep))
        return out

    def filter_normal(self, device: bool = False) -> "Stream":
        return self.filter_label(LABEL_FALSE, device=device)

    def normalize(self) -> "Stream":
        """Host-side ``normalize_fn`` (CPU path / oracles only)."""
        return self.map(lambda c: Chunk(normalize_np(c.x).astype(np.float32), c.label, c.keys, c.offsets, c.meta))

    def batch(self, batch_size: int, drop_remainder: bool = False) -> "Stream":
        """Re-chunk to exactly ``batch_size`` rows (last one short unless dropped)."""
        B = int(batch_size)

        def gen():
            buf: List[Chunk] = []
            have = 0
            for c in self:
                buf.append(c)
                have += len(c)
                while have >= B:
                    cat = Chunk.concat(buf)
                    yield cat.select(slice(0, B))
                    rest = cat.select(slice(B, None))
                    buf, have = ([rest] if len(rest) else []), len(rest)
            if have and not drop_remainder:
                yield Chunk.concat(buf)
        return self._derive(gen)

    def take(self, n: int) -> "Stream":
        def gen():
            for i, c in enumerate(self):
                if i >= n:
                    return
                yield c
        return self._derive(gen)

    def skip(self, n: int) -> "Stream":
        def gen():
            for i, c in enumerate(self):
                if i >= n:
                    yield c
        return self._derive(gen)

    def windows(self, look_back: int, horizon: int = 1) -> "WindowStream":
        """Sliding windows for next-event prediction (LSTM-.../cardata-v2.py:199-206).

        Yields ``(x [n, look_back, F], y [n, F])`` where ``y`` is the row
        ``horizon`` steps after each window's last row; windows span chunk
        boundaries (a carry of ``look_back + horizon - 1`` rows is kept).
        """
        return WindowStream(self, look_back, horizon)

    def collect(self) -> Chunk:
        return Chunk.concat(list(self))


class WindowStream:
    def __init__(self, base: Stream, look_back: int, horizon: int = 1):
        self.base, self.T, self.h = base, int(look_back), int(horizon)

    def __iter__(self):
        carry = np.zeros((0, NUM_FEATURES), dtype=np.float32)
        need = self.T + self.h - 1
        for c in self.base:
            rows = np.concatenate([carry, c.x]) if len(carry) else c.x
            n = rows.shape[0] - need
            if n > 0:
                idx = np.arange(n)[:, None] + np.arange(self.T)[None, :]
                yield rows[idx], rows[np.arange(n) + need]
            carry = rows[-need:] if need > 0 else rows[:0]


def sliding_windows(rows, look_back: int, horizon: int = 1):
    """Device-side ``window(look_back, shift=1)`` + ``skip(look_back)`` targets
    (LSTM-TensorFlow-IO-Kafka/cardata-v2.py:199-206) WITHOUT materialising the windows:
    ``X[b] = rows[b : b + look_back]`` is a strided view ``[n, T, F]`` with sequence
    stride F (one row), ``Y[b] = rows[b + look_back + horizon - 1]``.  The fused LSTM
    kernels read X in place (each base row is fetched once per window that contains it,
    from L2 / Infinity Cache, not T copies in HBM)."""
    T, h = int(look_back), int(horizon)
    if rows.dim() != 2 or not rows.is_contiguous():
        raise ValueError("rows must be a contiguous [N, F] tensor")
    n = rows.size(0) - T - h + 1
    if n <= 0:
        raise ValueError("fewer rows than look_back + horizon")
    F = rows.size(1)
    X = rows.as_strided((n, T, F), (F, F, 1), rows.storage_offset())
    Y = rows[T + h - 1:T + h - 1 + n]
    return X, Y


# ---------------------------------------------------------------------------
# sources
# ---------------------------------------------------------------------------
def from_arrays(x: np.ndarray, label: Optional[np.ndarray] = None, chunk: int = 65536) -> Stream:
    x = np.asarray(x, dtype=np.float32)
    lab = np.zeros(len(x), np.uint8) if label is None else np.asarray(label, dtype=np.uint8)

    def gen():
        for s in range(0, len(x), chunk):
            yield Chunk(x[s:s + chunk], lab[s:s + chunk])
    return Stream(gen)


def synthetic(n_rows: int, chunk: int = 65536, seed: int = 0, scenario: str = "full",
              failure_rate: float = 0.01, start: int = 0) -> Stream:
    """Synthetic car fleet (scenario.xml: 100 000 devices) -> raw rows + labels."""
    src = SyntheticCarSource.scenario(scenario, seed=seed, failure_rate=failure_rate)

    def gen():
        for s in range(start, start + n_rows, chunk):
            k = min(chunk, start + n_rows - s)
            raw, fail, dev, ts = src.generate(k, start=s)
            yield Chunk(raw, np.where(fail, LABEL_TRUE, LABEL_FALSE).astype(np.uint8),
                        [f"electric-vehicle-{d:05d}" for d in dev] if k <= 4096 else None,
                        meta={"timestamp": ts, "device": dev})
    return Stream(gen)


def csv(path: str, chunk: int = 65536) -> Stream:
    """``testdata/car-sensor-data.csv``; no failure column -> every row is "false"."""
    def gen():
        x, t, cars = load_csv(path)
        for s in range(0, len(x), chunk):
            yield Chunk(x[s:s + chunk], np.zeros(min(chunk, len(x) - s), np.uint8), list(cars[s:s + chunk]),
                        meta={"timestamp": t[s:s + chunk]})
    return Stream(gen)


def json_lines(path: str, chunk: int = 65536) -> Stream:
    """JSON-lines car records (LSTM-.../cardata-v1.json: snake_case + camelCase keys)."""
    def gen():
        rows, labels = [], []
        with open(path) as f:
            for line in f:
                line = line.strip()
                if not line:
                    continue
                rec = json.loads(line)
                vals = {}
                for k, v in rec.items():
                    c = canonical(k)
                    if c is not None and c not in vals:
                        vals[c] = v
                rows.append([float(vals.get(n, 0.0) or 0.0) for n in FEATURES])
                labels.append(vals.get(LABEL, "false") if LABEL in vals else "false")
                if len(rows) == chunk:
                    yield Chunk(np.asarray(rows, np.float32), label_codes(labels))
                    rows, labels = [], []
        if rows:
            yield Chunk(np.asarray(rows, np.float32), label_codes(labels))
    return Stream(gen)


def kafka(servers: str, topics: Sequence[str], schema="cardata-v1", group: Optional[str] = None,
          eof: bool = True, config: Optional[Sequence[str]] = None, max_bytes: int = 4 << 20,
          framing: bool = True, commit: bool = False, resume: bool = False,
          idle_timeout_s: Optional[float] = None, workers: int = 1, native: bool = False,
          shard=None, assign: str = "auto", plan=None, ordered: bool = False) -> Stream:
    """Kafka topic(s) of (Confluent-framed) Avro car records -> raw feature chunks.

    ``topics``: ``"topic:partition:offset"`` specs; ``"topic:*:offset"`` is every partition.

    ``native=True``: the partition-parallel C++ feed (:mod:`streamml.kafka.feed`) decodes
    records straight into page-locked slabs; the Stream still iterates host chunks, and a
    GPU ``fit`` picks up ``stream.native_feed`` to stream slabs to the device with no
    Python-side row handling (``filter_normal(device=True)`` becomes a decode-time filter).

    ``shard``: read only this rank's share of the listed partitions (:mod:`streamml.kafka.assign`)
    -- ``"auto"`` (the ``torch.distributed`` rank / world, a no-op without a process group) or
    ``(rank, world)``.  ``assign``: ``"split"`` (equal contiguous offset ranges; bounded reads),
    ``"partitions"`` (whole partitions, ``p % world``), ``"keys"`` (key-hash shares, per-key
    order; Python reader only), ``"auto"``: split when ``eof`` else partitions.  Under a process
    group every rank resolves the same log snapshot (an all-reduce of the offsets), so starting
    an iteration of a sharded stream is collective -- as every ``fit`` epoch is.  The stream
    carries ``stream.shard = (rank, world)``; ``fit`` then trains each rank on its own rows.

    ``plan``: a ready share plan (e.g. :class:`streamml.kafka.assign.SegmentPlan`) instead of one
    built from ``shard`` / ``assign``.  ``ordered`` (Python reader, ``workers`` > 1): batches in the
    sequential reader's cursor order rather than completion order -- a deterministic row order."""
    from ..kafka import KafkaDataset
    from ..kafka.client import parse_topic_spec
    from .avro import AvroCodec

    # ``plan``: a ready share plan (e.g. kafka.assign.SegmentPlan: continuous training in bounded
    # segments from checkpointed positions) instead of one built from ``shard`` / ``assign``
    if plan is not None:
        pass
    elif shard is not None:
        from ..kafka.assign import ShardPlan, torch_sync
        if shard == "auto":
            import torch.distributed as dist
            pg = dist.is_available() and dist.is_initialized()
            rank, world = (dist.get_rank(), dist.get_world_size()) if pg else (0, 1)
            sync = torch_sync if pg else None
        else:
            rank, world = (int(v) for v in shard)
            sync = None
        mode = ("split" if eof else "partitions") if assign == "auto" else assign
        if mode == "split" and (commit or resume):
            raise ValueError("assign='split' cuts partitions between ranks: per-partition offset commits do not "
                             "apply (checkpoint the position instead, or use assign='partitions')")
        plan = ShardPlan([parse_topic_spec(t) for t in topics], rank, world, mode, sync)
    codec = AvroCodec(schema)
    cols = []
    for name in FEATURES:
        match = [i for i, f in enumerate(codec.numeric_fields) if canonical(f) == name]
        if not match:
            raise ValueError(f"schema has no field for feature {name}")
        cols.append(match[0])
    label_field = next((f for f in codec.text_fields if canonical(f) == LABEL), None)

    if native:
        from ..kafka.feed import NativeFeed
        names = [f.name for f in codec.fields]
        feature_idx = [names.index(codec.numeric_fields[c]) for c in cols]
        label_idx = names.index(label_field) if label_field is not None else -1
        spec = NativeFeed(servers, topics, codec, feature_idx, label_idx, config=config, workers=workers,
                          max_bytes=max_bytes, eof=eof, framing=framing, group=group, resume=resume,
                          commit=commit, idle_timeout_s=idle_timeout_s, plan=plan)

        def native_gen():
            for rows, labs in spec.host_chunks():
                yield Chunk(rows, labs)
        out = Stream(native_gen)
        out.native_feed = spec
        out.shard = None if plan is None else (plan.rank, plan.world)
        out.plan = plan
        return out

    def gen():
        # label codes and str keys come straight from C++ (no per-record Python objects
        # for the text column, no second pass over the keys)
        from ..kafka.assign import key_mask
        ds = KafkaDataset(topics, servers=servers, group=group, eof=eof, config_global=config, codec=codec,
                          max_bytes=max_bytes, framing=framing, commit=commit, resume=resume,
                          idle_timeout_s=idle_timeout_s, with_text=False, str_keys=True, workers=workers,
                          plan=plan, ordered=ordered)
        for b in ds:
            ok = b["ok"].astype(bool)
            x = b["numeric"][:, cols]
            if label_field is not None:
                lab = np.array(b["text_codes"][label_field], dtype=np.uint8, copy=True)
            else:
                lab = np.zeros(len(x), np.uint8)
            lab[~ok] = LABEL_MISSING
            keys = b["keys"]
            c = Chunk(np.ascontiguousarray(x), lab, keys, b["offsets"],
                      meta={"topic": b["topic"], "partition": b["partition"], "errors": int(b["n_errors"]),
                            "ok": ok})
            hr = b.get("hash_range")
            if hr is not None:   # keys share: the cars of this partition another replica owns are skipped
                m = key_mask(keys, hr[0], hr[1])
                if not m.all():
                    c = c.select(m)
                    c.meta["ok"] = ok[m]
                if len(c) == 0:
                    continue
            yield c
    out = Stream(gen)
    out.shard = None if plan is None else (plan.rank, plan.world)
    out.plan = plan
    return out
