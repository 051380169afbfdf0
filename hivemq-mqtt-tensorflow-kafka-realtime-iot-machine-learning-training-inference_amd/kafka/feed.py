"""Native partition-parallel Kafka feed (``csrc/io/feed.cpp``): records -> pinned slabs.

The reference's input path is ``KafkaDataset -> substr(e, 5) -> decode_avro ->
normalize_fn -> filter(y == "false") -> batch(B)``, one tf.string at a time
(AUTOENCODER-TensorFlow-IO-Kafka/cardata-v3.py:44-75, 200-218).  ``NativeFeed`` runs the
fetch + Confluent-unframe + Avro decode + feature projection + label filter in
``workers`` C++ threads (one broker connection each, disjoint partitions) that write
float32 rows and label codes directly into page-locked ring slots (``PinnedRing``,
``hipHostMalloc``).  Python only moves slot numbers: each filled slot is submitted to the
copy engine immediately (several H2D copies in flight), waited for on the consumer's
stream, and handed back to the workers once its copy has landed.  No per-record Python
objects, no numpy hop, no host memcpy between decode and DMA.
"""
from __future__ import annotations

import collections
import time
from typing import Iterator, List, Optional, Sequence, Tuple

import numpy as np

from ..ops._ext import load_io
from .client import KafkaClient, KafkaError, offset_reset_policy, parse_config, parse_topic_spec


def _auth(config) -> Tuple[str, str, str, str, int]:
    cfg = parse_config(config)
    proto = cfg.get("security.protocol", "plaintext").lower()
    mech = ""
    if proto in ("sasl_plaintext", "sasl_ssl"):
        if proto == "sasl_ssl":
            raise KafkaError("TLS is not supported by the native client")
        mech = cfg.get("sasl.mechanisms", cfg.get("sasl.mechanism", "PLAIN")).upper()
    return (cfg.get("client.id", "streamml"), mech, cfg.get("sasl.username", ""), cfg.get("sasl.password", ""),
            int(cfg.get("socket.timeout.ms", 30000)))


class NativeFeed:
    """A re-iterable feed specification: every ``host_chunks`` / ``device_chunks`` call
    resolves the partition range (``eof=True``: up to the end offsets at that moment, as
    tfio's ``eof`` -- each Keras epoch re-reads the bounded stream, python-scripts/README.md:116)
    and runs a fresh set of worker threads."""

    def __init__(self, servers: str, topics: Sequence[str], codec, feature_fields: Sequence[int],
                 label_field: int = -1, config: Optional[Sequence[str]] = None, workers: int = 1,
                 max_bytes: int = 4 << 20, max_wait_ms: int = 100, eof: bool = True, framing: bool = True,
                 group: Optional[str] = None, resume: bool = False, commit: bool = False,
                 idle_timeout_s: Optional[float] = None, plan=None):
        self.servers = servers
        self.plan = plan              # kafka.assign.ShardPlan: this rank's share, resolved per iteration
        self.specs = [parse_topic_spec(t) for t in topics]
        self.codec = codec
        self.feature_fields = [int(f) for f in feature_fields]
        self.label_field = int(label_field)
        self.config = list(config or [])
        self.workers = max(1, int(workers))
        self.max_bytes = int(max_bytes)
        self.max_wait_ms = int(max_wait_ms)
        self.eof = eof
        self.framing = framing
        self.group = group
        self.resume = resume and group is not None
        self.commit = commit and group is not None
        self.idle_timeout_s = idle_timeout_s
        # librdkafka's check.crcs (default false): verify every record batch's CRC-32C
        self.check_crcs = str(parse_config(self.config).get("check.crcs", "false")).lower() in ("true", "1")
        self.last_stats: dict = {}
        self.staged = None            # stage(): pre-fetched record values instead of the broker

    def stage(self, buf, offsets) -> "NativeFeed":
        """Serve every later iteration from ``len(offsets) - 1`` pre-staged record values (value i =
        ``buf[offsets[i]:offsets[i+1]]``, as fetched responses hold them) instead of fetching: the
        workers decode contiguous shares of them straight into the pinned ring, so the decode +
        H2D + train path runs without the broker's socket threads sharing the CPUs (a bench mode
        that measures the consumer side; no partitions, no commits)."""
        arr = buf if isinstance(buf, np.ndarray) else np.frombuffer(buf, np.uint8)
        self.staged = (np.ascontiguousarray(arr), np.ascontiguousarray(offsets, dtype=np.int64))
        return self

    @property
    def features(self) -> int:
        return len(self.feature_fields)

    def _start(self, client: KafkaClient, topic: str, partition: int, offset: int) -> int:
        start = -1
        if self.resume:
            start = client.committed(self.group, topic, partition)
        if start < 0:
            if offset == -1:
                start = client.latest(topic, partition)
            elif offset == -2:
                start = client.earliest(topic, partition)
            else:
                start = offset
        first = client.earliest(topic, partition)
        if start < first:   # deleted by retention (or a stale commit): auto.offset.reset
            policy = offset_reset_policy(self.config)
            if policy == "none":
                raise KafkaError(f"{topic}:{partition}: offset {start} below the log start {first} "
                                 f"(auto.offset.reset=none)")
            start = first if policy == "earliest" else client.latest(topic, partition)
        return int(start)

    def _parts(self, client: KafkaClient) -> List[Tuple[str, int, int, int]]:
        if self.plan is not None:   # this rank's share of the partitions (kafka/assign.py)
            shares = self.plan.resolve(client, lambda t, p, o: self._start(client, t, p, o), self.eof)
            if any(not s.whole_keys for s in shares):
                raise KafkaError("the native feed reads whole partitions or offset ranges; assign='keys' "
                                 "needs the Python reader (native=False) or the serving loop")
            return [s.as_part() for s in shares]
        from .assign import expand_specs
        specs = expand_specs(self.specs, client.partitions() if any(p == -1 for _, p, _ in self.specs) else {})
        parts = []
        for topic, partition, offset in specs:
            start = self._start(client, topic, partition, offset)
            end = client.latest(topic, partition) if self.eof else -1
            parts.append((topic, partition, start, int(end)))
        return parts

    def _make(self, keep_label: Optional[int]):
        staged = self.staged is not None
        client = None if staged else KafkaClient(self.servers, self.config)
        parts = [] if staged else self._parts(client)
        cid, mech, user, pw, tmo = _auth(self.config)
        f = load_io().KafkaFeed("127.0.0.1:9" if staged else client.servers, cid, mech, user, pw, tmo,
                                [fs.as_tuple() for fs in self.codec.fields], self.feature_fields,
                                self.label_field, -1 if keep_label is None else int(keep_label), self.framing,
                                self.max_bytes, self.max_wait_ms, self.workers,
                                -1.0 if self.idle_timeout_s is None else float(self.idle_timeout_s), parts,
                                check_crcs=self.check_crcs,
                                offset_reset={"earliest": 0, "latest": 1, "none": 2}[offset_reset_policy(self.config)])
        return f, client, parts

    def decode_only(self, buf, offsets, workers: int, repeats: int = 3, keep_label: Optional[int] = None):
        """The decoder alone: ``len(offsets) - 1`` pre-staged record values (Confluent Avro, value
        i = buf[offsets[i]:offsets[i+1]], as they sit in a fetch response) decoded by ``workers``
        C++ threads into private slabs -- no broker, no socket, no pinned ring.  Returns (best
        rows/s over ``repeats``, rows kept per pass)."""
        cid, mech, user, pw, tmo = _auth(self.config)
        f = load_io().KafkaFeed("127.0.0.1:9", cid, mech, user, pw, tmo, [fs.as_tuple() for fs in self.codec.fields],
                                self.feature_fields, self.label_field, -1 if keep_label is None else int(keep_label),
                                self.framing, self.max_bytes, self.max_wait_ms, 1, -1.0, [], check_crcs=False)
        rate, rows = f.decode_throughput(buf, np.ascontiguousarray(offsets, dtype=np.int64), int(workers), int(repeats))
        return float(rate), int(rows)

    def _begin(self, f, ptrs, slab_rows: int) -> None:
        if self.staged is not None:
            buf, offs = self.staged
            f.start_staged(ptrs, int(slab_rows), buf, offs, self.workers)
        else:
            f.start(ptrs, int(slab_rows))

    @staticmethod
    def _consumed(f, slab: int, marks: dict) -> None:
        """The consumer asked for the next slab: everything this one carried has been used."""
        for pi, pos in f.slab_marks(int(slab)):
            marks[int(pi)] = max(marks.get(int(pi), -1), int(pos))

    def _finish(self, f, client, parts, t0: float, marks: dict, exhausted: bool) -> None:
        """Commit (``commit=True``) at-least-once positions: the decode positions of the
        workers when the stream was drained to its end (``exhausted``), otherwise -- early
        stop, ``take``, an exception in the consumer -- only the publish-time marks of the
        slabs the consumer came back from (rows decoded ahead into queued or in-flight
        slabs are re-read by a resumed run, never skipped)."""
        st = dict(f.stats())
        st["wall_s"] = time.perf_counter() - t0
        st["workers"] = self.workers if self.staged is not None else min(self.workers, max(len(parts), 1))
        if self.staged is not None:
            st["source"] = "staged"
        st["committed"] = "end" if exhausted else "consumed-slabs"
        self.last_stats = st
        if not self.commit:
            return
        final = f.positions() if exhausted else None
        for pi, (topic, partition, start, _) in enumerate(parts):
            pos = int(final[pi]) if final is not None else marks.get(pi, -1)
            if pos > start or (final is not None and pos >= start):
                client.commit(self.group, topic, partition, pos)

    # ------------------------------------------------------------------ host
    def host_chunks(self, keep_label: Optional[int] = None, slab_rows: int = 65536,
                    slots: Optional[int] = None):
        """(rows [n, F] float32 copy, labels [n] uint8 copy) per filled slab (CPU consumers)."""
        f, client, parts = self._make(keep_label)
        F = self.features
        nslots = int(slots or 2 * self.workers + 2)
        bufs = [np.empty(slab_rows * (F * 4 + 1), np.uint8) for _ in range(nslots)]
        t0 = time.perf_counter()
        self._begin(f, [int(b.ctypes.data) for b in bufs], slab_rows)
        marks: dict = {}
        exhausted = False
        try:
            while True:
                code, slab, n = f.pop(1000)
                if code < 0:
                    exhausted = True
                    break
                if code == 0:
                    continue
                b = bufs[slab]
                rows = b[:n * F * 4].view(np.float32).reshape(n, F).copy()
                labs = b[n * F * 4:n * F * 4 + n].copy()
                mk = f.slab_marks(slab)
                f.recycle(slab)
                yield rows, labs
                for pi, pos in mk:
                    marks[int(pi)] = max(marks.get(int(pi), -1), int(pos))
        finally:
            f.stop()
            self._finish(f, client, parts, t0, marks, exhausted)

    def count_rows(self, keep_label: Optional[int] = None, slab_rows: int = 65536) -> int:
        """Fetch + decode the whole range and count the rows; slabs are recycled as they are
        published, never copied (the host decode rate alone, for scaling measurements)."""
        f, client, parts = self._make(keep_label)
        F = self.features
        nslots = 2 * self.workers + 2
        bufs = [np.empty(slab_rows * (F * 4 + 1), np.uint8) for _ in range(nslots)]
        t0 = time.perf_counter()
        self._begin(f, [int(b.ctypes.data) for b in bufs], slab_rows)
        total, exhausted = 0, False
        try:
            while True:
                code, slab, n = f.pop(1000)
                if code < 0:
                    exhausted = True
                    break
                if code:
                    total += int(n)
                    f.recycle(slab)
        finally:
            f.stop()
            self._finish(f, client, parts, t0, {}, exhausted)
        return total

    # ------------------------------------------------------------------ device
    def device_chunks(self, device, keep_label: Optional[int] = None, slab_rows: int = 32768,
                      slots: Optional[int] = None, inflight: Optional[int] = None) -> Iterator:
        """Device tensors [n, F] float32 of raw rows, one per filled slab, in publish order.

        ``keep_label`` filters at decode time (the host knows each record's label before
        the row is written, so dropped rows never reach the ring).  Up to ``inflight``
        slabs are submitted to the copy engine ahead of the one being consumed."""
        import torch

        from ..data.loader import pinned_ring
        dev = torch.device(device)
        if dev.index is None:
            dev = torch.device("cuda", torch.cuda.current_device())
        F = self.features
        nslots = int(slots or 2 * self.workers + 6)
        depth = int(inflight or max(2, nslots - self.workers - 1))
        slab_bytes = slab_rows * (F * 4 + 1)
        with pinned_ring(nslots, slab_bytes, dev.index) as ring:   # pooled: never freed mid-stream
            yield from self._device_chunks_on(ring, dev, keep_label, slab_rows, nslots, depth, slab_bytes)

    def _device_chunks_on(self, ring, dev, keep_label, slab_rows, nslots, depth, slab_bytes):
        import torch
        F = self.features
        bufs = [torch.empty(slab_bytes, dtype=torch.uint8, device=dev) for _ in range(nslots)]
        f, client, parts = self._make(keep_label)
        t0 = time.perf_counter()
        self._begin(f, [int(ring.host_ptr(i)) for i in range(nslots)], slab_rows)
        pending: collections.deque = collections.deque()
        done = False
        exhausted = False
        marks: dict = {}
        h2d_bytes = 0
        try:
            while pending or not done:
                while not done and len(pending) < depth:
                    code, slab, n = f.pop(0 if pending else 1000)
                    if code < 0:
                        done = True
                        break
                    if code == 0:
                        if pending:
                            break
                        continue
                    nb = n * F * 4
                    ring.submit(slab, bufs[slab], nb)    # copy engine starts on it now
                    h2d_bytes += nb
                    pending.append((slab, n))
                if not pending:
                    continue
                slab, n = pending.popleft()
                ring.wait(slab)
                yield bufs[slab][:n * F * 4].view(torch.float32).view(n, F)
                self._consumed(f, slab, marks)
                ring.release(slab)          # the consumer's kernels for this slab are enqueued
                ring.host_ptr(slab)         # its H2D copy has landed: the host slab is free
                f.recycle(slab)
            exhausted = True
        finally:
            f.stop()
            while pending:                  # drain copies that were submitted but not consumed
                slab, _ = pending.popleft()
                ring.wait(slab)
                ring.release(slab)
            self._finish(f, client, parts, t0, marks, exhausted)
            self.last_stats["h2d_bytes"] = h2d_bytes
