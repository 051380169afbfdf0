"""Host -> device streaming loader over the native pinned ring (``streamml._C.PinnedRing``).

Pipeline (all stages overlap; up to ``slots - 1`` H2D copies in flight):

1. a producer thread pulls :class:`~streamml.data.stream.Chunk` s from the stream
   (Kafka fetch + Avro decode run in C++ with the GIL released) -- or, for a
   native Kafka source, the C++ ingest feed (:mod:`streamml.kafka.feed`) whose
   worker threads decode records straight into the page-locked slots;
2. each chunk's raw rows (and, when the consumer filters on the device, its label
   codes right behind them) land in a page-locked ring slot, and the producer
   submits the slot's ``hipMemcpyAsync`` on the ring's copy stream immediately --
   it does not wait for the consumer to ask for the batch;
3. the consumer's stream waits on the slot's copy event; after the consumer's
   kernels for a slot are enqueued, a release event is recorded and the slot goes
   back to the producer (a free-slot semaphore orders that release before the
   slot's next submit, so the copy stream never waits on an unrecorded event).

``chunks()`` yields whole device chunks (the persistent-kernel ``fit`` path consumes
many Keras batches per launch); iterating the loader yields ``(rows, chunk)`` per
ring slot, or exact ``batch_rows``-row batches in device-filter mode.

Pinned rings come from a process-wide pool (:func:`pinned_ring`): allocating page-locked
memory is slow, and FREEING it (hipHostFree) synchronises the whole device -- which would
stall for as long as a persistent kernel that waits for this very stream's rows (the
one-launch streaming epoch, ``FusedAE.train_stream``) is running.
"""
from __future__ import annotations

import contextlib
import queue
import threading
import time
from typing import Iterator, Optional, Tuple

import numpy as np
import torch

from ..obs.metrics import ENGINE
from ..ops._ext import load_c
from .stream import Chunk, Stream

_END = object()

_RING_POOL: dict = {}
_POOL_LOCK = threading.Lock()


@contextlib.contextmanager
def pinned_ring(slots: int, slot_bytes: int, device_index: int):
    """A ``PinnedRing`` of this exact shape from the process-wide pool (allocated on first
    use), reset to all-idle and returned to the pool on exit -- never freed while the
    process runs (see the module docstring)."""
    key = (int(slots), int(slot_bytes), int(device_index))
    with _POOL_LOCK:
        free = _RING_POOL.setdefault(key, [])
        ring = free.pop() if free else None
    if ring is None:
        ring = load_c().PinnedRing(*key)
    try:
        yield ring
    finally:
        ring.reset()   # copies submitted but never consumed land before the next owner
        with _POOL_LOCK:
            _RING_POOL[key].append(ring)


class DeviceLoader:
    """``keep_label``: filter on the device instead of the host -- raw rows AND their
    label codes go through the ring, K8 ``normalize_filter`` compacts the rows whose
    label is ``keep_label`` in order (the kept count comes from the host-side labels,
    so no device->host sync), and in batch mode a device re-batcher emits exactly
    ``batch_rows`` rows per batch (the reference's ``filter(...)`` then ``batch(B)``,
    cardata-v3.py:212-218)."""

    def __init__(self, stream: Stream, device, max_rows: int, slots: int = 4, prefetch: int = 4,
                 features: int = 18, keep_label: Optional[int] = None, batch_rows: Optional[int] = None):
        self.stream = stream
        self.device = torch.device(device)
        if self.device.type != "cuda":
            raise RuntimeError("DeviceLoader needs a ROCm device")
        if self.device.index is None:
            self.device = torch.device("cuda", torch.cuda.current_device())
        self.max_rows = int(max_rows)
        self.features = int(features)
        self.slots = max(2, int(slots))
        self.prefetch = int(prefetch)
        self.row_bytes = self.features * 4
        # slot layout: n rows [n, F] float32, then n label bytes right behind them
        self.slot_bytes = self.max_rows * (self.row_bytes + 1)
        self.ring = None   # a pooled PinnedRing while iterating (pinned_ring)
        self.bufs = [torch.empty(self.slot_bytes, dtype=torch.uint8, device=self.device) for _ in range(self.slots)]
        self.rows = 0
        self.keep_label = keep_label
        self.batch_rows = int(batch_rows or max_rows)
        self.stats = {"h2d_bytes": 0, "chunks": 0, "producer_wait_s": 0.0, "consumer_wait_s": 0.0}

    # ------------------------------------------------------------------ views
    def _views(self, slot: int, n: int) -> Tuple[torch.Tensor, torch.Tensor]:
        rb = n * self.row_bytes
        buf = self.bufs[slot]
        return buf[:rb].view(torch.float32).view(n, self.features), buf[rb:rb + n]

    # ------------------------------------------------------------------ producer
    def _producer(self, q: "queue.Queue", stop: threading.Event, free: threading.Semaphore) -> None:
        with_labels = self.keep_label is not None
        i = 0
        try:
            for c in self.stream:
                for s in range(0, max(len(c), 1), self.max_rows):
                    if stop.is_set():
                        return
                    part = c if len(c) <= self.max_rows else c.select(slice(s, s + self.max_rows))
                    n = len(part)
                    if n == 0:
                        break
                    t0 = time.perf_counter()
                    while not free.acquire(timeout=0.1):
                        if stop.is_set():
                            return
                    self.stats["producer_wait_s"] += time.perf_counter() - t0
                    slot = i % self.slots
                    x = np.ascontiguousarray(part.x, dtype=np.float32)
                    self.ring.fill(slot, x, 0)
                    nbytes = n * self.row_bytes
                    if with_labels:
                        self.ring.fill(slot, np.ascontiguousarray(part.label, np.uint8), nbytes)
                        nbytes += n
                    self.ring.submit(slot, self.bufs[slot], nbytes)   # H2D starts now
                    self.stats["h2d_bytes"] += nbytes
                    q.put((slot, n, part))
                    i += 1
                    if len(c) <= self.max_rows:
                        break
        except BaseException as e:  # surfaced in the consumer
            q.put(e)
        finally:
            q.put(_END)

    def _slots(self) -> Iterator[Tuple[int, int, Chunk]]:
        """Ring slots in order, copy waited for on the consumer's stream; the slot is
        released (and handed back to the producer) when the consumer asks for the next."""
        with pinned_ring(self.slots, self.slot_bytes, self.device.index) as ring:
            self.ring = ring
            try:
                yield from self._slots_on_ring()
            finally:
                self.ring = None

    def _slots_on_ring(self) -> Iterator[Tuple[int, int, Chunk]]:
        q: "queue.Queue" = queue.Queue()
        stop = threading.Event()
        free = threading.Semaphore(self.slots)
        th = threading.Thread(target=self._producer, args=(q, stop, free), daemon=True)
        th.start()
        prev: Optional[int] = None
        try:
            while True:
                t0 = time.perf_counter()
                item = q.get()
                self.stats["consumer_wait_s"] += time.perf_counter() - t0
                if item is _END:
                    break
                if isinstance(item, BaseException):
                    raise item
                slot, n, c = item
                self.ring.wait(slot)
                self.rows += n
                self.stats["chunks"] += 1
                ENGINE.h2d_bytes.inc(n * self.row_bytes)
                ENGINE.ring_occupancy.set(q.qsize())
                prev = slot
                yield slot, n, c
                # the consumer asked for more: its kernels for `prev` are enqueued
                self.ring.release(prev)
                free.release()
                prev = None
        finally:
            if prev is not None:   # also when the consumer stops early (take / break)
                self.ring.release(prev)
                free.release()
            stop.set()
            th.join(timeout=10)

    # ------------------------------------------------------------------ consumers
    def __iter__(self):
        if self.keep_label is None:
            return self._iter_rows()
        return self._iter_filtered()

    def _iter_rows(self) -> Iterator[Tuple[torch.Tensor, Chunk]]:
        for slot, n, c in self._slots():
            yield self._views(slot, n)[0], c

    def _filtered_chunk(self, slot: int, n: int, c: Chunk) -> torch.Tensor:
        """K8 on one slot: the kept rows, raw (the train kernels normalise on load)."""
        rows, lab = self._views(slot, n)
        m = int(np.count_nonzero(np.asarray(c.label) == int(self.keep_label)))   # host labels: no sync
        if m == 0:
            return rows[:0]
        out, _, _ = load_c().normalize_filter(rows, self.features, lab, int(self.keep_label), None, None, False)
        return out[:m]

    def chunks(self) -> Iterator[torch.Tensor]:
        """Whole device chunks of raw rows (filtered on the device when ``keep_label`` is set)."""
        for slot, n, c in self._slots():
            if self.keep_label is None:
                yield self._views(slot, n)[0]
            else:
                kept = self._filtered_chunk(slot, n, c)
                if kept.size(0):
                    yield kept

    def _iter_filtered(self) -> Iterator[Tuple[torch.Tensor, None]]:
        """Device filter + exact re-batching.  Two staging buffers alternate, so carrying
        the remainder never copies a buffer onto itself and no batch is cloned (every
        op is ordered on the consumer's stream; a yielded batch stays valid until the
        consumer asks for the batch after the next one)."""
        B = self.batch_rows
        cap = B + self.max_rows
        stages = [torch.empty((cap, self.features), dtype=torch.float32, device=self.device) for _ in range(2)]
        cur, have = 0, 0
        for slot, n, c in self._slots():
            kept = self._filtered_chunk(slot, n, c)
            k = kept.size(0)
            if k:
                stages[cur][have:have + k].copy_(kept)
                have += k
            off = 0
            while have - off >= B:
                yield stages[cur][off:off + B], None
                off += B
            if off:
                rest = have - off
                if rest:
                    stages[cur ^ 1][:rest].copy_(stages[cur][off:have])
                cur ^= 1
                have = rest
        if have:
            yield stages[cur][:have], None
