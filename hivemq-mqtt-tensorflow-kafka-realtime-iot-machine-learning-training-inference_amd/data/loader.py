"""Host -> device streaming loader over the native pinned ring (``streamml._C.PinnedRing``).

Pipeline per micro-batch (all three stages overlap):

1. a background thread pulls :class:`~streamml.data.stream.Chunk` s from the
   stream (Kafka fetch + Avro decode run in C++ with the GIL released);
2. the chunk's raw feature rows are memcpy'd into a page-locked ring slot and
   ``hipMemcpyAsync``'d to that slot's device buffer on the ring's copy stream;
3. the consumer's current stream waits on the slot's copy event; when the
   consumer asks for the next batch, a release event is recorded so the slot's
   device buffer is not overwritten while kernels still read it.
"""
from __future__ import annotations

import queue
import threading
from typing import Iterator, Optional, Tuple

import numpy as np
import torch

from ..obs.metrics import ENGINE
from ..ops._ext import load_c
from .stream import Chunk, Stream

_END = object()


class DeviceLoader:
    """``keep_label``: filter on the device instead of the host -- raw rows AND their
    label codes go through the ring, K8 ``normalize_filter`` compacts the rows whose
    label is ``keep_label`` in order, and a device re-batcher emits exactly
    ``batch_rows`` rows per batch (the reference's ``filter(...)`` then ``batch(B)``,
    cardata-v3.py:212-218).  Yields ``(rows, None)`` in that mode."""

    def __init__(self, stream: Stream, device, max_rows: int, slots: int = 3, prefetch: int = 4,
                 features: int = 18, keep_label: Optional[int] = None, batch_rows: Optional[int] = None):
        self.stream = stream
        self.device = torch.device(device)
        if self.device.type != "cuda":
            raise RuntimeError("DeviceLoader needs a ROCm device")
        if self.device.index is None:
            self.device = torch.device("cuda", torch.cuda.current_device())
        self.max_rows = int(max_rows)
        self.features = int(features)
        self.slots = int(slots)
        self.prefetch = int(prefetch)
        C = load_c()
        self.ring = C.PinnedRing(self.slots, self.max_rows * self.features * 4, self.device.index)
        self.bufs = [torch.empty((self.max_rows, self.features), dtype=torch.float32, device=self.device)
                     for _ in range(self.slots)]
        self.rows = 0
        self.keep_label = keep_label
        self.batch_rows = int(batch_rows or max_rows)
        if keep_label is not None:
            self.lab_host = [torch.empty(self.max_rows, dtype=torch.uint8).pin_memory() for _ in range(self.slots)]
            self.lab_dev = [torch.empty(self.max_rows, dtype=torch.uint8, device=self.device)
                            for _ in range(self.slots)]

    def _producer(self, q: "queue.Queue", stop: threading.Event) -> None:
        try:
            for c in self.stream:
                if stop.is_set():
                    return
                for s in range(0, len(c), self.max_rows):
                    part = c if len(c) <= self.max_rows else c.select(slice(s, s + self.max_rows))
                    q.put(part)
                    if len(c) <= self.max_rows:
                        break
        except BaseException as e:  # surfaced in the consumer
            q.put(e)
        finally:
            q.put(_END)

    def __iter__(self):
        if self.keep_label is None:
            return self._iter_rows()
        return self._iter_filtered()

    def _iter_filtered(self) -> Iterator[Tuple[torch.Tensor, None]]:
        """Device filter + exact re-batching (staging buffer of up to 2 batches)."""
        from ..ops.preprocess import normalize_filter
        B = self.batch_rows
        stage = torch.empty((B + self.max_rows, self.features), dtype=torch.float32, device=self.device)
        have = 0
        for xb, c in self._iter_rows(with_labels=True):
            slot = self._last_slot
            kept, _ = normalize_filter(xb, self.lab_dev[slot][:len(xb)], int(self.keep_label))
            k = kept.size(0)
            if k:
                stage[have:have + k].copy_(kept)
                have += k
            while have >= B:
                out = stage[:B].clone()
                rest = have - B
                if rest:
                    stage[:rest].copy_(stage[B:have].clone())
                have = rest
                yield out, None
        if have:
            yield stage[:have].clone(), None

    def _iter_rows(self, with_labels: bool = False) -> Iterator[Tuple[torch.Tensor, Chunk]]:
        q: "queue.Queue" = queue.Queue(maxsize=self.prefetch)
        stop = threading.Event()
        th = threading.Thread(target=self._producer, args=(q, stop), daemon=True)
        th.start()
        i = 0
        prev: Optional[int] = None
        try:
            while True:
                item = q.get()
                if item is _END:
                    break
                if isinstance(item, BaseException):
                    raise item
                c: Chunk = item
                slot = i % self.slots
                n = len(c)
                x = np.ascontiguousarray(c.x, dtype=np.float32)
                self.ring.fill(slot, x)
                if prev is not None:
                    # consumer kernels for `prev` are enqueued by now; releasing before the
                    # next submit also orders a reused slot's copy after them (slots=1)
                    self.ring.release(prev)
                self.ring.submit(slot, self.bufs[slot], n * self.features * 4)
                if with_labels:
                    self.lab_host[slot][:n].copy_(torch.from_numpy(np.ascontiguousarray(c.label, np.uint8)))
                    self.lab_dev[slot][:n].copy_(self.lab_host[slot][:n], non_blocking=True)
                    self._last_slot = slot
                self.ring.wait(slot)
                self.rows += n
                ENGINE.h2d_bytes.inc(n * self.features * 4)
                ENGINE.ring_occupancy.set(q.qsize())
                yield self.bufs[slot][:n], c
                prev = slot
                i += 1
        finally:
            if prev is not None:   # also when the consumer stops early (take / break)
                self.ring.release(prev)
            stop.set()
            while th.is_alive():
                try:
                    q.get_nowait()
                except queue.Empty:
                    th.join(timeout=0.05)
