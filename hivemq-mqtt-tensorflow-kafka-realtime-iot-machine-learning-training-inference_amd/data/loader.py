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
    def __init__(self, stream: Stream, device, max_rows: int, slots: int = 3, prefetch: int = 4,
                 features: int = 18):
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

    def __iter__(self) -> Iterator[Tuple[torch.Tensor, Chunk]]:
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
                self.ring.submit(slot, self.bufs[slot], n * self.features * 4)
                if prev is not None:
                    self.ring.release(prev)   # consumer kernels for `prev` are enqueued by now
                self.ring.wait(slot)
                self.rows += n
                ENGINE.h2d_bytes.inc(n * self.features * 4)
                ENGINE.ring_occupancy.set(q.qsize())
                yield self.bufs[slot][:n], c
                prev = slot
                i += 1
            if prev is not None:
                self.ring.release(prev)
        finally:
            stop.set()
            while th.is_alive():
                try:
                    q.get_nowait()
                except queue.Empty:
                    th.join(timeout=0.05)
