"""``KafkaOutputSequence``: indexed result sink (reference cardata-v3.py:238-252).

The reference's ``OutputCallback.on_predict_batch_end`` calls
``sequence.setitem(index, np.array2string(row))`` per predicted row and
``flush()`` at the end; tfio buffers the items and produces them in index order.
This implementation keeps the same contract: items are buffered, produced in
ascending index order with no gaps (an item waits until every lower index has
arrived), in batched Produce requests.
"""
from __future__ import annotations

from typing import Dict, Optional, Sequence, Union

from .client import KafkaClient


from ..obs.metrics import ENGINE

class KafkaOutputSequence:
    def __init__(self, topic: str, servers: str = "fake://", configuration: Optional[Sequence[str]] = None,
                 partition: int = 0, batch_records: int = 4096, acks: int = 1):
        self.topic = topic
        self.partition = partition
        self.batch_records = int(batch_records)
        self.acks = acks
        self._client = KafkaClient(servers, configuration)
        self._pending: Dict[int, bytes] = {}
        self._keys: Dict[int, Optional[bytes]] = {}
        self._next = 0
        self._ready: list = []
        self._ready_keys: list = []
        self.produced = 0

    def setitem(self, index: int, message: Union[str, bytes], key: Optional[Union[str, bytes]] = None) -> None:
        if index < self._next or index in self._pending:
            raise IndexError(f"index {index} already written")
        self._pending[index] = message.encode() if isinstance(message, str) else bytes(message)
        self._keys[index] = key.encode() if isinstance(key, str) else key
        while self._next in self._pending:
            self._ready.append(self._pending.pop(self._next))
            self._ready_keys.append(self._keys.pop(self._next))
            self._next += 1
        if len(self._ready) >= self.batch_records:
            self._send()

    def extend(self, index: int, messages: Sequence[Union[str, bytes]],
               keys: Optional[Sequence[Optional[Union[str, bytes]]]] = None) -> None:
        """``setitem(index + i, messages[i], keys[i])`` for a contiguous run, in bulk: when the
        run starts at the next index to produce (the serving loop's case) the records go
        straight to the produce batch (list operations, no per-record Python bookkeeping)."""
        n = len(messages)
        if keys is not None and len(keys) != n:
            raise ValueError("keys and messages differ in length")
        if n == 0:
            return
        if index != self._next or self._pending:
            for i in range(n):
                self.setitem(index + i, messages[i], None if keys is None else keys[i])
            return
        self._ready.extend(m.encode() if isinstance(m, str) else m for m in messages)
        if keys is None:
            self._ready_keys.extend([None] * n)
        else:
            self._ready_keys.extend(k.encode() if isinstance(k, str) else k for k in keys)
        self._next += n
        while len(self._ready) >= self.batch_records:   # produce requests of batch_records, as setitem
            rest, rest_keys = self._ready[self.batch_records:], self._ready_keys[self.batch_records:]
            del self._ready[self.batch_records:], self._ready_keys[self.batch_records:]
            self._send()
            self._ready, self._ready_keys = rest, rest_keys

    def _send(self) -> None:
        if not self._ready:
            return
        keys = None if all(k is None for k in self._ready_keys) else self._ready_keys
        self._client.produce(self.topic, self.partition, self._ready, keys, None, self.acks)
        self.produced += len(self._ready)
        ENGINE.produced_records.inc(len(self._ready), topic=self.topic)
        self._ready, self._ready_keys = [], []

    def flush(self) -> None:
        if self._pending:
            raise RuntimeError(f"cannot flush: indices missing before {min(self._pending)}")
        self._send()
