"""Who reads what: a topic's log cut into per-rank (training) / per-replica (serving) shares.

The reference's only scale-out axis is the Kafka partition: ``sensor-data`` and
``model-predictions`` have 10 partitions (infrastructure/confluent/01_installConfluentPlatform.sh:180,
183), KSQL re-keys the Avro stream ``PARTITION BY CAR`` (:249), yet the consumer reads
``topic:0:offset`` only (AUTOENCODER-TensorFlow-IO-Kafka/cardata-v3.py:44-47).  Here every rank
of a data-parallel job, or every serving replica, reads a disjoint share of ALL partitions:

* ``"split"`` (bounded reads, ``eof=True``: training epochs) -- the partitions' offset ranges
  ``[start, end)`` laid end to end and cut into ``world`` contiguous pieces of equal record
  count (to one record).  A partition may be cut between two ranks; each rank fetches only
  its own offsets, so nothing is read twice and every record is read exactly once.
* ``"partitions"`` -- whole partitions, ``p % world == rank`` (Kafka consumer-group
  semantics; unbounded reads, offset commits per partition).  Skewed when ``world`` does not
  divide the partition count (8 ranks over 10 partitions: 2 vs 1).
* ``"keys"`` (serving, unbounded, per-key order) -- the key space balanced over the
  replicas: the partitions are laid on a line ``[0, P)`` and replica ``r`` owns
  ``[r P / W, (r + 1) P / W)``.  Where that cuts a partition, the replicas sharing it split
  its car keys by a 32-bit key hash (FNV-1a + fmix64, independent of the producer's murmur2
  partitioner), so every car is scored by exactly one replica, in order, and each replica
  carries ``P / W`` partitions' worth of keys at any ``W``.

A share is a list of :class:`Share` (topic, partition, start, end, hash range).
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Callable, Dict, List, Optional, Sequence, Tuple

HASH_SPACE = 1 << 32
MODES = ("split", "partitions", "keys")


@dataclass(frozen=True)
class Share:
    topic: str
    partition: int
    start: int
    end: int = -1                 # exclusive; -1 = follow the log (unbounded)
    hash_lo: int = 0              # key-hash interval [hash_lo, hash_hi) of this share (keys mode)
    hash_hi: int = HASH_SPACE

    @property
    def whole_keys(self) -> bool:
        return self.hash_lo == 0 and self.hash_hi == HASH_SPACE

    @property
    def rows(self) -> int:
        return max(self.end - self.start, 0) if self.end >= 0 else -1

    def as_part(self) -> Tuple[str, int, int, int]:
        return (self.topic, self.partition, self.start, self.end)


def key_hash(key) -> int:
    """32-bit share hash of a record key: the top half of fmix64(FNV-1a 64) (``scoreloop.cpp``
    computes the same).  ``None`` keys hash as the empty key."""
    if key is None:
        b = b""
    elif isinstance(key, str):
        b = key.encode()
    else:
        b = bytes(key)
    h = 0xCBF29CE484222325
    for c in b:
        h ^= c
        h = (h * 0x100000001B3) & 0xFFFFFFFFFFFFFFFF
    # FNV-1a alone leaves the top bits nearly constant for keys that differ in their last
    # characters ("electric-vehicle-00017" / "-00018"): MurmurHash3's fmix64 finaliser first
    M = 0xFFFFFFFFFFFFFFFF
    h ^= h >> 33
    h = (h * 0xFF51AFD7ED558CCD) & M
    h ^= h >> 33
    h = (h * 0xC4CEB9FE1A85EC53) & M
    h ^= h >> 33
    return h >> 32


def key_mask(keys, lo: int, hi: int):
    """Boolean mask of the keys whose share hash lies in ``[lo, hi)``."""
    import numpy as np
    if lo == 0 and hi == HASH_SPACE:
        return np.ones(len(keys), dtype=bool)
    h = np.fromiter((key_hash(k) for k in keys), dtype=np.int64, count=len(keys))
    return (h >= lo) & (h < hi)


def split_rows(ranges: Sequence[Tuple[str, int, int, int]], rank: int, world: int) -> List[Share]:
    """``"split"``: the bounded ranges ``(topic, partition, start, end)`` laid end to end (in the
    given order) and cut into ``world`` contiguous pieces whose record counts differ by at
    most one; rank ``rank``'s piece as a list of shares."""
    rank, world = int(rank), int(world)
    if not 0 <= rank < world:
        raise ValueError(f"rank {rank} outside world {world}")
    total = sum(max(e - s, 0) for _, _, s, e in ranges)
    lo, hi = total * rank // world, total * (rank + 1) // world
    out, pos = [], 0
    for topic, p, s, e in ranges:
        n = max(e - s, 0)
        a, b = max(lo, pos), min(hi, pos + n)
        if a < b:
            out.append(Share(topic, int(p), int(s + a - pos), int(s + b - pos)))
        pos += n
    return out


def round_robin(n_partitions: int, rank: int, world: int) -> List[int]:
    """``"partitions"``: partition ``p`` belongs to rank ``p % world``."""
    return [p for p in range(int(n_partitions)) if p % int(world) == int(rank)]


def key_shares(n_partitions: int, rank: int, world: int) -> List[Tuple[int, int, int]]:
    """``"keys"``: ``(partition, hash_lo, hash_hi)`` of replica ``rank``.  Integer arithmetic
    in units of 1/W of a partition, so neighbouring replicas share their bound exactly and the
    replicas' intervals tile every partition's hash space with no gap or overlap."""
    P, W, r = int(n_partitions), int(world), int(rank)
    if not 0 <= r < W:
        raise ValueError(f"rank {r} outside world {W}")
    lo_u, hi_u = r * P, (r + 1) * P           # replica's interval on the line, units of 1/W
    out = []
    for p in range(P):
        a, b = max(lo_u, p * W), min(hi_u, (p + 1) * W)
        if a < b:
            out.append((p, ((a - p * W) * HASH_SPACE) // W, ((b - p * W) * HASH_SPACE) // W))
    return out


def expand_specs(specs: Sequence[Tuple[str, int, int]], n_parts: Dict[str, int]) -> List[Tuple[str, int, int]]:
    """``(topic, partition, offset)`` specs with ``partition == -1`` ("topic:*:offset") expanded
    to every partition of the topic (``n_parts`` from the broker's metadata)."""
    out = []
    for topic, p, off in specs:
        if p == -1:
            if topic not in n_parts:
                raise ValueError(f"topic {topic!r} not in the broker's metadata")
            out.extend((topic, q, off) for q in range(int(n_parts[topic])))
        else:
            out.append((topic, int(p), int(off)))
    return out


class ShardPlan:
    """Resolves a rank's shares of the listed partitions, at every (re)iteration of a stream.

    ``sync(values, ops) -> values``: makes the log snapshot identical on every rank (the end
    offsets' MIN, the start offsets' MAX: each rank sees only records that exist for all of
    them); ``None`` without a process group.  Under ``torch.distributed`` it is an all-reduce,
    so resolving -- i.e. starting an iteration of a sharded stream -- is collective."""

    def __init__(self, specs: Sequence[Tuple[str, int, int]], rank: int, world: int, mode: str = "split",
                 sync: Optional[Callable] = None):
        if mode not in MODES:
            raise ValueError(f"assign must be one of {MODES}, got {mode!r}")
        self.specs = list(specs)
        self.rank, self.world, self.mode, self.sync = int(rank), int(world), mode, sync
        self.last: List[Share] = []

    def resolve(self, client, start_of: Callable[[str, int, int], int], bounded: bool) -> List[Share]:
        specs = expand_specs(self.specs, client.partitions() if any(p == -1 for _, p, _ in self.specs) else {})
        if self.mode == "split" and not bounded:
            raise ValueError("assign='split' needs a bounded read (eof=True); use 'partitions' or 'keys'")
        starts = [int(start_of(t, p, o)) for t, p, o in specs]
        ends = [int(client.latest(t, p)) if bounded else -1 for t, p, _ in specs]
        if self.sync is not None and self.world > 1:
            vals = self.sync(starts + ends, ["max"] * len(starts) + ["min"] * len(ends))
            starts, ends = vals[:len(starts)], vals[len(starts):]
        if self.mode == "split":
            shares = split_rows([(t, p, s, e) for (t, p, _), s, e in zip(specs, starts, ends)], self.rank, self.world)
        elif self.mode == "partitions":
            # whole partitions round-robin over the listed (topic, partition) pairs
            shares = [Share(t, p, s, e) for i, ((t, p, _), s, e) in enumerate(zip(specs, starts, ends))
                      if i % self.world == self.rank]
        else:
            shares = []
            by_topic: Dict[str, List[int]] = {}
            for i, (t, _, _) in enumerate(specs):
                by_topic.setdefault(t, []).append(i)
            for t, idx in by_topic.items():
                for j, lo, hi in key_shares(len(idx), self.rank, self.world):
                    i = idx[j]
                    shares.append(Share(t, specs[i][1], starts[i], ends[i], lo, hi))
        self.last = shares
        return shares


def torch_sync(values, ops):
    """``ShardPlan.sync`` over the default ``torch.distributed`` process group."""
    from ..parallel.dp import agree
    return agree(values, None, ops)


class SegmentPlan:
    """Continuous training from an unbounded topic, one bounded *segment* at a time.

    Rank ``rank`` owns the listed partitions ``i % world == rank`` (consumer-group style, as
    ``"partitions"``) and each :meth:`resolve` -- one ``fit`` epoch over the stream -- hands it
    ``[pos, min(pos + quota, log end))`` of every owned partition, from the plan's own positions.
    The positions move only in :meth:`advance`, which the caller invokes once the model has
    trained every record of the segment (``fit`` trains every row of every share,
    :meth:`Autoencoder._fit_stream_dp`), and :meth:`offsets` is what a checkpoint stores with the
    model (consumer offsets committed with checkpoints).  A job restarted from that
    checkpoint re-reads exactly the records after it: every record is trained once, in the same
    step boundaries, whatever crashed in between.  The reference's idea of training from the
    commit log with no other data store (README.md:124-128), made restartable."""

    def __init__(self, specs: Sequence[Tuple[str, int, int]], rank: int, world: int, quota: int,
                 offsets: Optional[Dict[str, int]] = None):
        if quota <= 0:
            raise ValueError("segment quota must be positive")
        self.specs = list(specs)
        self.rank, self.world, self.quota = int(rank), int(world), int(quota)
        self.mode = "partitions"
        self.sync = None
        self.positions: Dict[str, int] = {str(k): int(v) for k, v in (offsets or {}).items()}
        self.last: List[Share] = []

    @staticmethod
    def key(topic: str, partition: int) -> str:
        return f"{topic}:{int(partition)}"

    def resolve(self, client, start_of: Callable[[str, int, int], int], bounded: bool = True) -> List[Share]:
        specs = expand_specs(self.specs, client.partitions() if any(p == -1 for _, p, _ in self.specs) else {})
        shares = []
        for i, (t, p, o) in enumerate(specs):
            if i % self.world != self.rank:
                continue
            pos = self.positions.get(self.key(t, p), int(o))
            start = int(start_of(t, p, pos))   # honours auto.offset.reset below the log start
            end = min(start + self.quota, int(client.latest(t, p)))
            shares.append(Share(t, int(p), start, max(end, start)))
        self.last = shares
        return shares

    def advance(self) -> None:
        """The last resolved segment has been trained: its ends become the positions."""
        for s in self.last:
            self.positions[self.key(s.topic, s.partition)] = int(s.end)

    def offsets(self) -> Dict[str, int]:
        """This rank's partitions' positions (the checkpoint merges every rank's: they are disjoint;
        positions loaded for other ranks' partitions are not reported back)."""
        owned = {self.key(s.topic, s.partition) for s in self.last}
        return {k: v for k, v in self.positions.items() if k in owned}

    def segment_records(self) -> int:
        return sum(s.rows for s in self.last)
