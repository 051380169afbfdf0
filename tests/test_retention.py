"""Time / size retention of the in-process broker (Kafka retention.ms / retention.bytes, deleted in
whole segments by a periodic check) and the consumers' auto.offset.reset after OFFSET_OUT_OF_RANGE.
Reference: the topics are created with ``--config retention.ms=100000``
(infrastructure/confluent/01_installConfluentPlatform.sh:180, 183)."""
import time

import pytest

from streamml.kafka.client import FakeBroker, KafkaClient, error_code, offset_reset_policy
from streamml.kafka.dataset import KafkaDataset


def _fill(b, topic, n, batch=1024, part=0):  # noqa: E302
    for i in range(0, n, batch):
        b.append(topic, part, [b"v%08d" % k for k in range(i, min(n, i + batch))])


def test_time_retention_deletes_old_segments_and_consumer_resets():
    b = FakeBroker(retention_check_ms=20)
    try:
        b.create_topic("sensor-data", 2, retention_ms=150)
        b.create_topic("keep", 1)                      # broker default: unbounded
        _fill(b, "sensor-data", 4096)
        _fill(b, "keep", 2048)
        assert b.start_offset("sensor-data", 0) == 0
        time.sleep(0.4)                                # > retention.ms plus a check interval
        assert b.start_offset("sensor-data", 0) == 4096 and b.end_offset("sensor-data", 0) == 4096
        assert b.deleted_records >= 4096 and b.deleted_segments >= 4
        assert b.start_offset("keep", 0) == 0          # other topics keep their log
        b.create_topic("sensor-data", 2, retention_ms=-1)   # (no timing race with what follows)
        _fill(b, "sensor-data", 1000)                  # new records after the deletion
        c = KafkaClient(b.address)
        with pytest.raises(Exception) as ei:
            c.fetch("sensor-data", 0, 10)
        assert error_code(ei.value) == 1               # OFFSET_OUT_OF_RANGE
        ds = KafkaDataset(["sensor-data:0:0"], servers=b.address, eof=True)
        got = [int(o) for bt in ds for o in bt["offsets"]]
        assert got == list(range(4096, 5096))
        assert ds.records_skipped == 4096
        ds = KafkaDataset(["sensor-data:0:0"], servers=b.address, eof=True,
                          config_global=["auto.offset.reset=none"])
        with pytest.raises(Exception):
            list(ds)
    finally:
        b.stop()


def test_size_retention_keeps_newest_segment_and_bounds_bytes():
    b = FakeBroker(retention_check_ms=10_000)          # no background pass during the test
    try:
        b.create_topic("t", 1, retention_bytes=40_000)
        _fill(b, "t", 10 * 1024)
        before = b.log_bytes()
        dropped = b.enforce_retention()
        seg = before // 10 + 1                          # one 1024-record segment
        # Kafka's rule: delete while the log minus its oldest segment still holds retention.bytes
        assert dropped > 0 and 40_000 <= b.log_bytes() < 40_000 + seg
        assert b.end_offset("t", 0) == 10 * 1024 and b.start_offset("t", 0) > 0
        assert b.log_segments() >= 1
        b.create_topic("t", 1, retention_bytes=0)
        b.enforce_retention()
        assert b.log_segments() == 1                   # the newest segment always stays
    finally:
        b.stop()


def test_latest_reset_and_bounded_cursor_done():
    b = FakeBroker(retention_check_ms=10_000)
    try:
        b.create_topic("t", 1, retention_ms=0)
        _fill(b, "t", 2048)
        time.sleep(0.01)
        b.enforce_retention()
        _fill(b, "t", 512)
        ds = KafkaDataset(["t:0:0"], servers=b.address, eof=False, idle_timeout_s=0.3,
                          config_global=["auto.offset.reset=largest"])
        assert list(ds) == []                          # jumped to the end, nothing new arrived
        assert ds.records_skipped == 2048 + 512
    finally:
        b.stop()


def test_offset_reset_policy_aliases():
    assert offset_reset_policy([]) == "earliest"
    assert offset_reset_policy(["auto.offset.reset=smallest"]) == "earliest"
    assert offset_reset_policy(["auto.offset.reset=end"]) == "latest"
    assert offset_reset_policy({"auto.offset.reset": "error"}) == "none"
    with pytest.raises(ValueError):
        offset_reset_policy(["auto.offset.reset=middle"])


def test_connection_threads_are_reaped():
    import os
    # relative to the process's own threads at the start (torch / OpenMP pools of earlier tests
    # in the same pytest process vary with the machine)
    base = len(os.listdir(f"/proc/{os.getpid()}/task"))
    b = FakeBroker()
    try:
        b.create_topic("t", 1)
        for _ in range(50):
            c = KafkaClient(b.address)
            c.partitions()
            del c
        import gc
        gc.collect()
        time.sleep(0.2)
        KafkaClient(b.address).partitions()            # an accept reaps the finished threads
        # the broker's threads are native; count them via /proc: the 50 finished connections'
        # threads are gone, the broker's own few remain
        n = len(os.listdir(f"/proc/{os.getpid()}/task")) - base
        assert n < 25, (n, base)
    finally:
        b.stop()


def _avro_records(n, seed=0):
    import numpy as np
    from streamml.data import stream as S
    from streamml.data.avro import AvroCodec
    from streamml.data.produce import encode_chunk
    c = next(iter(S.synthetic(n, chunk=n, seed=seed, failure_rate=0.0)))
    buf, offs = encode_chunk(AvroCodec("cardata-v1"), c.x, c.label)
    return c.x.astype(np.float32), buf, np.asarray(offs)


def _expire(b, topic, n_old, seed=1):
    _, buf, offs = _avro_records(n_old, seed)
    b.append_buffer(topic, 0, buf, offs)
    time.sleep(0.01)
    assert b.enforce_retention() > 0 and b.start_offset(topic, 0) == n_old


def test_scoring_loop_resets_after_retention():
    """The C++ serving loop positioned inside a deleted range (explicit start 0) follows
    auto.offset.reset instead of failing, and counts what it jumped over."""
    from streamml.kafka.scoreloop import LowLatencyScorer
    from streamml.ops._ext import load_io
    b = FakeBroker(retention_check_ms=10_000)
    try:
        b.create_topic("S", 1, retention_ms=0)
        b.create_topic("R", 1)
        _expire(b, "S", 3000)
        b.create_topic("S", 1, retention_ms=-1)        # keep what comes next
        x, buf, offs = _avro_records(500, seed=2)
        b.append_buffer("S", 0, buf, offs)
        loop = LowLatencyScorer(b.address, "S", "R", [0], load_io().EchoScorer(18, 5.0), starts=[0], max_wait_ms=5)
        st = loop.run(idle_timeout_s=0.3)
        assert st["events"] == 500 and st["reset_skipped"] == 3000
        assert loop.positions() == [3500]
    finally:
        b.stop()


def test_native_feed_resets_after_retention(monkeypatch):
    """The C++ feed worker gets OFFSET_OUT_OF_RANGE for a deleted position and resets to the log
    start (the Python start-offset clamp is bypassed so the worker itself sees the error)."""
    import numpy as np
    from streamml.data.avro import AvroCodec
    from streamml.kafka.feed import NativeFeed
    b = FakeBroker(retention_check_ms=10_000)
    try:
        b.create_topic("F", 1, retention_ms=0)
        _expire(b, "F", 2048)
        b.create_topic("F", 1, retention_ms=-1)
        x, buf, offs = _avro_records(700, seed=3)
        b.append_buffer("F", 0, buf, offs)
        monkeypatch.setattr(NativeFeed, "_start", lambda self, client, t, p, o: int(o))
        feed = NativeFeed(b.address, ["F:0:0"], AvroCodec("cardata-v1"), list(range(18)))
        rows = np.concatenate([r for r, _ in feed.host_chunks(slab_rows=256)])
        np.testing.assert_array_equal(rows, x)
        assert feed.last_stats["reset_skipped"] == 2048
    finally:
        b.stop()


def test_ordered_parallel_reader_matches_sequential_order():
    """KafkaDataset(workers > 1, ordered=True) yields exactly the sequential reader's batches."""
    b = FakeBroker()
    try:
        b.create_topic("o", 5)
        for p in range(5):
            _fill(b, "o", 3000 + 500 * p, part=p)
        seq = [(bt["partition"], list(bt["offsets"])) for bt in
               KafkaDataset(["o:*:0"], servers=b.address, eof=True, max_bytes=20_000)]
        for _ in range(3):
            par = [(bt["partition"], list(bt["offsets"])) for bt in
                   KafkaDataset(["o:*:0"], servers=b.address, eof=True, max_bytes=20_000, workers=3, ordered=True)]
            assert par == seq
    finally:
        b.stop()


def test_rescaled_serving_groups_seeded_from_previous_commits():
    """serve: a replica's per-replica group (<base>.<r>-of-<w>, used when a partition is shared by
    key) starts from the minimum position the previous layout committed (at-least-once)."""
    from streamml.cli.serve import seed_group_offsets
    b = FakeBroker()
    try:
        b.create_topic("s", 3)
        c = KafkaClient(b.address)
        c.commit("g.0-of-2", "s", 1, 700)       # old layout: two replicas shared partition 1
        c.commit("g.1-of-2", "s", 1, 650)
        c.commit("g", "s", 0, 900)
        got = seed_group_offsets(c, "s", "g", "g.2-of-3", [0, 1, 2])
        assert got == {0: 900, 1: 650}         # partition 2 was never consumed: left alone
        assert c.committed("g.2-of-3", "s", 1) == 650 and c.committed("g.2-of-3", "s", 2) < 0
        c.commit("g.2-of-3", "s", 1, 800)       # an existing commit is never overwritten
        assert seed_group_offsets(c, "s", "g", "g.2-of-3", [1]) == {}
        # a sibling of the same replica count owns another key share: never a seed
        c.commit("g.0-of-3", "s", 2, 500)
        assert seed_group_offsets(c, "s", "g", "g.1-of-3", [2]) == {}
    finally:
        b.stop()
