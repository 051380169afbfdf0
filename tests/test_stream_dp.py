"""Data-parallel training from a partitioned Kafka topic (SURVEY.md 2.4 "stream / partition
parallelism"; the reference's topics have 10 partitions, 01_installConfluentPlatform.sh:180,
re-keyed PARTITION BY CAR, :249, but its consumer reads partition 0 only, cardata-v3.py:44-47).

Each rank streams its own share of every partition (kafka/assign.py) into ``Autoencoder.fit``;
no rank collects the topic.  Checked at 2 and 4 ranks over gloo against a broker with 8
partitions of uneven length: the shares are disjoint and cover every record exactly once, the
label-filtered union is exactly the rows trained, every rank runs the same number of optimizer
steps, and the replicas end bit-identical."""
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
TOPIC = "SENSOR_DATA_S_AVRO"


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def make_broker(rows=4999, partitions=8, failure_rate=0.05, seed=3):
    """An in-process broker (this process; the ranks reach it over 127.0.0.1) holding ``rows``
    keyed car events spread over ``partitions`` by the Kafka murmur2 partitioner."""
    from streamml.data import produce as prod
    from streamml.data import stream as st
    from streamml.kafka import FakeBroker
    b = FakeBroker()
    b.create_topic(TOPIC, partitions)
    n = prod.produce(st.synthetic(rows, chunk=1024, seed=seed, failure_rate=failure_rate), b.address, TOPIC,
                     create=False, partitions=partitions)
    assert n == rows
    return b


def run_ranks(out, broker, world, batch=64, epochs=2, device="cpu", assign="split", native="0", engine="auto",
              dp="auto", extra_env=None, timeout=600):
    env = dict(os.environ, OMP_NUM_THREADS="2", **(extra_env or {}))
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={world}",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}",
           os.path.join(HERE, "helpers", "stream_dp_worker.py"), str(out), broker.address, TOPIC, str(batch),
           str(epochs), device, assign, native, engine, dp]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=timeout, env=env)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    return [dict(np.load(out / f"rank{k}.npz")) for k in range(world)]


def check_run(broker, ranks, batch, epochs, partitions=8):
    # every record of every partition in exactly one rank's share
    seen = {}
    for k, z in enumerate(ranks):
        for p, o in zip(z["parts"].tolist(), z["offs"].tolist()):
            assert (p, o) not in seen, f"record {p}:{o} read by ranks {seen[(p, o)]} and {k}"
            seen[(p, o)] = k
    total = sum(broker.end_offset(TOPIC, p) for p in range(partitions))
    assert len(seen) == total
    # shares balanced to one record
    sizes = [len(z["offs"]) for z in ranks]
    assert max(sizes) - min(sizes) <= 1, sizes
    # every label-filtered row trained, once per epoch; the same step count everywhere
    normal = sum(int((z["labels"] == 0).sum()) for z in ranks)
    for z in ranks:
        np.testing.assert_array_equal(z["rows"], [normal] * epochs)
    its = {int(z["iterations"]) for z in ranks}
    assert len(its) == 1, its
    per_rank_max = max(int((z["labels"] == 0).sum()) for z in ranks)
    assert its.pop() >= epochs * -(-per_rank_max // batch)
    # replicas bit-identical
    w0 = [ranks[0][f"arr_{i}"] for i in range(8)]
    for z in ranks[1:]:
        for i, w in enumerate(w0):
            np.testing.assert_array_equal(z[f"arr_{i}"], w)
    assert all(np.isfinite(z["loss"]).all() for z in ranks)


@pytest.fixture(scope="module")
def broker():
    b = make_broker()
    yield b
    b.stop()


@pytest.mark.dist
@pytest.mark.parametrize("world", [2, 4])
def test_stream_dp_split_shares(tmp_path, broker, world):
    ranks = run_ranks(tmp_path, broker, world, batch=64, epochs=2)
    check_run(broker, ranks, 64, 2)
    # split shares: contiguous offset ranges, no (partition, offset) in two shares
    allsh = np.concatenate([z["shares"] for z in ranks])
    for p in range(8):
        sh = sorted((s, e) for q, s, e in allsh.tolist() if q == p)
        for (s0, e0), (s1, _) in zip(sh, sh[1:]):
            assert e0 == s1


@pytest.mark.dist
def test_stream_dp_partition_shares_uneven(tmp_path, broker):
    """assign='partitions' (whole partitions, p % world) at 3 ranks over 8 partitions: shares of
    unequal size; the tail phase still trains every row and keeps the step counts equal."""
    ranks = run_ranks(tmp_path, broker, 3, batch=64, epochs=1, assign="partitions")
    owned = [sorted(set(z["shares"][:, 0].tolist())) for z in ranks]
    assert owned == [[0, 3, 6], [1, 4, 7], [2, 5]]
    seen = set()
    for z in ranks:
        pairs = set(zip(z["parts"].tolist(), z["offs"].tolist()))
        assert not (pairs & seen)
        seen |= pairs
    normal = sum(int((z["labels"] == 0).sum()) for z in ranks)
    for z in ranks:
        assert z["rows"].tolist() == [normal]
    assert len({int(z["iterations"]) for z in ranks}) == 1


def test_split_rows_exact():
    from streamml.kafka.assign import split_rows
    ranges = [("t", p, 10 * p, 10 * p + n) for p, n in enumerate([5, 0, 17, 3, 9, 1, 0, 12])]
    total = sum(n for *_, n in [(0, 0, 0, e - s) for _, _, s, e in ranges])
    for world in (1, 2, 3, 4, 8, 13, 64):
        got = [split_rows(ranges, r, world) for r in range(world)]
        sizes = [sum(s.rows for s in g) for g in got]
        assert sum(sizes) == total and max(sizes) - min(sizes) <= 1
        cover = sorted((s.partition, o) for g in got for s in g for o in range(s.start, s.end))
        assert cover == sorted((p, o) for _, p, s, e in ranges for o in range(s, e))


def test_expand_star_spec():
    from streamml.kafka.assign import expand_specs
    from streamml.kafka.client import parse_topic_spec
    assert parse_topic_spec("T:*:5") == ("T", -1, 5)
    assert expand_specs([("T", -1, 5), ("U", 2, 0)], {"T": 3}) == [("T", 0, 5), ("T", 1, 5), ("T", 2, 5),
                                                                   ("U", 2, 0)]
