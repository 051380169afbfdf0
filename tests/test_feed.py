"""Native partition-parallel Kafka feed (csrc/io/feed.cpp) vs the chunk-by-chunk Python path.

The feed decodes Confluent-framed Avro records straight into slabs (the pinned ring on a
GPU box; plain numpy buffers here) with an optional decode-time label filter -- the
reference's KafkaDataset -> substr -> decode_avro -> filter(y == "false") chain
(AUTOENCODER-TensorFlow-IO-Kafka/cardata-v3.py:44-75, 212)."""
import numpy as np
import pytest

from streamml.data import stream as S
from streamml.data.avro import AvroCodec
from streamml.data.produce import encode_chunk
from streamml.kafka import fake_broker
from streamml.kafka.client import KafkaClient
from streamml.ops import load_io


@pytest.fixture(scope="module")
def topic():
    name = "feed-unit"
    b = fake_broker(name)
    b.create_topic("T", 4)
    codec = AvroCodec("cardata-v1")
    for i, c in enumerate(S.synthetic(30_000, chunk=2_500, seed=7, failure_rate=0.1)):
        buf, offs = encode_chunk(codec, c.x, c.label)
        b.append_buffer("T", i % 4, buf, offs)
    return f"fake://{name}", [f"T:{p}:0" for p in range(4)]


def _per_partition(servers, specs, native, workers=1):
    out = {}
    for s in specs:
        cs = list(S.kafka(servers, [s], workers=workers, native=native))
        out[s] = (np.concatenate([c.x for c in cs]), np.concatenate([c.label for c in cs]))
    return out


def test_feed_rows_and_labels_match_python_path(topic):
    servers, specs = topic
    a = _per_partition(servers, specs, native=False)
    z = _per_partition(servers, specs, native=True)
    for s in specs:
        np.testing.assert_array_equal(a[s][0], z[s][0])
        np.testing.assert_array_equal(a[s][1], z[s][1])


@pytest.mark.parametrize("workers", [1, 3, 8])
def test_feed_parallel_every_record_once(topic, workers):
    servers, specs = topic
    ref = np.concatenate([c.x for c in S.kafka(servers, specs)])
    got = np.concatenate([c.x for c in S.kafka(servers, specs, workers=workers, native=True)])
    assert got.shape == ref.shape == (30_000, 18)
    # same multiset of rows (partition interleaving differs); per-partition order: test above
    key = lambda x: x[np.lexsort(x.T[::-1])]
    np.testing.assert_array_equal(key(got), key(ref))


def test_feed_decode_time_label_filter(topic):
    servers, specs = topic
    feed = S.kafka(servers, specs, workers=2, native=True).native_feed
    n_kept = 0
    for rows, labs in feed.host_chunks(keep_label=0):
        assert np.all(labs == 0)
        n_kept += len(rows)
    ref = S.kafka(servers, specs).filter_normal().collect()
    assert n_kept == len(ref) and feed.last_stats["dropped"] == 30_000 - n_kept
    assert feed.last_stats["records"] == 30_000 and feed.last_stats["errors"] == 0


def test_feed_bounded_eof_rereads_to_current_end(topic):
    servers, _ = topic
    b = fake_broker("feed-eof")
    b.create_topic("E", 1)
    codec = AvroCodec("cardata-v1")
    c = next(iter(S.synthetic(1000, chunk=1000, seed=1)))
    buf, offs = encode_chunk(codec, c.x, c.label)
    b.append_buffer("E", 0, buf, offs)
    st = S.kafka("fake://feed-eof", ["E:0:0"], native=True)
    assert sum(len(x) for x in st) == 1000
    b.append_buffer("E", 0, buf, offs)
    assert sum(len(x) for x in st) == 2000       # each epoch reads to the end offset at its start
    assert sum(len(x) for x in S.kafka("fake://feed-eof", ["E:0:1500"], native=True)) == 500


def test_feed_commits_positions():
    b = fake_broker("feed-commit")
    b.create_topic("C", 2)
    codec = AvroCodec("cardata-v1")
    c = next(iter(S.synthetic(600, chunk=600, seed=3)))
    buf, offs = encode_chunk(codec, c.x, c.label)
    b.append_buffer("C", 0, buf, offs)
    b.append_buffer("C", 1, buf, offs)
    st = S.kafka("fake://feed-commit", ["C:0:0", "C:1:0"], group="g1", commit=True, workers=2, native=True)
    assert sum(len(x) for x in st) == 1200
    cl = KafkaClient("fake://feed-commit")
    assert cl.committed("g1", "C", 0) == 600 and cl.committed("g1", "C", 1) == 600


def test_feed_early_stop_commits_only_consumed_slabs():
    """At-least-once: stopping after the first slab commits that slab's publish-time
    position, never the workers' decode-ahead positions; a resumed run reads the rest."""
    from streamml.kafka.feed import NativeFeed
    b = fake_broker("feed-early")
    b.create_topic("E", 1)
    codec = AvroCodec("cardata-v1")
    c = next(iter(S.synthetic(5000, chunk=5000, seed=5)))
    buf, offs = encode_chunk(codec, c.x, c.label)
    b.append_buffer("E", 0, buf, offs)
    feed = NativeFeed("fake://feed-early", ["E:0:0"], codec, list(range(18)), group="g", commit=True,
                      resume=True)
    it = feed.host_chunks(slab_rows=1000, slots=4)
    first, _ = next(it)          # the workers decode ahead into the other slots meanwhile
    next(it)                     # coming back for slab 1 marks slab 0 consumed
    it.close()                   # the consumer stops while slab 1 is in its hands
    cl = KafkaClient("fake://feed-early")
    assert cl.committed("g", "E", 0) == 1000, cl.committed("g", "E", 0)
    assert feed.last_stats["committed"] == "consumed-slabs"
    rest = sum(len(r) for r, _ in feed.host_chunks(slab_rows=1000))   # resumes at the commit
    assert rest == 4000 and feed.last_stats["committed"] == "end"
    assert cl.committed("g", "E", 0) == 5000
    np.testing.assert_array_equal(first, c.x[:1000].astype(np.float32))


def test_feed_malformed_records_become_nan_missing():
    b = fake_broker("feed-bad")
    b.create_topic("M", 1)
    cl = KafkaClient("fake://feed-bad")
    codec = AvroCodec("cardata-v1")
    c = next(iter(S.synthetic(3, chunk=3, seed=0)))
    buf, offs = encode_chunk(codec, c.x, c.label)
    good = [bytes(buf[offs[i]:offs[i + 1]]) for i in range(3)]
    cl.produce("M", 0, [good[0], b"\x00\x00\x00\x00\x01\xff\xff", good[2]])
    rows, labs = zip(*S.kafka("fake://feed-bad", ["M:0:0"], native=True).native_feed.host_chunks())
    x, lab = np.concatenate(rows), np.concatenate(labs)
    assert x.shape == (3, 18) and np.isnan(x[1]).all() and lab[1] == 2
    np.testing.assert_array_equal(x[[0, 2]], c.x[[0, 2]].astype(np.float32))


def test_label_code_matches_python():
    lc = load_io().label_code
    assert [lc(b"false"), lc(b" TRUE "), lc(b""), lc(b"maybe")] == [0, 1, 2, 2]


def _bare_feed(codec, feature_idx, label_idx):
    """A KafkaFeed that is never started: only its decode plan is exercised."""
    return load_io().KafkaFeed("127.0.0.1:9", "t", "", "", "", 1000, [f.as_tuple() for f in codec.fields],
                               feature_idx, label_idx, -1, True, 1 << 20, 100, 1, -1.0, [])


def test_fast_decode_plan_matches_codec():
    """The car schema compiles to 5 runs (9 doubles, 4 ints, 4 doubles, 1 int, the label)
    and decodes every record exactly as the Avro codec; truncated / over-long values fail."""
    codec = AvroCodec("cardata-v1")
    names = [f.name for f in codec.fields]
    feat = [names.index(n) for n in codec.numeric_fields]
    f = _bare_feed(codec, feat, names.index(codec.text_fields[0]))
    assert f.fast_plan == 5
    c = next(iter(S.synthetic(500, chunk=500, seed=11, failure_rate=0.3)))
    buf, offs = encode_chunk(codec, c.x, c.label)
    for i in range(500):
        ok, row, lab = f.decode_row(bytes(buf[offs[i]:offs[i + 1]]))
        assert ok and lab == int(c.label[i])
        np.testing.assert_array_equal(np.asarray(row, np.float32), c.x[i].astype(np.float32))
    v = bytes(buf[offs[0]:offs[1]])
    assert not f.decode_row(v[:-3])[0] and not f.decode_row(v + b"\x00")[0]
    # a projection that skips / reorders fields leaves the fast plan's runs consistent
    g = _bare_feed(codec, feat[::-1][:5], -1)
    ok, row, _ = g.decode_row(v)
    assert ok and np.asarray(row, np.float32).tolist() == c.x[0].astype(np.float32)[::-1][:5].tolist()


def test_feed_check_crcs_config(topic):
    """librdkafka's check.crcs=true turns on per-batch CRC-32C verification (default off)."""
    servers, specs = topic
    st = S.kafka(servers, specs[:1], native=True, config=["check.crcs=true"])
    assert st.native_feed.check_crcs
    ref = S.kafka(servers, specs[:1], native=True)
    assert not ref.native_feed.check_crcs
    np.testing.assert_array_equal(np.concatenate([c.x for c in st]), np.concatenate([c.x for c in ref]))


@pytest.mark.parametrize("workers", [1, 3])
def test_feed_staged_values_match_fetched(topic, workers):
    """NativeFeed.stage(): pre-staged record values decoded by the workers into the slabs give the
    same rows (as a multiset: workers publish in any order) and the same decode-time filter as
    fetching them from the broker; each later iteration re-reads the staged values."""
    servers, specs = topic
    codec = AvroCodec("cardata-v1")
    bufs, offs, base = [], [np.zeros(1, np.int64)], 0
    for c in S.synthetic(30_000, chunk=2_500, seed=7, failure_rate=0.1):
        b, o = encode_chunk(codec, c.x, c.label)
        bufs.append(np.frombuffer(b, np.uint8)[:int(o[-1])])
        offs.append(np.asarray(o[1:], np.int64) + base)
        base += int(o[-1])
    buf, offs = np.concatenate(bufs), np.concatenate(offs)
    feed = S.kafka(servers, specs, workers=workers, native=True).native_feed
    feed.stage(buf, offs)
    key = lambda x: x[np.lexsort(x.T[::-1])]   # noqa: E731
    ref = np.concatenate([r for r, _ in S.kafka(servers, specs, native=True).native_feed.host_chunks(keep_label=0)])
    for _ in range(2):
        got = np.concatenate([r for r, labs in feed.host_chunks(keep_label=0) if np.all(labs == 0)])
        np.testing.assert_array_equal(key(got), key(ref))
        assert feed.last_stats["records"] == 30_000 and feed.last_stats["source"] == "staged"
        assert feed.last_stats["dropped"] == 30_000 - len(ref)
