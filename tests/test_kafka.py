"""Kafka wire protocol: client <-> in-process broker over real sockets."""
import numpy as np
import pytest

from streamml.data.avro import AvroCodec
from streamml.kafka import FakeBroker, KafkaClient, KafkaDataset, KafkaOutputSequence, parse_topic_spec
from streamml.ops import load_io

SASL = ["security.protocol=sasl_plaintext", "sasl.username=test", "sasl.password=test123", "sasl.mechanisms=PLAIN"]


@pytest.fixture()
def broker():
    b = FakeBroker()
    b.create_topic("t", 3)
    yield b
    b.stop()


def test_crc32c_known_vector():
    assert load_io().crc32c(b"123456789") == 0xE3069283


def test_topic_spec():
    assert parse_topic_spec("SENSOR_DATA_S_AVRO:0:0") == ("SENSOR_DATA_S_AVRO", 0, 0)
    assert parse_topic_spec("x") == ("x", 0, 0)


def test_produce_fetch_roundtrip(broker):
    c = KafkaClient(broker.address)
    assert c.partitions() == {"t": 3}
    base = c.produce("t", 1, [b"a", b"bb", b""], keys=[b"k1", None, b"k3"], timestamps=[10, 11, 12])
    assert base == 0
    assert c.produce("t", 1, [b"ccc"]) == 3
    r = c.fetch("t", 1, 0)
    vo = r["value_offsets"]
    vals = [r["values"][vo[i]:vo[i + 1]] for i in range(len(vo) - 1)]
    assert vals == [b"a", b"bb", b"", b"ccc"]
    assert list(r["offsets"]) == [0, 1, 2, 3] and list(r["timestamps"][:3]) == [10, 11, 12]
    assert r["keys"][0] == b"k1" and r["high_watermark"] == 4
    assert list(c.fetch("t", 1, 2)["offsets"]) == [2, 3]     # mid-batch start offset filtered
    assert c.earliest("t", 1) == 0 and c.latest("t", 1) == 4 and c.latest("t", 0) == 0


def test_sasl_plain(broker):
    b = FakeBroker(sasl_username="test", sasl_password="test123")
    try:
        b.create_topic("s", 1)
        c = KafkaClient(b.address, SASL)
        c.produce("s", 0, [b"x"])
        assert c.latest("s", 0) == 1
        with pytest.raises(Exception):
            KafkaClient(b.address, SASL[:2] + ["sasl.password=wrong", SASL[3]]).latest("s", 0)
        with pytest.raises(Exception):
            KafkaClient(b.address).latest("s", 0)   # no auth
    finally:
        b.stop()


def test_group_offsets_commit_resume(broker):
    c = KafkaClient(broker.address)
    c.produce("t", 0, [bytes([i]) for i in range(10)])
    assert c.committed("g", "t", 0) == -1
    ds = KafkaDataset(["t:0:0"], servers=broker.address, group="g", commit=True, max_bytes=64)
    n = sum(len(b["offsets"]) for b in ds)
    assert n == 10 and c.committed("g", "t", 0) == 10
    c.produce("t", 0, [b"late"])
    ds2 = KafkaDataset(["t:0:0"], servers=broker.address, group="g", resume=True)
    got = [m for m in ds2.messages()]
    assert got == [b"late"]


def test_eof_bounded_and_reiterable(broker):
    c = KafkaClient(broker.address)
    c.produce("t", 2, [b"%d" % i for i in range(1000)])
    ds = KafkaDataset(["t:2:0"], servers=broker.address, max_bytes=1000)
    a = list(ds.messages())
    c.produce("t", 2, [b"more"])
    assert len(a) == 1000 and a[0] == b"0" and a[-1] == b"999"
    assert len(list(ds.messages())) == 1001      # each epoch re-reads to the current end (README:116)
    assert len(list(KafkaDataset(["t:2:990"], servers=broker.address).messages())) == 11


def test_fault_injection_retries(broker):
    c = KafkaClient(broker.address)
    for _ in range(50):   # one record batch (log segment) each: a fetch returns whole batches
        c.produce("t", 0, [b"x"])
    broker.set_faults(fail_every=2)
    ds = KafkaDataset(["t:0:0"], servers=broker.address, max_bytes=40)
    assert len(list(ds.messages())) == 50
    assert broker.injected_failures > 0


def test_fetch_decode_avro_pipeline(broker):
    codec = AvroCodec("cardata-v1")
    rng = np.random.default_rng(0)
    num = rng.uniform(0, 50, size=(500, 18))
    num[:, 9:13] = np.round(num[:, 9:13])
    num[:, 17] = 2000
    lab = ["false"] * 450 + ["true"] * 50
    buf, offs = codec.encode(num, {"FAILURE_OCCURRED": lab})
    broker.append_buffer("t", 0, buf, offs)
    ds = KafkaDataset(["t:0:0"], servers=broker.address, codec=codec, max_bytes=8192)
    feats, labels = [], []
    for b in ds:
        feats.append(b["numeric"])
        labels += b["text"]["FAILURE_OCCURRED"]
    x = np.concatenate(feats)
    np.testing.assert_allclose(x, num.astype(np.float32), rtol=1e-6)
    assert labels == [s.encode() for s in lab]


def test_output_sequence_orders_by_index(broker):
    out = KafkaOutputSequence("t", servers=broker.address, partition=1, batch_records=3)
    for i in [2, 0, 1, 4, 3]:
        out.setitem(i, f"[{i}]")
    out.flush()
    assert [v for _, _, v in broker.read("t", 1, 0)] == [b"[0]", b"[1]", b"[2]", b"[3]", b"[4]"]
    with pytest.raises(IndexError):
        out.setitem(1, "dup")


def test_fake_scheme_resolves_to_inprocess_broker():
    from streamml.kafka import fake_broker
    b = fake_broker("unit")
    b.create_topic("u", 1)
    c = KafkaClient("fake://unit")
    c.produce("u", 0, [b"hi"])
    assert list(KafkaDataset(["u:0:0"], servers="fake://unit").messages()) == [b"hi"]


def test_partition_parallel_consumption_matches_serial():
    """workers > 1: every record exactly once, per-partition order kept, labels from C++ codes."""
    import numpy as np
    from streamml.data import stream as S
    from streamml.data.avro import AvroCodec
    from streamml.data.produce import encode_chunk
    from streamml.kafka import fake_broker
    b = fake_broker("parallel-consume")
    b.create_topic("T", 5)
    codec = AvroCodec("cardata-v1")
    for i, c in enumerate(S.synthetic(20_000, chunk=1500, seed=2, failure_rate=0.2)):
        buf, offs = encode_chunk(codec, c.x, c.label)
        b.append_buffer("T", i % 5, buf, offs)
    specs = [f"T:{p}:0" for p in range(5)]
    serial = list(S.kafka("fake://parallel-consume", specs, max_bytes=64 << 10))
    par = list(S.kafka("fake://parallel-consume", specs, max_bytes=64 << 10, workers=3))

    def by_part(chunks):
        out = {}
        for c in chunks:
            out.setdefault(c.meta["partition"], []).append(c)
        return {p: (np.concatenate([c.x for c in cs]), np.concatenate([c.label for c in cs]),
                    np.concatenate([c.offsets for c in cs])) for p, cs in out.items()}
    a, z = by_part(serial), by_part(par)
    assert sorted(a) == sorted(z) == list(range(5))
    for p in a:
        for u, v in zip(a[p], z[p]):
            np.testing.assert_array_equal(u, v)
    labels = np.concatenate([c.label for c in serial])
    assert 0.1 < (labels == 1).mean() < 0.3 and set(np.unique(labels)) <= {0, 1}
