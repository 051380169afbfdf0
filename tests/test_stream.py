"""Streaming pipeline: sources, tf.data-style transforms vs numpy oracles, Kafka round trip."""
import os

import numpy as np
import pytest

from streamml.data import stream as S
from streamml.data.cardata import FEATURES, normalize_np
from streamml.data.produce import produce

FIX = os.path.join(os.path.dirname(__file__), "fixtures")


def test_csv_source_matches_fixture():
    c = S.csv(os.path.join(FIX, "car-sensor-data.csv"), chunk=3000).collect()
    assert c.x.shape == (10000, 18) and (c.label == 0).all()
    assert c.keys[1] == "car2"
    np.testing.assert_allclose(c.x[0, :3], [39.395103, 34.53991, 123.317406], rtol=1e-6)
    assert set(np.unique(c.x[:, FEATURES.index("control_unit_firmware")])) <= {1000.0, 2000.0}


def test_jsonl_source_handles_both_key_styles():
    c = S.json_lines(os.path.join(FIX, "cardata-v1.jsonl")).collect()
    assert c.x.shape == (10, 18)
    assert c.x[0, FEATURES.index("coolant_temp")] == np.float32(262.26807)
    assert c.x[0, FEATURES.index("tire_pressure_11")] == 33


def test_filter_batch_take_skip_match_tfdata_semantics():
    rng = np.random.default_rng(0)
    x = rng.uniform(0, 10, size=(1000, 18)).astype(np.float32)
    lab = rng.integers(0, 3, size=1000).astype(np.uint8)
    st = S.from_arrays(x, lab, chunk=77).filter_normal().batch(32).skip(2).take(5)
    got = [c.x for c in st]
    ref = x[lab == 0]
    ref_batches = [ref[i:i + 32] for i in range(0, len(ref), 32)][2:7]
    assert len(got) == 5
    for a, b in zip(got, ref_batches):
        np.testing.assert_array_equal(a, b)
    # re-iterable (each epoch restarts the source)
    assert len(list(st)) == 5


def test_normalize_stage_is_reference_normalize_fn():
    x = np.random.default_rng(1).uniform(0, 100, size=(10, 18)).astype(np.float32)
    got = S.from_arrays(x).normalize().collect().x
    np.testing.assert_allclose(got, normalize_np(x), rtol=1e-6)


def test_windows_cross_chunk_boundaries():
    x = np.arange(50 * 18, dtype=np.float32).reshape(50, 18)
    T = 4
    wins = list(S.from_arrays(x, chunk=7).windows(T))
    xs = np.concatenate([w[0] for w in wins])
    ys = np.concatenate([w[1] for w in wins])
    assert xs.shape == (50 - T, T, 18)
    for i in range(50 - T):
        np.testing.assert_array_equal(xs[i], x[i:i + T])
        np.testing.assert_array_equal(ys[i], x[i + T])


@pytest.mark.parametrize("T,h", [(4, 1), (1, 1), (5, 3)])
def test_sliding_windows_are_views_equal_to_window_stream(T, h):
    import torch
    x = np.random.default_rng(T).standard_normal((40, 18)).astype(np.float32)
    wins = list(S.from_arrays(x, chunk=9).windows(T, h))
    xs = np.concatenate([w[0] for w in wins])
    ys = np.concatenate([w[1] for w in wins])
    base = torch.from_numpy(x)
    X, Y = S.sliding_windows(base, T, h)
    assert X.data_ptr() == base.data_ptr() and X.stride() == (18, 18, 1)   # no copy
    np.testing.assert_array_equal(X.numpy(), xs)
    np.testing.assert_array_equal(Y.numpy(), ys)


def test_label_codes():
    assert list(S.label_codes([b"false", "true", "", None, b"FALSE"])) == [0, 1, 2, 2, 0]


def test_synthetic_to_kafka_and_back():
    from streamml.kafka import fake_broker
    src = S.synthetic(5000, chunk=1000, seed=3, failure_rate=0.1)
    n = produce(src, "fake://stream-test", "SENSOR_DATA_S_AVRO", partitions=1)
    assert n == 5000
    back = S.kafka("fake://stream-test", ["SENSOR_DATA_S_AVRO:0:0"], max_bytes=64 << 10).collect()
    ref = src.collect()
    np.testing.assert_allclose(back.x, ref.x, rtol=1e-6)
    np.testing.assert_array_equal(back.label, ref.label)
    assert 0.05 < (back.label == 1).mean() < 0.15
    fake_broker("stream-test").stop()


def test_partition_by_key():
    from streamml.kafka import KafkaClient
    src = S.synthetic(2000, chunk=500, seed=1)  # chunks <= 4096 carry car keys
    produce(src, "fake://pbk", "sensor-data", partitions=4)
    c = KafkaClient("fake://pbk")
    counts = [c.latest("sensor-data", p) for p in range(4)]
    assert sum(counts) == 2000 and min(counts) > 0


def test_select_slice_with_keys():
    c = S.Chunk(np.zeros((5, 18), np.float32), np.zeros(5, np.uint8), list("abcde"), np.arange(5))
    assert c.select(slice(1, 3)).keys == ["b", "c"]
    assert c.select(np.array([True, False, True, False, False])).keys == ["a", "c"]
    b = list(S.Stream(lambda: iter([c, c])).batch(3))
    assert [x.keys for x in b] == [list("abc"), list("dea"), list("bcd"), ["e"]]
