"""``Autoencoder.fit`` on the persistent small-batch kernel vs an fp32 torch Keras oracle.

The reference's primary job is cardata-v3's ``fit(batch(100).take(100), epochs=20)``
(AUTOENCODER-TensorFlow-IO-Kafka/cardata-v3.py:176-177, 212-222).  These tests run
that step sequence -- array input with Keras' short final batch, and a streamed,
label-filtered, ``take``-capped input -- through ``fit(engine="persistent")`` and
compare the parameter trajectory with plain fp32 PyTorch Keras-Adam steps
(rtol 2e-4: the kernel is fp32 end to end)."""
import numpy as np
import pytest
import torch

from streamml.data import stream as S
from streamml.data.cardata import normalize_affine
from streamml.models.autoencoder import Autoencoder
from streamml.models.reference import TorchAE

pytestmark = pytest.mark.gpu


def _oracle(model_w, xn, B, nsteps):
    ref = TorchAE([(18, 14), (14, 7), (7, 7), (7, 18)], ("tanh", "relu", "tanh", "relu"), 1e-7, model_w)
    for s in range(nsteps):
        ref.step(torch.from_numpy(xn[s * B:(s + 1) * B]))
    return ref


def _compare(m, ref, steps):
    assert m.iterations == steps
    for got, want in zip(m.get_weights(), ref.get_weights()):
        np.testing.assert_allclose(got, want, rtol=2e-4, atol=2e-5)


@pytest.mark.parametrize("B,n", [(100, 100 * 100 + 37), (32, 32 * 64), (128, 128 * 20 + 5)])
def test_fit_array_persistent_matches_torch(cuda_device, B, n):
    rng = np.random.default_rng(5)
    raw = rng.uniform(0, 40, size=(n, 18)).astype(np.float32)
    sc, sh = normalize_affine()
    xn = (raw * sc + sh).astype(np.float32)
    m = Autoencoder(device=cuda_device, input_normalizer="cardata", seed=3)
    w0 = m.get_weights()
    m.compile()
    h = m.fit(raw, epochs=1, batch_size=B, shuffle=False, verbose=0, engine="persistent")
    steps = -(-n // B)
    ref = _oracle(w0, xn, B, steps)
    _compare(m, ref, steps)
    rm = ref.read_metrics()
    assert abs(h.history["loss"][-1] - rm["loss"]) <= 1e-4 * max(1.0, rm["loss"])
    assert abs(h.history["accuracy"][-1] - rm["accuracy"]) < 1e-6


def test_fit_stream_filtered_take_matches_torch(cuda_device):
    """filter_normal(device=True) -> batch(100).take(100), as cardata-v3.py:212-218."""
    B, take = 100, 100
    src = S.synthetic(30_000, chunk=7_001, seed=2, failure_rate=0.05)   # chunks straddle batches
    m = Autoencoder(device=cuda_device, input_normalizer="cardata", seed=1)
    w0 = m.get_weights()
    m.compile()
    m.fit(src.filter_normal(device=True), epochs=1, batch_size=B, steps_per_epoch=take, verbose=0,
          engine="persistent")
    kept = src.filter_normal().collect().x
    sc, sh = normalize_affine()
    xn = (kept * sc + sh).astype(np.float32)
    ref = _oracle(w0, xn, B, take)
    _compare(m, ref, take)


def test_fit_persistent_shuffled_close_to_launch_path(cuda_device):
    """Same shuffled epochs through both engines: the bf16 launch path stays close."""
    rng = np.random.default_rng(9)
    raw = rng.uniform(0, 40, size=(100 * 30, 18)).astype(np.float32)
    a = Autoencoder(device=cuda_device, input_normalizer="cardata", seed=4)
    b = Autoencoder(device=cuda_device, input_normalizer="cardata", seed=4)
    a.compile()
    b.compile()
    ha = a.fit(raw, epochs=2, batch_size=100, verbose=0, engine="persistent")
    hb = b.fit(raw, epochs=2, batch_size=100, verbose=0, engine="launch")
    assert a.iterations == b.iterations == 60
    for ga, gb in zip(a.get_weights(), b.get_weights()):
        assert np.max(np.abs(ga - gb)) < 2e-3 * 60
    assert abs(ha.history["loss"][-1] - hb.history["loss"][-1]) < 0.05 * hb.history["loss"][-1]


def test_fit_auto_engine_picks_persistent(cuda_device, monkeypatch):
    m = Autoencoder(device=cuda_device, input_normalizer="cardata")
    m.compile()
    calls = []
    orig = m.backend.train_rows
    monkeypatch.setattr(m.backend, "train_rows", lambda *a, **k: calls.append(1) or orig(*a, **k))
    m.fit(np.random.default_rng(0).uniform(0, 40, (1000, 18)).astype(np.float32), batch_size=100, verbose=0)
    assert calls, "fit(batch_size=100) did not use the persistent kernel"
    with pytest.raises(ValueError):
        m.fit(np.zeros((1000, 18), np.float32), batch_size=256, verbose=0, engine="persistent")


def test_fit_native_kafka_feed_matches_torch(cuda_device):
    """Kafka (in-process broker) -> native C++ feed (decode-time label filter, pinned slabs,
    H2D) -> persistent-kernel fit: the same Keras trajectory as the fp32 oracle on the
    filtered rows (one partition, so the row order is the log order)."""
    from streamml.data.avro import AvroCodec
    from streamml.data.produce import encode_chunk
    from streamml.kafka import fake_broker
    b = fake_broker("fit-native-gpu")
    b.create_topic("SENSOR_DATA_S_AVRO", 1)
    codec = AvroCodec("cardata-v1")
    src = S.synthetic(25_000, chunk=5_000, seed=11, failure_rate=0.05)
    for c in src:
        buf, offs = encode_chunk(codec, c.x, c.label)
        b.append_buffer("SENSOR_DATA_S_AVRO", 0, buf, offs)
    st = S.kafka("fake://fit-native-gpu", ["SENSOR_DATA_S_AVRO:0:0"], native=True)
    B, take = 100, 150
    m = Autoencoder(device=cuda_device, input_normalizer="cardata", seed=2)
    w0 = m.get_weights()
    m.compile()
    m.fit(st.filter_normal(device=True), epochs=1, batch_size=B, steps_per_epoch=take, verbose=0,
          engine="persistent")
    kept = src.filter_normal().collect().x
    sc, sh = normalize_affine()
    ref = _oracle(w0, (kept * sc + sh).astype(np.float32), B, take)
    _compare(m, ref, take)
    assert st.native_feed.last_stats["records"] > 0


def test_native_device_chunks_equal_host_rows(cuda_device):
    from streamml.data.avro import AvroCodec
    from streamml.data.produce import encode_chunk
    from streamml.kafka import fake_broker
    b = fake_broker("chunks-native-gpu")
    b.create_topic("T", 3)
    codec = AvroCodec("cardata-v1")
    for i, c in enumerate(S.synthetic(40_000, chunk=4_000, seed=5, failure_rate=0.1)):
        buf, offs = encode_chunk(codec, c.x, c.label)
        b.append_buffer("T", i % 3, buf, offs)
    specs = [f"T:{p}:0" for p in range(3)]
    feed = S.kafka("fake://chunks-native-gpu", specs, workers=3, native=True).native_feed
    dev = torch.cat([x.clone() for x in feed.device_chunks(cuda_device, keep_label=0, slab_rows=4096)])
    host = np.concatenate([r for r, _ in feed.host_chunks(keep_label=0)])
    got = dev.cpu().numpy()
    key = lambda x: x[np.lexsort(x.T[::-1])]
    assert got.shape == host.shape
    np.testing.assert_array_equal(key(got), key(host))
    assert feed.last_stats["dropped"] > 0
