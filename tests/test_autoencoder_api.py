"""Keras-like Autoencoder API on the CPU path (torch reference backend)."""
import os

import numpy as np
import pytest
import torch

from streamml.data import stream as S
from streamml.data.cardata import normalize_np
from streamml.models.autoencoder import Autoencoder, load_model
from streamml.models.reference import ae_forward_torch
from streamml.nn import KafkaPredictionSink, ModelCheckpoint, TensorBoard
from streamml.obs import read_scalars

FIX = os.path.join(os.path.dirname(__file__), "fixtures")


@pytest.fixture(scope="module")
def car_rows():
    return S.csv(os.path.join(FIX, "car-sensor-data.csv")).collect().x


def test_fit_cpu_csv_loss_decreases(car_rows, tmp_path):
    m = Autoencoder(device="cpu", input_normalizer="cardata", seed=1)
    m.compile(optimizer="adam", loss="mean_squared_error", metrics=["accuracy"])
    h = m.fit(car_rows[:4000], epochs=3, batch_size=32, verbose=0,
              callbacks=[TensorBoard(str(tmp_path / "logs"))], validation_data=(car_rows[4000:5000],))
    assert len(h.history["loss"]) == 3 and h.history["loss"][-1] < h.history["loss"][0]
    assert set(h.history) >= {"loss", "accuracy", "val_loss", "val_accuracy"}
    assert m.iterations == 3 * 125
    ev = [f for f in os.listdir(tmp_path / "logs" / "train")]
    sc = read_scalars(str(tmp_path / "logs" / "train" / ev[0]))
    assert [t for _, _, t, _ in sc].count("epoch_loss") == 3
    assert abs(sc[0][3] - h.history["loss"][0]) < 1e-5


def test_save_load_roundtrip_cpu(car_rows, tmp_path):
    m = Autoencoder(device="cpu", input_normalizer="cardata")
    m.compile()
    m.fit(car_rows[:640], epochs=1, batch_size=32, verbose=0)
    p = str(tmp_path / "model1.h5")
    m.save(p)
    m2 = load_model(p, device="cpu", input_normalizer="cardata")
    for a, b in zip(m.get_weights(), m2.get_weights()):
        np.testing.assert_array_equal(a, b)
    assert m2.iterations == 20
    np.testing.assert_allclose(m.predict(car_rows[:100]), m2.predict(car_rows[:100]), rtol=1e-6)
    # training continues from the restored Adam state exactly
    m.fit(car_rows[640:960], epochs=1, batch_size=32, verbose=0, shuffle=False)
    m2.fit(car_rows[640:960], epochs=1, batch_size=32, verbose=0, shuffle=False)
    for a, b in zip(m.get_weights(), m2.get_weights()):
        np.testing.assert_allclose(a, b, rtol=1e-5, atol=1e-7)


def test_load_reference_model_and_score():
    m = load_model(os.path.join(FIX, "autoencoder_sensor_anomaly_detection.h5"), device="cpu")
    assert m.spec.input_dim == 30 and m.iterations == 35545
    assert m.count_params() == 835
    assert m.spec.activity_l1 == pytest.approx(1e-7)
    x = np.random.default_rng(0).standard_normal((64, 30)).astype(np.float32)
    y_ref, _ = ae_forward_torch(torch.from_numpy(x), [torch.from_numpy(w) for w in m.get_weights()],
                                m.spec.activations)
    np.testing.assert_allclose(m.predict(x, batch_size=16), y_ref.numpy(), rtol=1e-5, atol=1e-6)
    s = m.score(x)
    np.testing.assert_allclose(s, ((y_ref.numpy() - x) ** 2).mean(1), rtol=1e-5)
    assert m.detect(x, threshold=5.0).dtype == bool
    assert "Total params: 835" in m.summary(print_fn=None)


def test_quirk_file_loads():
    m = load_model(os.path.join(FIX, "autoencoder_sensor_anomaly_detection_fully_trained_100_epochs.h5"),
                   device="cpu")
    assert m.layer_names[1] == "dense_4" and m.weight_names[0] == "dense_4_1/kernel:0"
    assert m.iterations == 167132


def test_checkpoint_best_only(car_rows, tmp_path):
    m = Autoencoder(device="cpu", input_normalizer="cardata")
    m.compile()
    ck = ModelCheckpoint(str(tmp_path / "best.h5"), monitor="val_loss", save_best_only=True)
    m.fit(car_rows[:320], epochs=3, batch_size=32, verbose=0, callbacks=[ck], validation_data=(car_rows[320:480],))
    assert len(ck.saved) >= 1 and os.path.exists(tmp_path / "best.h5")


def test_stream_fit_and_kafka_prediction_sink(car_rows):
    from streamml.kafka import fake_broker
    b = fake_broker("ae-api")
    b.create_topic("model-predictions", 1)
    m = Autoencoder(device="cpu", input_normalizer="cardata")
    m.compile()
    st = S.from_arrays(car_rows[:1000], chunk=333)
    h = m.fit(st, epochs=1, batch_size=100, verbose=0, steps_per_epoch=5)
    assert m.iterations == 5 and h.history["loss"]
    sink = KafkaPredictionSink(100, "model-predictions", "fake://ae-api")
    out = m.predict(car_rows[:250], batch_size=100, callbacks=[sink])
    recs = b.read("model-predictions", 0, 0)
    assert len(recs) == 250
    assert recs[7][2].decode() == np.array2string(out[7])


def test_compile_rejects_unknown_minibatch_precision():
    import pytest as _pt

    from streamml.models.autoencoder import Autoencoder
    with _pt.raises(ValueError):
        Autoencoder(device="cpu").compile(minibatch_precision="fp8")
    Autoencoder(device="cpu").compile(minibatch_precision="bf16")   # a no-op on the CPU backend
