"""Generic Keras-style builder (streamml.nn): Sequential / functional Model, compile/fit/
predict/evaluate/save/load_model, including loading the reference's own .h5 files."""
import os

import numpy as np
import pytest
import torch

import streamml.nn as nn

FIX = os.path.join(os.path.dirname(__file__), "fixtures")


def _ae(D=18):
    inp = nn.Input(shape=(D,))
    e = nn.Dense(14, activation="tanh", activity_regularizer=nn.regularizers.l1(1e-7))(inp)
    e = nn.Dense(7, activation="relu")(e)
    d = nn.Dense(7, activation="tanh")(e)
    d = nn.Dense(D, activation="relu")(d)
    return nn.Model(inputs=inp, outputs=d, device="cpu")


def test_functional_autoencoder_matches_dedicated_model(tmp_path):
    from streamml.models.autoencoder import Autoencoder
    m = _ae()
    m.compile(metrics=["accuracy"], loss="mean_squared_error", optimizer="adam")
    assert m.count_params() == 571 and not m.fused
    assert [l.name for l in m.layers] == ["input_1", "dense", "dense_1", "dense_2", "dense_3"]
    ref = Autoencoder(device="cpu")
    ref.set_weights(m.get_weights())
    ref.compile()
    x = np.random.default_rng(0).uniform(-1, 1, (640, 18)).astype(np.float32)
    h1 = m.fit(x, x, epochs=2, batch_size=32, shuffle=False, verbose=0)
    h2 = ref.fit(x, epochs=2, batch_size=32, shuffle=False, verbose=0)
    np.testing.assert_allclose(h1.history["loss"], h2.history["loss"], rtol=1e-5)
    for a, b in zip(m.get_weights(), ref.get_weights()):
        np.testing.assert_allclose(a, b, rtol=1e-5, atol=1e-6)
    path = str(tmp_path / "ae.h5")
    m.save(path)
    m2 = nn.load_model(path, device="cpu")
    assert m2.functional and m2.layers[1].activity_regularizer.l1 == pytest.approx(1e-7)
    np.testing.assert_allclose(m2.predict(x), m.predict(x), rtol=1e-6)
    assert m2.opt.state()[0] == m.opt.state()[0] == 40
    # the dedicated loader reads the generic model's file too
    from streamml.models.autoencoder import load_model as ae_load
    np.testing.assert_allclose(ae_load(path, device="cpu").predict(x), m.predict(x), rtol=1e-5, atol=1e-6)


def test_load_reference_h5():
    from streamml.models.autoencoder import load_model as ae_load
    for f in ("autoencoder_sensor_anomaly_detection.h5",
              "autoencoder_sensor_anomaly_detection_fully_trained_100_epochs.h5"):
        m = nn.load_model(os.path.join(FIX, f), device="cpu")
        assert m.count_params() == 835
        x = np.random.default_rng(1).normal(size=(256, 30)).astype(np.float32)
        np.testing.assert_allclose(m.predict(x), ae_load(os.path.join(FIX, f), device="cpu").predict(x),
                                   rtol=1e-5, atol=1e-6)
    assert m.opt.state()[0] == 167132


def test_sequential_lstm_reference_stack(tmp_path):
    from streamml.models.lstm import LSTMPredictor
    T = 3
    s = nn.Sequential([nn.LSTM(32, activation="relu", input_shape=(T, 18), return_sequences=True),
                       nn.LSTM(16, activation="relu"), nn.RepeatVector(T),
                       nn.LSTM(16, activation="relu", return_sequences=True),
                       nn.LSTM(32, activation="relu", return_sequences=True),
                       nn.TimeDistributed(nn.Dense(18))], device="cpu")
    s.compile(metrics=["accuracy"], loss="mean_squared_error", optimizer="adam")
    assert s.count_params() == 18642
    ref = LSTMPredictor.reference(look_back=T, device="cpu")
    ref.fp.set(s.get_weights())
    xs = np.random.default_rng(2).uniform(-1, 1, (32, T, 18)).astype(np.float32)
    np.testing.assert_allclose(s.predict(xs), ref.forward(torch.as_tensor(xs)).detach().numpy(), rtol=1e-5,
                               atol=1e-6)
    s.fit(xs, xs[:, -1], epochs=1, batch_size=8, verbose=0)
    path = str(tmp_path / "lstm.h5")
    s.save(path)
    s2 = nn.load_model(path, device="cpu")
    np.testing.assert_allclose(s2.predict(xs), s.predict(xs), rtol=1e-6)
    # and the dedicated LSTM loader reads it
    np.testing.assert_allclose(LSTMPredictor.load(path, device="cpu").predict(xs).reshape(32, T, 18),
                               s.predict(xs), rtol=1e-5, atol=1e-6)


def test_mnist_sequential_sparse_ce(tmp_path):
    from streamml.data.mnist import synthetic_mnist
    x, y = synthetic_mnist(2000, seed=0)
    m = nn.Sequential([nn.Flatten(input_shape=(28, 28)), nn.Dense(64, activation="relu"), nn.Dropout(0.2),
                       nn.Dense(10, activation="softmax")], device="cpu")
    m.compile(optimizer="adam", loss="sparse_categorical_crossentropy", metrics=["accuracy"])
    h = m.fit(x / 255.0, y, epochs=2, batch_size=32, validation_data=(x[:500] / 255.0, y[:500]), verbose=0)
    assert h.history["val_accuracy"][-1] > 0.9
    p = m.predict(x[:10] / 255.0)
    np.testing.assert_allclose(p.sum(1), 1, rtol=1e-5)
    m.save(str(tmp_path / "mn.h5"))
    m2 = nn.load_model(str(tmp_path / "mn.h5"), device="cpu")
    np.testing.assert_allclose(m2.predict(x[:10] / 255.0), p, rtol=1e-5, atol=1e-7)


@pytest.mark.parametrize("loss", ["mae", "binary_crossentropy", "categorical_crossentropy"])
def test_other_losses_train(loss):
    rng = np.random.default_rng(3)
    x = rng.normal(size=(512, 8)).astype(np.float32)
    if loss == "binary_crossentropy":
        y = (x[:, :1] > 0).astype(np.float32)
        m = nn.Sequential([nn.Dense(8, activation="relu", input_shape=(8,)), nn.Dense(1, activation="sigmoid")],
                          device="cpu")
    elif loss == "categorical_crossentropy":
        y = np.eye(3, dtype=np.float32)[np.argmax(x[:, :3], 1)]
        m = nn.Sequential([nn.Dense(16, activation="relu", input_shape=(8,)), nn.Dense(3, activation="softmax")],
                          device="cpu")
    else:
        y = x[:, :2] * 0.5
        m = nn.Sequential([nn.Dense(2, input_shape=(8,))], device="cpu")
    m.compile(optimizer=nn.optimizers.Adam(learning_rate=1e-2), loss=loss, metrics=["accuracy"])
    h = m.fit(x, y, epochs=5, batch_size=32, verbose=0)
    assert h.history["loss"][-1] < h.history["loss"][0]


def test_fit_on_stream_and_generator():
    from streamml.data import stream as st
    m = _ae()
    m.compile(metrics=["accuracy"])
    s = st.synthetic(2000, chunk=512).normalize()
    h = m.fit(s, epochs=1, batch_size=100, steps_per_epoch=10, verbose=0)
    assert h.history["loss"][0] > 0
    gen = lambda: ((np.ones((4, 18), np.float32), np.ones((4, 18), np.float32)) for _ in range(3))  # noqa: E731
    m.fit(gen, epochs=1, verbose=0)
