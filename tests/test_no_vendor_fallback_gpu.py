"""The reference models run on the in-tree HIP kernels only: training, prediction and
evaluation of the dense autoencoder (D = 18 and 30), both LSTM stacks and the MNIST MLP
never reach the hipBLASLt fallbacks of ops/dense.py / ops/lstm.py (counted in
ops._ext.FALLBACKS; SML_STRICT_KERNELS=1 would raise)."""
import numpy as np
import pytest
import torch

from streamml.ops import _ext

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def _strict(monkeypatch):
    monkeypatch.setenv("SML_STRICT_KERNELS", "1")
    _ext.FALLBACKS.clear()
    yield
    assert not _ext.FALLBACKS, dict(_ext.FALLBACKS)


@pytest.mark.parametrize("D", [18, 30])
def test_autoencoder_paths(cuda_device, D):
    from streamml.models.autoencoder import Autoencoder
    x = np.random.default_rng(0).uniform(-1, 1, size=(5000, D)).astype(np.float32)
    m = Autoencoder(input_dim=D, device=cuda_device)
    m.compile()
    for bs, eng in ((32, "persistent"), (1000, "launch"), (1024, "auto")):
        m.fit(x, epochs=1, batch_size=bs, verbose=0, engine=eng)
    m.predict(x)
    m.evaluate(x)
    m.score(x)


@pytest.mark.parametrize("stack,T,B", [("reference", 1, 1), ("reference", 1, 64), ("two_layer", 50, 256),
                                       ("reference", 5, 32)])
def test_lstm_paths(cuda_device, stack, T, B):
    from streamml.models.lstm import LSTMPredictor
    ctor = LSTMPredictor.reference if stack == "reference" else LSTMPredictor.two_layer
    m = ctor(look_back=T, device=cuda_device)
    rng = np.random.default_rng(1)
    x = rng.uniform(-1, 1, size=(B * 4, T, 18)).astype(np.float32)
    y = rng.uniform(-1, 1, size=(B * 4, 18)).astype(np.float32)
    m.fit(x, y, epochs=1, batch_size=B, verbose=0)
    m.predict(x)


def test_mlp_paths(cuda_device):
    from streamml.models.mlp import MLPClassifier
    rng = np.random.default_rng(2)
    x = rng.integers(0, 255, size=(512, 28, 28)).astype(np.uint8)
    y = rng.integers(0, 10, size=512)
    for hidden, drop in ((128, 0.0), (512, 0.2)):
        m = MLPClassifier(hidden=hidden, dropout=drop, device=cuda_device)
        m.fit(x, y, epochs=1, batch_size=32, verbose=0)
        m.predict(x)


def test_wide_dense_autoencoder_sequential(cuda_device):
    """An autoencoder wider than the fused AE kernel (100 -> 64 -> 32 -> 64 -> 100) built with
    nn.Sequential trains and predicts on the layer-by-layer engine: K1/K2 for the narrow
    layers, the general MFMA GEMM for the wide ones -- no vendor fallback."""
    from streamml import nn
    rng = np.random.default_rng(3)
    x = rng.uniform(-1, 1, size=(4096, 100)).astype(np.float32)
    m = nn.Sequential([nn.Dense(64, activation="tanh", input_shape=(100,)), nn.Dense(32, activation="relu"),
                       nn.Dense(64, activation="tanh"), nn.Dense(100)], device=cuda_device)
    m.compile(optimizer="adam", loss="mean_squared_error")
    h = m.fit(x, x, epochs=3, batch_size=256, verbose=0)
    assert h.history["loss"][-1] < h.history["loss"][0]
    assert m.predict(x[:300]).shape == (300, 100)
