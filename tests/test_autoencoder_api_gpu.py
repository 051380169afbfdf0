"""Autoencoder API on the ROCm path: fused kernels, DeviceLoader ring, save/load."""
import os

import numpy as np
import pytest
import torch

from streamml.data import stream as S
from streamml.models.autoencoder import Autoencoder, load_model

pytestmark = pytest.mark.gpu
FIX = os.path.join(os.path.dirname(__file__), "fixtures")


def test_gpu_fit_matches_cpu_fit(cuda_device):
    x = S.csv(os.path.join(FIX, "car-sensor-data.csv")).collect().x[:3200]
    res = {}
    for dev in ("cpu", cuda_device):
        m = Autoencoder(device=dev, input_normalizer="cardata", seed=4)
        m.compile()
        h = m.fit(x, epochs=2, batch_size=32, verbose=0, shuffle=False)
        res[str(dev)] = (h.history["loss"], m.get_weights())
    (lc, wc), (lg, wg) = res["cpu"], res[str(cuda_device)]
    assert abs(lc[-1] - lg[-1]) / lc[-1] < 0.05, (lc, lg)
    assert np.median(np.abs(np.concatenate([(a - b).ravel() for a, b in zip(wc, wg)]))) < 2e-3


def test_gpu_stream_fit_through_pinned_ring(cuda_device, tmp_path):
    st = S.synthetic(200_000, chunk=50_000, seed=2, failure_rate=0.0)
    m = Autoencoder(device=cuda_device, input_normalizer="cardata")
    m.compile()
    h = m.fit(st, epochs=2, batch_size=16384, verbose=0)
    assert h.history["loss"][1] < h.history["loss"][0]
    assert m.iterations == 2 * (200_000 // 16384 + 1)
    p = str(tmp_path / "m.h5")
    m.save(p)
    m2 = load_model(p, device=cuda_device, input_normalizer="cardata")
    xs = st.collect().x[:1000]
    np.testing.assert_allclose(m.score(xs), m2.score(xs), rtol=1e-6)


def test_reference_model_on_gpu(cuda_device):
    m = load_model(os.path.join(FIX, "autoencoder_sensor_anomaly_detection.h5"), device=cuda_device)
    mc = load_model(os.path.join(FIX, "autoencoder_sensor_anomaly_detection.h5"), device="cpu")
    x = np.random.default_rng(0).standard_normal((4096, 30)).astype(np.float32)
    np.testing.assert_allclose(m.score(x), mc.score(x), rtol=3e-2, atol=3e-3)
