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


def test_evaluate_forward_only_matches_train_kernel_metrics(cuda_device):
    """evaluate() runs the forward kernel with on-device metric sums (no backward); its loss
    and accuracy equal the train kernel's metric sums on the same rows (gradients(), which
    computes the same forward) and the fp32 torch oracle."""
    from streamml.models.reference import ae_loss_torch
    x = S.csv(os.path.join(FIX, "car-sensor-data.csv")).collect().x[:9000]
    m = Autoencoder(device=cuda_device, input_normalizer="cardata", seed=3)
    m.compile()
    loss, acc = m.evaluate(x, batch_size=4096)
    _, metr = m.backend.gradients(torch.from_numpy(np.ascontiguousarray(x, np.float32)).to(cuda_device))
    sq, ab, corr, rows = metr
    want_loss = (sq / 18 + 1e-7 * ab) / rows
    assert abs(loss - want_loss) <= 1e-5 * want_loss
    assert abs(acc - corr / rows) <= 2.0 / rows          # argmax near-ties may differ by a row
    mc = Autoencoder(device="cpu", input_normalizer="cardata", seed=3)
    mc.compile()
    lc, ac = mc.evaluate(x)
    assert abs(loss - lc) <= 2e-2 * lc                   # bf16 MFMA vs fp32 torch
    assert abs(acc - ac) <= 0.02


def test_predict_and_score_stay_on_device_until_the_end(cuda_device):
    """Device inputs: one forward pass per batch on the device, one copy back at the end;
    identical to per-batch host round trips."""
    rng = np.random.default_rng(5)
    x = rng.uniform(0, 40, size=(10_000, 18)).astype(np.float32)
    m = Autoencoder(device=cuda_device, input_normalizer="cardata", seed=1)
    m.compile()
    xd = torch.from_numpy(x).to(cuda_device)
    p_dev = m.predict(xd, batch_size=1000)
    p_host = m.predict(x, batch_size=1000)
    np.testing.assert_array_equal(p_dev, p_host)
    r, s = m.reconstruct_and_score(xd, batch_size=3000)
    np.testing.assert_array_equal(r, p_host)
    np.testing.assert_allclose(s, m.score(x), rtol=0, atol=0)
    seen = []

    class CB:
        def set_model(self, model):
            pass

        def on_predict_batch_end(self, b, logs):
            seen.append(logs["outputs"].shape)

        def on_predict_end(self):
            pass

    m.predict(xd, batch_size=4096, callbacks=[CB()])
    assert seen == [(4096, 18), (4096, 18), (1808, 18)]
