"""Persistent per-event scorer (ae_serve.hip) vs the fused forward kernel and the torch fp32 reference."""
import time

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _model(dev, normalizer="cardata"):
    from streamml.models.autoencoder import Autoencoder
    m = Autoencoder(device=dev, seed=4, input_normalizer=normalizer)
    m.compile()
    return m


def test_scores_match_reference(cuda_device):
    from streamml.data.cardata import SyntheticCarSource, normalize_np
    from streamml.models.reference import ae_forward_torch
    from streamml.ops.serve import ScoringServer
    m = _model(cuda_device)
    raw, _, _, _ = SyntheticCarSource.scenario("full", seed=2).generate(500)
    xn = torch.as_tensor(normalize_np(raw), dtype=torch.float32)
    w = [torch.as_tensor(a) for a in m.get_weights()]
    y, _ = ae_forward_torch(xn, w, list(m.spec.activations))
    ref = ((y - xn) ** 2).mean(1).numpy()
    with ScoringServer(m, threshold=0.05, slots=256, idle_seconds=0.5) as srv:
        s, f = srv.score(raw[:1])
        np.testing.assert_allclose(s, ref[:1], rtol=1e-4, atol=1e-6)
        s, f, r = srv.infer(raw)           # 500 rows > 256 slots: chunked + back-pressure
        np.testing.assert_allclose(s, ref, rtol=1e-4, atol=1e-6)
        np.testing.assert_array_equal(f, ref > 0.05)
        np.testing.assert_allclose(r, y.numpy(), rtol=1e-4, atol=1e-5)
        # idle exit + transparent relaunch
        time.sleep(1.2)
        s2, _ = srv.score(raw[:64])
        np.testing.assert_allclose(s2, ref[:64], rtol=1e-4, atol=1e-6)
        assert srv.launches >= 2
        lat = srv.latency_us(raw[:200], qps=20000)
        assert lat.shape == (200,) and np.all(lat > 0)


def test_matches_fused_forward_kernel(cuda_device):
    from streamml.ops.serve import ScoringServer
    m = _model(cuda_device, normalizer=None)
    x = np.random.default_rng(0).uniform(-1, 1, (300, 18)).astype(np.float32)
    fused = m.score(x)
    with ScoringServer(m, slots=1024) as srv:
        s, _ = srv.score(x)
    # the fused kernel computes in bf16 MFMA, the server in fp32 VALU
    np.testing.assert_allclose(s, fused, rtol=3e-2, atol=1e-4)
