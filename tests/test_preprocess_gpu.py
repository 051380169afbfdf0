"""K8 normalize_filter HIP kernel vs a numpy fp32 oracle (order-preserving compaction)."""
import numpy as np
import pytest
import torch

from streamml.data.cardata import normalize_affine
from streamml.ops.preprocess import normalize_filter, normalize_filter_reference

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("n,keep,frac", [(1, 0, 0.5), (4095, 0, 0.3), (4096, 0, 0.01), (100_003, 0, 0.5),
                                         (300_000, 1, 0.02), (70_000, -1, 0.5), (0, 0, 0.5)])
def test_normalize_filter_matches_numpy(cuda_device, n, keep, frac):
    rng = np.random.default_rng(n)
    x = (rng.uniform(0, 1, size=(n, 18)) * 100).astype(np.float32)
    labels = (rng.uniform(size=n) < frac).astype(np.uint8)     # 1 = failure_occurred "true"
    scale, shift = normalize_affine()
    got, idx = normalize_filter(torch.from_numpy(x).to(cuda_device), torch.from_numpy(labels), keep, scale, shift,
                                want_index=True)
    want, widx = normalize_filter_reference(x, labels, keep, scale, shift)
    assert got.shape == want.shape
    np.testing.assert_array_equal(idx.cpu().numpy(), widx)
    np.testing.assert_allclose(got.cpu().numpy(), want, rtol=1e-6, atol=1e-6)


def test_normalize_only_strided_rows(cuda_device):
    rng = np.random.default_rng(3)
    wide = rng.normal(size=(5000, 21)).astype(np.float32)
    x = torch.from_numpy(wide).to(cuda_device)[:, :18]
    got, _ = normalize_filter(x, None, -1, np.full(18, 2.0), np.full(18, -1.0))
    np.testing.assert_allclose(got.cpu().numpy(), wide[:, :18] * 2 - 1, rtol=1e-6, atol=1e-6)


def test_fit_with_device_filter_equals_host_filter(cuda_device):
    """filter(y == "false") -> batch(B) on the host vs K8 compaction + device re-batching:
    same batches in the same order, so the trained weights are bit-identical."""
    from streamml.data import stream as st
    from streamml.models.autoencoder import Autoencoder

    src = st.synthetic(5000, chunk=700, seed=4, failure_rate=0.3)
    weights = []
    for device_filter in (False, True):
        ae = Autoencoder(device=cuda_device, input_normalizer="cardata", seed=1)
        ae.compile()
        ae.fit(src.filter_normal(device=device_filter), epochs=2, batch_size=256, verbose=0)
        torch.cuda.synchronize()
        weights.append(ae.get_weights())
    for a, b in zip(*weights):
        np.testing.assert_array_equal(a, b)
