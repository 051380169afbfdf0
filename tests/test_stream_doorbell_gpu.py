"""Streaming epoch on ONE persistent-kernel launch (``FusedAE.train_stream``).

The kernel (``csrc/kernels/ae_minibatch.hip`` streaming mode) is launched before the
first chunk and takes its batches from a device ring as ``push`` lands them behind a
doorbell (``csrc/runtime/stream_ring.cpp``).  Batches straddle chunk boundaries inside
the ring, the ring wraps many times (a small ring forces back-pressure), and the last
``n % B`` rows are Keras' short final batch -- so the trajectory must be the one of
``train_rows`` over the concatenated rows (same kernel, same batches: bit-identical),
which ``tests/test_fit_persistent_gpu.py`` pins to the fp32 torch oracle.  Reference
job: AUTOENCODER-TensorFlow-IO-Kafka/cardata-v3.py:44-75 (stream) and :212-222 (fit).
"""
import numpy as np
import pytest
import torch

from streamml.data import stream as S
from streamml.models.autoencoder import Autoencoder

pytestmark = pytest.mark.gpu


def _pair(dev, seed=3):
    a = Autoencoder(device=dev, input_normalizer="cardata", seed=seed)
    b = Autoencoder(device=dev, input_normalizer="cardata", seed=seed)
    a.compile()
    b.compile()
    return a, b


def _chunks(x, sizes):
    out, i, k = [], 0, 0
    while i < x.size(0):
        n = sizes[k % len(sizes)]
        out.append(x[i:i + n])
        i += n
        k += 1
    return out


@pytest.mark.parametrize("B,n,ring", [(100, 100 * 57 + 41, 400), (32, 32 * 200, 64), (128, 128 * 33 + 127, 1 << 20)])
def test_train_stream_equals_train_rows(cuda_device, B, n, ring):
    raw = torch.from_numpy(np.random.default_rng(B).uniform(0, 40, size=(n, 18)).astype(np.float32)).to(cuda_device)
    a, b = _pair(cuda_device)
    steps, rows = a.backend.train_stream(_chunks(raw, [37, 1000, 5, 333, 100]), B, ring_rows=ring)
    s2, r2 = b.backend.train_rows(raw, B)
    assert (steps, rows) == (s2, r2) == (-(-n // B), n)
    for ga, gb in zip(a.get_weights(), b.get_weights()):
        np.testing.assert_array_equal(ga, gb)
    torch.testing.assert_close(a.backend.metrics, b.backend.metrics, rtol=0, atol=0)


def test_train_stream_take_and_strided_chunks(cuda_device):
    """``take(k)`` stops the kernel after k batches (no short batch); chunks may be
    column views of wider rows (row stride > features)."""
    B, k = 100, 40
    wide = torch.from_numpy(np.random.default_rng(1).uniform(0, 40, size=(9000, 20)).astype(np.float32)).to(cuda_device)
    raw = wide[:, :18]
    a, b = _pair(cuda_device, seed=8)
    steps, rows = a.backend.train_stream(_chunks(raw, [777, 1234]), B, max_steps=k, ring_rows=1000)
    s2, _ = b.backend.train_rows(raw.contiguous(), B, max_steps=k)
    assert steps == s2 == k and rows == k * B
    for ga, gb in zip(a.get_weights(), b.get_weights()):
        np.testing.assert_array_equal(ga, gb)


def test_train_stream_empty_and_short(cuda_device):
    a, b = _pair(cuda_device)
    assert a.backend.train_stream(iter(()), 100) == (0, 0)
    assert a.iterations == 0
    x = torch.from_numpy(np.random.default_rng(2).uniform(0, 40, size=(57, 18)).astype(np.float32)).to(cuda_device)
    assert a.backend.train_stream([x[:20], x[20:]], 100) == (1, 57)   # only the short batch
    b.backend.train_rows(x, 100)
    for ga, gb in zip(a.get_weights(), b.get_weights()):
        np.testing.assert_array_equal(ga, gb)


def test_fit_stream_doorbell_equals_chunk_launches(cuda_device, monkeypatch):
    """``fit`` on a stream: the one-launch doorbell epoch vs the launch-per-chunk path."""
    src = S.synthetic(40_000, chunk=6_001, seed=4, failure_rate=0.05)
    a, b = _pair(cuda_device, seed=6)
    a.fit(src.filter_normal(device=True), epochs=2, batch_size=100, verbose=0, engine="persistent")
    monkeypatch.setenv("SML_STREAM_DOORBELL", "0")
    b.fit(src.filter_normal(device=True), epochs=2, batch_size=100, verbose=0, engine="persistent")
    assert a.iterations == b.iterations > 0
    for ga, gb in zip(a.get_weights(), b.get_weights()):
        np.testing.assert_array_equal(ga, gb)
