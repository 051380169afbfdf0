"""Batch boundaries of the throughput engine's single-pass paths, on CPU with a recording
backend (the GPU numerics are pinned in tests/test_fit_throughput_gpu.py).

``Autoencoder._fit_stream_throughput`` trains a batch that lies inside one device chunk in
place and assembles only a batch straddling chunks in a carry buffer; the sequence of
batches must be exactly ``batch(B)`` over the concatenated stream, capped by ``take`` and
ending with Keras' short batch.  ``_fit_array_throughput`` trains single-pass epochs in
place (no pack) and packs once when the rows will be replayed (PACK_MIN_PASSES)."""
import numpy as np
import pytest
import torch

from streamml.models.autoencoder import Autoencoder


class Recorder:
    """Stands in for FusedAE: records what each call trained."""

    def __init__(self):
        self.steps, self.packs, self.ring_steps = [], 0, 0
        self.ring_xpack = None
        self.cursor = torch.zeros(1, dtype=torch.int64)

    def step(self, x, global_batch=None, allreduce=None):
        self.steps.append(x.clone())

    def pack_ring(self, x, batch, **kw):
        self.packs += 1
        self.ring_xpack = object()

    def step_ring(self, global_batch=None, allreduce=None):
        self.ring_steps += 1


def _model(monkeypatch, chunks):
    m = Autoencoder(device="cpu")
    rec = Recorder()
    monkeypatch.setattr(Autoencoder, "backend", property(lambda self: rec))
    monkeypatch.setattr(m, "_stream_device_chunks", lambda stream: iter(chunks))
    return m, rec


@pytest.mark.parametrize("sizes,B,take", [([37, 1000, 5, 333, 100], 100, None), ([250, 250], 100, None),
                                          ([7] * 50, 32, None), ([1000, 1000], 128, 9), ([64, 64, 64], 64, None),
                                          ([10], 100, None)])
def test_stream_batches_are_batch_B_over_the_stream(monkeypatch, sizes, B, take):
    rows = torch.arange(sum(sizes) * 18, dtype=torch.float32).reshape(-1, 18)
    chunks, i = [], 0
    for n in sizes:
        chunks.append(rows[i:i + n])
        i += n
    m, rec = _model(monkeypatch, chunks)
    steps = m._fit_stream_throughput(None, B, take, 1, None, 0, 0)
    want = [rows[j:j + B] for j in range(0, rows.size(0), B)]
    if take is not None:
        want = want[:take]
    assert steps == len(want) == len(rec.steps)
    for got, w in zip(rec.steps, want):
        assert torch.equal(got, w)
    assert rec.packs == 0   # single-pass rows are never packed


def test_array_fit_packs_only_replayed_rows(monkeypatch):
    m, rec = _model(monkeypatch, [])
    x = torch.randn(1000, 18)
    # one epoch left: in place
    m._fit_array_throughput(x, 100, None, False, 0, 0, 0, 1, None, 0, epochs_left=1)
    assert rec.packs == 0 and len(rec.steps) == 10 and rec.ring_steps == 0
    # three or more epochs left: pack once, then reuse it
    m._fit_array_throughput(x, 100, None, False, 0, 0, 0, 1, None, 0, epochs_left=Autoencoder.PACK_MIN_PASSES)
    m._fit_array_throughput(x, 100, None, False, 0, 0, 1, 1, None, 0, epochs_left=Autoencoder.PACK_MIN_PASSES - 1)
    assert rec.packs == 1 and rec.ring_steps == 20
