"""``Autoencoder.fit(engine="throughput")``: the large-batch mode on the headline kernel.

A shuffled epoch's rows are tile-packed (K8, the shuffle fused into the pack) and every
full batch runs the packed-pair bf16 MFMA train kernel + slab-reduce/Adam
(``FusedAE.step_ring``); unshuffled rows are packed once when they will be replayed
(>= Autoencoder.PACK_MIN_PASSES epochs) and otherwise trained in place by the direct fused
step; Keras' short last batch runs the plain fused step.  The oracle is
``tests/helpers/bf16_ref.py`` -- gradients with the kernels' bf16 rounding points, Keras
Adam (eps 1e-7) in float64 -- so the whole epoch's parameter trajectory is checked at
1e-3 relative (reference job: AUTOENCODER-TensorFlow-IO-Kafka/cardata-v3.py:212-222)."""
import math

import numpy as np
import pytest
import torch

from streamml.data import stream as S
from streamml.data.cardata import normalize_affine
from streamml.models.autoencoder import Autoencoder

pytestmark = pytest.mark.gpu


def _adam_oracle(w0, xn, batches, lr=1e-3, b1=0.9, b2=0.999, eps=1e-7):
    """Keras Adam over the given row-index batches of the normalised rows xn (float64)."""
    from helpers.bf16_ref import ae_bf16_reference
    w = [torch.as_tensor(a).double() for a in w0]
    m = [torch.zeros_like(a) for a in w]
    v = [torch.zeros_like(a) for a in w]
    sq = ab = rows = 0.0
    for t, idx in enumerate(batches, start=1):
        g, (s, a) = ae_bf16_reference(torch.from_numpy(xn[idx]), [x.float().numpy() for x in w])
        sq, ab, rows = sq + s, ab + a, rows + len(idx)
        lr_t = lr * math.sqrt(1 - b2 ** t) / (1 - b1 ** t)
        for i in range(len(w)):
            gi = torch.as_tensor(g[i]).double()
            m[i] = b1 * m[i] + (1 - b1) * gi
            v[i] = b2 * v[i] + (1 - b2) * gi * gi
            w[i] = w[i] - lr_t * m[i] / (v[i].sqrt() + eps)
    return [a.numpy() for a in w], (sq / 18 + 1e-7 * ab) / rows


def _relerr(got, want):
    a = np.concatenate([np.ravel(x) for x in got]).astype(np.float64)
    b = np.concatenate([np.ravel(x) for x in want]).astype(np.float64)
    return float(np.linalg.norm(a - b) / np.linalg.norm(b))


def _data(n, seed):
    raw = np.random.default_rng(seed).uniform(0, 40, size=(n, 18)).astype(np.float32)
    sc, sh = normalize_affine()
    xn = (raw.astype(np.float64) * np.float32(sc) + np.float32(sh)).astype(np.float32)   # = the kernels' fmaf
    return raw, xn


@pytest.mark.parametrize("shuffle", [False, True])
def test_fit_throughput_epoch_vs_bf16_reference(cuda_device, shuffle):
    B, n = 4096, 4096 * 6 + 1000      # 6 packed batches + Keras' short last batch
    raw, xn = _data(n, 3)
    m = Autoencoder(device=cuda_device, input_normalizer="cardata", seed=2)
    w0 = m.get_weights()
    m.compile()
    xd = torch.from_numpy(raw).to(cuda_device)
    h = m.fit(xd, epochs=1, batch_size=B, shuffle=shuffle, seed=9, verbose=0, engine="throughput")
    assert m.last_fit_engine == "throughput" and m.iterations == 7
    order = (m.backend.perm_indices(n, Autoencoder.shuffle_key(9, 0, 0)).cpu().numpy() if shuffle else np.arange(n))
    batches = [order[i:i + B] for i in range(0, n, B)]
    want, loss = _adam_oracle(w0, xn, batches)
    assert _relerr(m.get_weights(), want) < 1e-3
    assert abs(h.history["loss"][-1] - loss) <= 1e-3 * loss


def test_fit_throughput_reuses_pack_across_unshuffled_epochs(cuda_device):
    B, n = 2048, 2048 * 4
    raw, xn = _data(n, 4)
    m = Autoencoder(device=cuda_device, input_normalizer="cardata", seed=5)
    w0 = m.get_weights()
    m.compile()
    xd = torch.from_numpy(raw).to(cuda_device)
    m.fit(xd, epochs=3, batch_size=B, shuffle=False, verbose=0, engine="throughput")
    assert m.iterations == 12
    want, _ = _adam_oracle(w0, xn, [np.arange(i, i + B) for _ in range(3) for i in range(0, n, B)])
    assert _relerr(m.get_weights(), want) < 1e-3


def test_fit_throughput_stream_vs_bf16_reference(cuda_device):
    """A stream whose chunks straddle batches and pack rounds: batch(B) exactly."""
    B = 1024
    src = S.synthetic(1024 * 20 + 300, chunk=3001, seed=6)
    raw = np.concatenate([c.x for c in src])
    sc, sh = normalize_affine()
    xn = (raw.astype(np.float64) * np.float32(sc) + np.float32(sh)).astype(np.float32)
    m = Autoencoder(device=cuda_device, input_normalizer="cardata", seed=7)
    w0 = m.get_weights()
    m.compile()
    m.fit(src, epochs=1, batch_size=B, verbose=0, engine="throughput")
    n = len(raw)
    assert m.iterations == -(-n // B)
    want, _ = _adam_oracle(w0, xn, [np.arange(i, min(i + B, n)) for i in range(0, n, B)])
    assert _relerr(m.get_weights(), want) < 1e-3


def test_fit_auto_picks_throughput_for_large_batches(cuda_device):
    raw, _ = _data(4096, 8)
    m = Autoencoder(device=cuda_device, input_normalizer="cardata")
    m.compile()
    m.fit(raw, epochs=1, batch_size=1024, verbose=0)
    assert m.last_fit_engine == "throughput"
    m.fit(raw, epochs=1, batch_size=100, verbose=0)
    assert m.last_fit_engine == "persistent"


@pytest.mark.parametrize("n", [1, 2, 17, 4096, 1_000_003])
def test_pack_shuffle_is_a_bijection(cuda_device, n):
    """The in-kernel epoch shuffle (keyed Feistel bijection, cycle-walked into [0, n))."""
    m = Autoencoder(device=cuda_device, input_normalizer="cardata")
    m.compile()
    idx = m.backend.perm_indices(n, 12345).cpu().numpy()
    assert np.array_equal(np.sort(idx), np.arange(n))
    if n > 1000:   # and it actually shuffles: few fixed points, low correlation with the identity
        assert (idx == np.arange(n)).mean() < 0.01
        assert abs(np.corrcoef(idx, np.arange(n))[0, 1]) < 0.05
    other = m.backend.perm_indices(n, 54321).cpu().numpy()
    assert n < 17 or not np.array_equal(idx, other)


def test_pack_with_perm_key_equals_indexed_pack(cuda_device):
    from streamml.ops._ext import load_c
    C = load_c()
    raw, _ = _data(4096 + 37, 11)
    x = torch.from_numpy(raw).to(cuda_device)
    sc, sh = (torch.tensor(a, dtype=torch.float32, device=cuda_device) for a in normalize_affine())
    idx = C.perm_indices(x, x.size(0), 777, 0, 4096)
    a = C.pack_tiles_argmax(x, 18, sc, sh, idx, None)
    b = C.pack_tiles_argmax(x, 18, sc, sh, None, None, perm_key=777, perm_n=x.size(0), n_rows=4096)
    assert torch.equal(a, b)
    c = C.pack_tiles_argmax(x[idx].contiguous(), 18, sc, sh)
    assert torch.equal(a, c)


def test_fit_throughput_repacks_after_in_place_update(cuda_device):
    """Two unshuffled fits on the same device array with an in-place update between them:
    the second fit must train on the NEW rows (the pack key carries the version counter),
    not on the ring packed from the old ones."""
    B, n = 2048, 2048 * 4
    raw1, xn1 = _data(n, 21)
    raw2, xn2 = _data(n, 22)
    m = Autoencoder(device=cuda_device, input_normalizer="cardata", seed=5)
    w0 = m.get_weights()
    m.compile()
    xd = torch.from_numpy(raw1).to(cuda_device)
    m.fit(xd, epochs=3, batch_size=B, shuffle=False, verbose=0, engine="throughput")
    xd.copy_(torch.from_numpy(raw2))
    m.fit(xd, epochs=3, batch_size=B, shuffle=False, verbose=0, engine="throughput")
    b = [np.arange(i, i + B) for _ in range(3) for i in range(0, n, B)]
    # one Adam trajectory over both fits (the optimizer state carries across fit calls)
    xcat = np.concatenate([xn1, xn2])
    want, _ = _adam_oracle(w0, xcat, b + [x + n for x in b])
    assert _relerr(m.get_weights(), want) < 1e-3
