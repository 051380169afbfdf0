"""LSTM family: Keras semantics on CPU (torch reference) + persistence."""
import numpy as np
import torch

from streamml.data import stream as S
from streamml.models.lstm import LSTMPredictor
from streamml.ops.lstm import lstm_reference


def _np_lstm(x, W, U, b, act):
    B, T, _ = x.shape
    u = U.shape[0]
    h = np.zeros((B, u))
    c = np.zeros((B, u))
    f_act = (lambda z: np.maximum(z, 0)) if act == "relu" else np.tanh
    sig = lambda z: 1 / (1 + np.exp(-z))
    out = []
    for t in range(T):
        z = x[:, t] @ W + h @ U + b
        i, f, g, o = z[:, :u], z[:, u:2 * u], z[:, 2 * u:3 * u], z[:, 3 * u:]
        c = sig(f) * c + sig(i) * f_act(g)
        h = sig(o) * f_act(c)
        out.append(h)
    return np.stack(out, 1)


def test_reference_lstm_matches_numpy_keras_math():
    rng = np.random.default_rng(0)
    x = rng.standard_normal((3, 5, 18))
    W, U, b = rng.standard_normal((18, 64)) * 0.2, rng.standard_normal((16, 64)) * 0.2, rng.standard_normal(64) * 0.1
    for act in ("relu", "tanh"):
        got = lstm_reference(*(torch.tensor(a) for a in (x, W, U, b)), activation=act).numpy()
        np.testing.assert_allclose(got, _np_lstm(x, W, U, b, act), rtol=1e-10, atol=1e-12)


def test_param_counts():
    assert LSTMPredictor.reference(look_back=1, device="cpu").count_params() == 18642
    m = LSTMPredictor.two_layer(look_back=50, device="cpu")
    assert m.count_params() == (18 * 128 + 32 * 128 + 128) + (32 * 64 + 16 * 64 + 64) + (16 * 18 + 18)


def test_forget_bias_and_orthogonal_init():
    m = LSTMPredictor.reference(device="cpu")
    W, U, b = m.fp.get()[:3]
    assert (b[32:64] == 1).all() and (b[:32] == 0).all()
    np.testing.assert_allclose(U @ U.T, np.eye(32), atol=1e-5)


def test_cpu_training_reduces_loss_on_windows():
    x = S.synthetic(3000, chunk=1000, seed=0, failure_rate=0.0)
    m = LSTMPredictor.two_layer(look_back=8, device="cpu", seed=1)
    h = m.fit(x, epochs=3, batch_size=64, verbose=0, take=20)
    assert h.history["loss"][-1] < h.history["loss"][0]
    assert int(m.fp.iter.item()) == 60


def test_save_load_roundtrip(tmp_path):
    m = LSTMPredictor.reference(look_back=1, device="cpu")
    xs = np.random.default_rng(1).uniform(-1, 1, (40, 1, 18)).astype(np.float32)
    ys = np.random.default_rng(2).uniform(-1, 1, (40, 18)).astype(np.float32)
    m.fit(xs, ys, epochs=1, batch_size=1, verbose=0, take=10)    # reference: batch 1
    p = str(tmp_path / "lstm.h5")
    m.save(p)
    m2 = LSTMPredictor.load(p, device="cpu")
    assert [L["name"] for L in m2.layers] == ["lstm", "lstm_1", "repeat_vector", "lstm_2", "lstm_3",
                                              "time_distributed"]
    np.testing.assert_allclose(m.predict(xs), m2.predict(xs), rtol=1e-6)
    assert int(m2.fp.iter.item()) == 10
    from streamml.ckpt import load_keras_h5
    ck = load_keras_h5(p)
    assert [n for n, _ in ck.weights["lstm"]] == ["lstm/kernel:0", "lstm/recurrent_kernel:0", "lstm/bias:0"]
    assert ck.model_config["class_name"] == "Sequential"


def test_persistent_trainer_skips_exactly_the_zero_gradient_parameters():
    """look_back 1: U and the forget-gate columns get zero gradient; the persistent kernel
    carries the other 6 450 of the 18 642 parameters."""
    from streamml.ops import lstm_persistent as lp
    m = LSTMPredictor.reference(look_back=1, device="cpu", seed=0)
    assert m.count_params() == 18642
    assert int((~lp._inactive_mask(m))[:m.fp.n].sum()) == 6450
    assert not lp.supported(m)              # CPU model: the autograd path
    x = torch.randn(5, 1, 18)
    y = torch.randn(5, 18)
    m.train_step(x, y)
    g = m.fp.grad[lp._inactive_mask(m)]
    assert float(g.abs().max()) == 0.0
    assert lp.check_inactive(m)


def test_zero_padded_lstm_weights_are_exact():
    """ops.lstm.pad_lstm_weights: a u-unit layer padded to a kernel width gives the same h
    (the padded units stay exactly 0) and the same weight gradients (float64, CPU oracle)."""
    import numpy as np
    import torch

    from streamml.ops.lstm import lstm_reference, pad_lstm_weights, padded_units
    assert [padded_units(u) for u in (1, 16, 17, 50, 64, 65, 128, 129)] == [16, 16, 32, 64, 64, 128, 128, None]
    rng = np.random.default_rng(0)
    for u, act in ((20, "relu"), (50, "tanh"), (100, "tanh")):
        up = padded_units(u)
        x = torch.tensor(rng.uniform(-1, 1, (4, 6, 18)))
        W, U, b = (torch.tensor(rng.standard_normal(s) * 0.3, requires_grad=True)
                   for s in ((18, 4 * u), (u, 4 * u), (4 * u,)))
        h = lstm_reference(x, W, U, b, act)
        g = torch.tensor(rng.standard_normal(h.shape))
        gW, gU, gb = torch.autograd.grad((h * g).sum(), (W, U, b))
        hp = lstm_reference(x, *pad_lstm_weights(W, U, b, up), act)
        assert torch.equal(hp[..., u:], torch.zeros_like(hp[..., u:]))
        assert torch.allclose(hp[..., :u], h, rtol=0, atol=1e-12)
        pW, pU, pb = torch.autograd.grad((hp[..., :u] * g).sum(), (W, U, b))
        for a_, b_ in ((pW, gW), (pU, gU), (pb, gb)):
            assert torch.allclose(a_, b_, rtol=0, atol=1e-12)
