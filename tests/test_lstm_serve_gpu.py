"""Persistent per-event LSTM scorer (csrc/kernels/lstm_serve.hip) vs a float64 torch oracle.

Events of several car keys arrive interleaved; per key the device keeps the last
``look_back`` normalised events and its latest forecast.  For every event the oracle
recomputes the key's window from scratch (Keras stateless LSTM semantics, gate order
i, f, c, o, sigmoid recurrent activation) and checks the forecast, the score against
the key's previous forecast and the flag (reference: LSTM-TensorFlow-IO-Kafka/
cardata-v2.py:220-273 streams one prediction per event)."""
import numpy as np
import pytest
import torch

from streamml.data.cardata import normalize_affine
from streamml.models.lstm import LSTMPredictor

pytestmark = pytest.mark.gpu


def _forward(model, window, dtype=torch.float64):
    """[T, F] normalised window -> forecast [F] (torch, CPU, ``dtype``)."""
    P = [torch.as_tensor(a).to(dtype) for a in model.fp.get()]
    h = torch.as_tensor(window).to(dtype)[None]
    for L in model.layers:
        if L["kind"] == "lstm":
            W, U, b = P[L["params"]:L["params"] + 3]
            u = L["units"]
            hh = torch.zeros(1, u, dtype=dtype)
            c = torch.zeros(1, u, dtype=dtype)
            act = torch.relu if L["activation"] == "relu" else torch.tanh
            outs = []
            for t in range(h.shape[1]):
                z = h[:, t] @ W + hh @ U + b
                i, f, g, o = z.split(u, dim=1)
                c = torch.sigmoid(f) * c + torch.sigmoid(i) * act(g)
                hh = torch.sigmoid(o) * act(c)
                outs.append(hh)
            h = torch.stack(outs, 1) if L["return_sequences"] else hh
        elif L["kind"] == "repeat":
            h = h[:, None].expand(1, L["n"], h.shape[-1])
        else:
            K, b = P[L["params"]:L["params"] + 2]
            h = h @ K + b
    return (h[0, -1] if h.dim() == 3 else h[0]).double().numpy()


@pytest.mark.parametrize("stack,T", [("two_layer", 5), ("reference", 1), ("two_layer", 50), ("reference", 3)])
def test_lstm_serve_matches_oracle(cuda_device, stack, T):
    from streamml.ops.serve import LSTMScoringServer
    ctor = LSTMPredictor.two_layer if stack == "two_layer" else LSTMPredictor.reference
    m = ctor(look_back=T, device=cuda_device, seed=4)
    rng = np.random.default_rng(T)
    nkeys = 7 if T < 10 else 2
    n = (T + 12) * nkeys + 5
    keys = rng.integers(0, nkeys, size=n)
    raw = rng.uniform(0, 40, size=(n, 18)).astype(np.float32)
    sc, sh = normalize_affine()
    xn = (raw.astype(np.float64) * np.float32(sc) + np.float32(sh)).astype(np.float32)
    thr = 0.05
    with LSTMScoringServer(m, nkeys=nkeys, threshold=thr) as srv:
        pred, score, flag = srv.forecast(raw, keys)
    hist = {k: [] for k in range(nkeys)}
    last = {}
    checked = 0
    for i in range(n):
        k = int(keys[i])
        cnt = len(hist[k])
        if cnt >= T:   # scored against the key's previous forecast (the kernel's own)
            want = float(np.mean((xn[i].astype(np.float64) - last[k]) ** 2))
            assert abs(score[i] - want) <= 2e-3 * max(want, 1e-3), (i, score[i], want)
            assert flag[i] == (1 if want > thr else 0) or abs(want - thr) < 1e-5
        else:
            assert flag[i] == 2 and np.isnan(score[i])
        hist[k].append(xn[i])
        if len(hist[k]) >= T:
            # the float64 oracle, with room for the window's own fp32 conditioning: a random
            # relu LSTM over 50 steps grows to |h| ~ 1e3 and plain fp32 torch already differs
            # from float64 by up to 2 % there, so for such a window the bound adds 8x its
            # largest fp32-vs-fp64 gap and 5e-4 of its largest output (rounding differences
            # are amplified chaotically; a wrong window, key or state is off by O(|f|))
            w = np.stack(hist[k][-T:])
            f = _forward(m, w)
            gap = np.abs(_forward(m, w, torch.float32) - f)
            err = np.abs(pred[i].astype(np.float64) - f)
            tol = 2e-4 * np.abs(f) + 2e-5 + 8 * gap.max() + (5e-4 * np.abs(f).max() if gap.max() > 1e-3 else 0.0)
            assert np.all(err <= tol), (i, float(err.max()), float(gap.max()))
            last[k] = pred[i].astype(np.float64)
            checked += 1
        else:
            assert not pred[i].any()
    assert checked >= 5 * nkeys


def test_lstm_serve_latency_and_reset(cuda_device):
    import time

    from streamml.ops.serve import LSTMScoringServer
    m = LSTMPredictor.two_layer(look_back=50, device=cuda_device)
    rng = np.random.default_rng(1)
    rows = rng.uniform(0, 40, size=(600, 18)).astype(np.float32)
    keys = np.zeros(600, np.int64)
    with LSTMScoringServer(m, nkeys=10, idle_seconds=5.0) as srv:
        lat = srv.latency_us(rows, keys, qps=20000)
        assert lat.shape == (600,) and np.all(lat > 0)
        t0 = time.perf_counter()
        srv.reset()             # stops the resident kernel first: no wait for its idle timeout
        assert time.perf_counter() - t0 < 1.0
        _, s, f = srv.forecast(rows[:3], keys[:3])
        assert np.all(f == 2)
        with pytest.raises(Exception):
            srv.forecast(rows[:1], np.array([10]))   # keys are validated on the host


@pytest.mark.parametrize("stack,T", [("reference", 1), ("two_layer", 8)])
def test_cli_persistent_predict_matches_window_predict(cuda_device, stack, T):
    """``cardata-lstm ... predict`` on ROCm streams the events through the forecaster; its
    forecasts for windows [skip, skip + take) equal model.predict on those windows (the
    batched path runs bf16 MFMA kernels, the forecaster fp32: bf16-level agreement)."""
    from streamml.cli.cardata_lstm import _predict_persistent, _windows
    ctor = LSTMPredictor.two_layer if stack == "two_layer" else LSTMPredictor.reference
    m = ctor(look_back=T, device=cuda_device, seed=2)
    rows = np.random.default_rng(3).uniform(-1, 1, size=(300, 18)).astype(np.float32)
    skip, take = 40, 100
    got = _predict_persistent(m, rows, skip, take)
    want = m.predict(_windows(rows, T)[skip:skip + take])
    want = want.reshape(len(want), -1, 18)[:, -1]
    assert got.shape == want.shape == (take, 18)
    np.testing.assert_allclose(got, want, rtol=0, atol=3e-2)


@pytest.mark.parametrize("act", ["relu", "tanh"])
def test_ref1_kernel_matches_general_kernel(cuda_device, monkeypatch, act):
    """The reference stack at look_back 1 runs on the one-wave register-resident kernel by
    default; SML_LSTM_SERVE_GENERIC=1 forces the general 4-wave kernel.  Both must give the
    same forecasts, scores and flags on the same interleaved event stream (fp32, different
    summation orders)."""
    from streamml.models.lstm import REFERENCE_STACK
    from streamml.ops.serve import LSTMScoringServer
    stack = [tuple(act if v == "relu" else v for v in layer) for layer in REFERENCE_STACK]
    m = LSTMPredictor(look_back=1, stack=stack, device=cuda_device, seed=11)
    rng = np.random.default_rng(5)
    n, nkeys = 400, 9
    keys = rng.integers(0, nkeys, size=n)
    raw = rng.uniform(0, 40, size=(n, 18)).astype(np.float32)
    out = {}
    for generic in ("0", "1"):
        monkeypatch.setenv("SML_LSTM_SERVE_GENERIC", generic)
        with LSTMScoringServer(m, nkeys=nkeys, threshold=0.05) as srv:
            out[generic] = srv.forecast(raw, keys)
    (pa, sa, fa), (pb, sb, fb) = out["0"], out["1"]
    np.testing.assert_allclose(pa, pb, rtol=1e-4, atol=1e-5)
    np.testing.assert_allclose(sa, sb, rtol=1e-4, atol=1e-6, equal_nan=True)
    agree = (fa == fb) | (np.abs(sa - 0.05) < 1e-4)   # a score within rounding of the threshold may flip
    assert agree.all()
