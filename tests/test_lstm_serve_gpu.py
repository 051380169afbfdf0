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


@pytest.mark.parametrize("T", [1, 3])
def test_cli_predict_engines_return_the_same_shape(cuda_device, T):
    """``--predict-engine auto`` picks the persistent forecaster only for one-step-output
    stacks, and both engines return model.predict's shape."""
    import types

    from streamml.cli.cardata_lstm import _predict
    m = LSTMPredictor.reference(look_back=T, device=cuda_device, seed=2)
    rows = np.random.default_rng(5).uniform(-1, 1, size=(200, 18)).astype(np.float32)
    outs = {}
    for eng in ("auto", "batch", "persistent"):
        ns = types.SimpleNamespace(look_back=T, skip=2, batch_size=10, predict_take=5, predict_engine=eng)
        outs[eng] = _predict(ns, None, None, rows, m, None)
    assert outs["auto"].shape == outs["batch"].shape
    if T == 1:
        assert outs["persistent"].shape == outs["batch"].shape == (50, 1, 18)
        np.testing.assert_allclose(outs["persistent"], outs["batch"], rtol=0, atol=3e-2)


def test_lstm_predict_keeps_device_input_on_device(cuda_device):
    m = LSTMPredictor.two_layer(look_back=4, device=cuda_device, seed=1)
    x = torch.rand(300, 4, 18, device=cuda_device)
    out = m.predict(x, batch_size=128)
    assert isinstance(out, torch.Tensor) and out.device == x.device
    np.testing.assert_allclose(out.cpu().numpy(), m.predict(x.cpu().numpy(), batch_size=128), rtol=0, atol=1e-5)


@pytest.mark.parametrize("stack,T", [("reference", 1), ("two_layer", 5)])
def test_lstm_kafka_low_latency_path_matches_oracle(cuda_device, stack, T):
    """``serve --model lstm --low-latency``'s path: Kafka (several cars interleaved over two
    partitions) -> C++ loop (car key -> device slot) -> persistent forecaster -> result
    records.  Every record's forecast (``reconstruction``) and score are checked against the
    float64 oracle of that car's own window."""
    import json

    from streamml.data.avro import AvroCodec
    from streamml.data.produce import encode_chunk
    from streamml.kafka import KafkaClient, fake_broker
    from streamml.kafka.scoreloop import LowLatencyScorer
    from streamml.ops.serve import LSTMScoringServer

    ctor = LSTMPredictor.two_layer if stack == "two_layer" else LSTMPredictor.reference
    m = ctor(look_back=T, device=cuda_device, seed=6)
    rng = np.random.default_rng(11 + T)
    n, ncar = 240, 6
    raw = rng.uniform(0, 40, size=(n, 18)).astype(np.float32)
    from streamml.data.cardata import FEATURES, INT_FEATURES
    for j, f in enumerate(FEATURES):   # the Avro schema's int fields carry whole numbers
        if f in INT_FEATURES:
            raw[:, j] = np.round(raw[:, j])
    cars = [f"vehicles/sensor/data/electric-vehicle-{int(c):05d}" for c in rng.integers(0, ncar, size=n)]
    part = np.array([hash(c) % 2 for c in cars])        # a car's events stay in one partition
    name = f"lstm-ll-{stack}-{T}"
    b = fake_broker(name)
    b.create_topic("S", 2)
    b.create_topic("R", 2)
    codec = AvroCodec("cardata-v1")
    cli = KafkaClient(f"fake://{name}")
    idx = {p: np.nonzero(part == p)[0] for p in (0, 1)}
    for p in (0, 1):
        buf, offs = encode_chunk(codec, raw[idx[p]].astype(np.float64), np.zeros(len(idx[p]), np.uint8))
        cli.produce("S", p, [bytes(buf[offs[i]:offs[i + 1]]) for i in range(len(idx[p]))],
                    keys=[cars[i].encode() for i in idx[p]])
    thr = 0.05
    with LSTMScoringServer(m, nkeys=16, threshold=thr) as srv:
        loop = LowLatencyScorer(f"fake://{name}", "S", "R", [0, 1], srv, starts=[0, 0], emit_recon=True,
                                max_wait_ms=5, max_batch=32)
        st = loop.run(idle_timeout_s=0.3)
    assert st["events"] == n and st["keys"] == len(set(cars))
    sc, sh = normalize_affine()
    xn = (raw.astype(np.float64) * np.float32(sc) + np.float32(sh)).astype(np.float32)
    checked = 0
    for p in (0, 1):
        recs = [json.loads(r[2]) for r in b.read("R", p, 0)]
        assert [r["offset"] for r in recs] == list(range(len(idx[p])))
        hist, last = {}, {}
        for r, i in zip(recs, idx[p]):
            c = cars[i]
            assert r["car"] == c
            h = hist.setdefault(c, [])
            if len(h) >= T:
                want = float(np.mean((xn[i].astype(np.float64) - last[c]) ** 2))
                assert abs(r["score"] - want) <= 2e-3 * max(want, 1e-3) + 1e-6, (r, want)
                assert r["anomaly"] == (want > thr) or abs(want - thr) < 1e-5
            else:
                assert np.isnan(r["score"]) and r["anomaly"] is False
            h.append(xn[i])
            got = np.array(r["reconstruction"].strip("[]").split(), dtype=np.float64)
            if len(h) >= T:
                f = _forward(m, np.stack(h[-T:]))
                assert np.all(np.abs(got - f) <= 2e-4 * np.abs(f) + 1e-4), (i, got, f)
                last[c] = got   # the printed forecast (8 significant digits) is the next score's reference
                checked += 1
            else:
                assert not got.any()
    assert checked >= n - ncar * T


@pytest.mark.parametrize("stack,T", [
    ([("lstm", 32, True, "relu"), ("lstm", 16, False, "relu"), ("dense", 18, False)], 50),   # config 3
    ([("lstm", 32, True, "tanh"), ("lstm", 24, True, "tanh"), ("lstm", 16, False, "tanh"), ("dense", 18, False)], 20),
    ([("lstm", 20, True, "tanh"), ("lstm", 32, True, "tanh"), ("dense", 18, False)], 7),   # TimeDistributed head
    ([("lstm", 8, False, "relu"), ("dense", 18, False)], 64),
])
def test_pipelined_stack_kernel_matches_general_kernel(cuda_device, monkeypatch, stack, T):
    """LSTM stacks under one Dense head run on the pipelined variant (one wave per layer,
    step counters in LDS instead of barriers); SML_LSTM_SERVE_GENERIC=1 forces the
    barrier-per-step kernel.  Same forecasts / scores / flags on an interleaved stream."""
    from streamml.ops.serve import LSTMScoringServer
    m = LSTMPredictor(look_back=T, stack=stack, device=cuda_device, seed=13)
    rng = np.random.default_rng(T)
    nkeys = 3
    n = (T + 10) * nkeys
    keys = rng.integers(0, nkeys, size=n)
    raw = rng.uniform(0, 40, size=(n, 18)).astype(np.float32)
    out = {}
    for generic in ("0", "1"):
        monkeypatch.setenv("SML_LSTM_SERVE_GENERIC", generic)
        with LSTMScoringServer(m, nkeys=nkeys, threshold=0.05) as srv:
            out[generic] = srv.forecast(raw, keys)
    (pa, sa, fa), (pb, sb, fb) = out["0"], out["1"]
    assert np.abs(pb).max() > 0
    scale = max(np.abs(pb).max(), 1.0)
    # fp32 with different summation orders: a 50-step random relu stack grows to |h| ~ 1e2..1e3
    # and amplifies rounding chaotically (see test_lstm_serve_matches_oracle), so relu stacks
    # get 0.5 % of the largest output; a wrong window, key or state is off by O(|f|)
    relu = any(layer[0] == "lstm" and layer[3] == "relu" for layer in stack)
    np.testing.assert_allclose(pa, pb, rtol=2e-4, atol=(5e-3 if relu else 2e-5) * scale)
    np.testing.assert_allclose(sa, sb, rtol=2e-2 if relu else 1e-3, atol=1e-6, equal_nan=True)
    agree = (fa == fb) | (np.abs(sa - 0.05) < (2e-2 if relu else 1e-3))
    assert agree.all()
