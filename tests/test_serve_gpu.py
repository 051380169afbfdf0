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


def test_scorer_accepts_32_features(cuda_device):
    """The AE scorer takes rows of up to 32 features (the LSTM forecaster's limit is 31: its
    request word 31 carries the key) -- the D = 32 boundary of ADVICE r03."""
    from streamml.models.autoencoder import Autoencoder
    from streamml.models.reference import ae_forward_torch
    from streamml.ops.serve import ScoringServer
    m = Autoencoder(input_dim=32, device=cuda_device, seed=1)   # weights only: no training backend
    x = np.random.default_rng(3).uniform(-1, 1, (100, 32)).astype(np.float32)
    y, _ = ae_forward_torch(torch.from_numpy(x), [torch.as_tensor(a) for a in m.get_weights()],
                            list(m.spec.activations))
    ref = ((y - torch.from_numpy(x)) ** 2).mean(1).numpy()
    with ScoringServer(m, slots=256) as srv:
        s, _ = srv.score(x)
    np.testing.assert_allclose(s, ref, rtol=1e-4, atol=1e-6)


def test_matches_fused_forward_kernel(cuda_device):
    from streamml.ops.serve import ScoringServer
    m = _model(cuda_device, normalizer=None)
    x = np.random.default_rng(0).uniform(-1, 1, (300, 18)).astype(np.float32)
    fused = m.score(x)
    with ScoringServer(m, slots=1024) as srv:
        s, _ = srv.score(x)
    # the fused kernel computes in bf16 MFMA, the server in fp32 VALU
    np.testing.assert_allclose(s, fused, rtol=3e-2, atol=1e-4)


def test_low_latency_loop_end_to_end(cuda_device):
    """serve --low-latency path: Kafka -> C++ decode -> persistent GPU scorer -> C++ JSON
    records -> Kafka.  Every record's score equals the scorer's own result for that row
    and the record text is byte-identical to the Python serve formatting."""
    import json
    import threading

    from streamml.data import stream as S
    from streamml.data.avro import AvroCodec
    from streamml.data.produce import encode_chunk
    from streamml.kafka import fake_broker
    from streamml.kafka.scoreloop import LowLatencyScorer, paced_produce
    from streamml.ops.serve import ScoringServer

    name = "gpu-lowlat"
    b = fake_broker(name)
    b.create_topic("SENSOR", 1)
    b.create_topic("RESULTS", 1)
    c = next(iter(S.synthetic(600, chunk=600, seed=5, failure_rate=0.05)))
    buf, offs = encode_chunk(AvroCodec("cardata-v1"), c.x, c.label)
    keys = [f"car{i % 17}" for i in range(600)]
    m = _model(cuda_device)
    with ScoringServer(m, threshold=0.5, slots=256) as srv:
        ref_s, ref_f, ref_r = srv.infer(c.x)
        loop = LowLatencyScorer(f"fake://{name}", "SENSOR", "RESULTS", [0], srv, starts=[0], emit_recon=True,
                                max_wait_ms=50, record_latency=True)
        out = {}
        th = threading.Thread(target=lambda: out.update(loop.run(max_events=600, idle_timeout_s=10.0)))
        th.start()
        sent = paced_produce(f"fake://{name}", "SENSOR", 0, bytes(buf), offs, keys=keys, qps=5000.0)
        th.join(60)
    assert not th.is_alive() and out["events"] == 600
    res = b.read("RESULTS", 0, 0)
    assert len(res) == 600
    for off, key, val in res:
        d = json.loads(val)
        i = d["offset"]
        assert key.decode() == keys[i] == d["car"]
        # the scorer's last-ulp rounding can depend on which slot / batch position an
        # event lands in, so values are compared to the reference call with a tolerance;
        # the C++ formatter itself is byte-checked against json / numpy in test_scoreloop.py
        np.testing.assert_allclose(np.float32(d["score"]), ref_s[i], rtol=1e-5)
        assert d["anomaly"] == bool(np.float32(d["score"]) > 0.5)
        rec = np.array(d["reconstruction"].strip("[]").split(), dtype=np.float32)
        np.testing.assert_allclose(rec, ref_r[i], rtol=1e-5, atol=1e-7)
        assert set(d) == {"car", "partition", "offset", "score", "anomaly", "reconstruction"}
    lat = loop.latency_records()
    d_us = (lat[np.argsort(lat[:, 1]), 2] - sent) / 1e3
    assert np.percentile(d_us, 50) < 2000
