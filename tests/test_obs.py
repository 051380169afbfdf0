"""Observability: engine metrics wiring, Prometheus exposition + HTTP endpoint, rocprof helpers,
TensorBoard event round trip against the reference's own TF2 event files."""
import glob
import os
import urllib.request

import numpy as np
import pytest

from streamml.obs import profile as prof
from streamml.obs.metrics import ENGINE, REGISTRY

REF_LOGS = "/root/reference/python-scripts/autoencoder-anomaly-detection/logs"


def test_engine_metrics_wired_through_pipeline():
    from streamml.data import produce as prod
    from streamml.data import stream as st
    from streamml.kafka import KafkaOutputSequence, fake_broker
    from streamml.models.autoencoder import Autoencoder
    b0 = ENGINE.ingest_records.value(topic="obs-t")
    fake_broker("obs").create_topic("obs-t", 1)
    prod.produce(st.synthetic(3000, chunk=1000), "fake://obs", "obs-t", create=False)
    rows = st.kafka("fake://obs", ["obs-t:0:0"]).collect()
    assert len(rows) == 3000
    assert ENGINE.ingest_records.value(topic="obs-t") - b0 == 3000
    assert ENGINE.ingest_bytes.value(topic="obs-t") > 3000 * 50
    ae = Autoencoder(device="cpu", input_normalizer="cardata", name="obs-ae")
    ae.compile()
    t0 = ENGINE.train_rows.value(model="obs-ae")
    ae.fit(rows.x, epochs=1, batch_size=100, verbose=0)
    assert ENGINE.train_rows.value(model="obs-ae") - t0 == 3000
    assert ENGINE.train_steps.value(model="obs-ae") >= 30
    ae.detect(rows.x[:100], threshold=-1.0)
    assert ENGINE.anomaly_events.value(model="obs-ae") >= 100
    out = KafkaOutputSequence("obs-out", "fake://obs")
    for i in range(5):
        out.setitem(i, f"m{i}")
    out.flush()
    assert ENGINE.produced_records.value(topic="obs-out") >= 5
    text = REGISTRY.exposition()
    for name in ("ingest_records_total", "train_rows_total", "train_step_latency_us", "anomaly_events_total",
                 "h2d_bytes_total", "ring_buffer_occupancy"):
        assert name in text


def test_metrics_http_endpoint():
    srv = REGISTRY.serve(0)
    try:
        port = srv.server_address[1]
        body = urllib.request.urlopen(f"http://127.0.0.1:{port}/metrics", timeout=10).read().decode()
        assert "# TYPE ingest_records_total counter" in body
    finally:
        srv.shutdown()


def test_rocprof_command_rules(tmp_path):
    cmd = prof.rocprof_command(["python3", "bench.py", "--steps", "5"], str(tmp_path))
    assert cmd[:2] == ["rocprofv3", "--kernel-trace"] and "--stats" in cmd
    i = cmd.index("--")
    assert cmd[i + 1] == "python3"
    pmc = prof.rocprof_command(["python3", "bench.py"], str(tmp_path), pmc=prof.PMC_DEFAULT)
    assert "--pmc" in pmc and "--stats" not in pmc and "--sys-trace" not in pmc
    with pytest.raises(ValueError):
        prof.rocprof_command(["env", "A=1", "python3"], str(tmp_path))


def test_kernel_stats_markdown(tmp_path):
    p = tmp_path / "k.csv"
    p.write_text('"Name","Calls","TotalDurationNs","AverageNs","Percentage","MinNs","MaxNs","StdDev"\n'
                 '"void sml::(anonymous namespace)::wgrad_kernel<2, 8, float, float>(float const*, long)",24,'
                 '4118044,171585.1,24.18,1,2,3\n'
                 '"void (anonymous namespace)::lstm_bwd_kernel<32>((anonymous namespace)::LstmBwdArgs<32>)",12,'
                 '2550705,212558.7,14.98,1,2,3\n')
    rows = prof.load_kernel_stats(str(p))
    assert rows[0]["calls"] == 24 and abs(rows[0]["avg_us"] - 171.5851) < 1e-3
    md = prof.stats_markdown(rows)
    assert "`wgrad_kernel<2, 8, float, float>`" in md and "`lstm_bwd_kernel<32>`" in md


def test_device_timer_cpu_noop():
    t = prof.DeviceTimer()
    with t.section("x"):
        pass
    assert isinstance(t.summary(), dict)


@pytest.mark.skipif(not os.path.isdir(REF_LOGS), reason="reference logs not mounted")
def test_tensorboard_roundtrip_with_reference_tags(tmp_path):
    from streamml.nn.callbacks import TensorBoard
    from streamml.obs.tfevents import read_scalars
    ref = glob.glob(os.path.join(REF_LOGS, "train", "events.out.tfevents.*.v2"))
    ref_tags = set()
    for f in ref:
        ref_tags |= {t for _, _, t, _ in read_scalars(f)}
    tb = TensorBoard(str(tmp_path))
    for e in range(3):
        tb.on_epoch_end(e, {"loss": 1.0 / (e + 1), "accuracy": 0.5 + 0.1 * e, "val_loss": 0.9, "val_accuracy": 0.6})
    tb.on_train_end()
    ours = glob.glob(str(tmp_path / "train" / "events.out.tfevents.*"))
    assert ours
    got = read_scalars(ours[0])
    tags = {t for _, _, t, _ in got}
    assert {"epoch_loss", "epoch_accuracy"} <= tags
    if ref_tags:
        assert {"epoch_loss", "epoch_accuracy"} <= ref_tags
    vals = [v for _, _, t, v in got if t == "epoch_loss"]
    np.testing.assert_allclose(vals, [1.0, 0.5, 1.0 / 3], rtol=1e-6)


def test_grafana_dashboard_queries_exported_metrics():
    """Every panel of deploy/grafana/streamml.json queries a metric this package exports
    (engine metrics + the MQTT broker collector), and the committed copy is current."""
    import json
    from streamml.mqtt import MqttBroker
    from streamml.obs import dashboard, metrics
    with MqttBroker(port=0):
        text = metrics.REGISTRY.exposition()
    for name in dashboard.metric_names():
        assert f"# TYPE {name} " in text or f"\n{name} " in text or f"\n{name}{{" in text, name
    committed = json.load(open(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                            "deploy", "grafana", "streamml.json")))
    assert committed == dashboard.build()


def test_tensorboard_histograms_images_and_keras_summary(tmp_path):
    """TensorBoard(histogram_freq, write_images, write_graph) as TF2 writes them: per-weight
    histograms tagged 'dense/kernel_0', weight images, the 'keras' model-config tensor
    (plugin graph_keras_model, tensor before metadata as in the reference's own logs)."""
    import json
    import warnings

    from streamml.models.autoencoder import Autoencoder
    from streamml.nn.callbacks import TensorBoard
    from streamml.obs.tfevents import read_values
    m = Autoencoder(device="cpu", seed=1)
    m.compile()
    x = np.random.default_rng(0).uniform(-1, 1, (512, 18)).astype(np.float32)
    with warnings.catch_warnings():
        warnings.simplefilter("error")    # no profile_batch warning when it is 0
        tb = TensorBoard(str(tmp_path), histogram_freq=2, write_images=True, profile_batch=0)
    m.fit(x, epochs=3, batch_size=64, verbose=0, callbacks=[tb])
    f = glob.glob(str(tmp_path / "train" / "events.out.tfevents.*"))[0]
    vals = read_values(f)
    keras = [p for _, t, k, p in vals if t == "keras"]
    assert len(keras) == 1 and keras[0]["plugin"] == "graph_keras_model"
    cfg = json.loads(keras[0]["strings"][0])
    assert cfg["class_name"] == "Model" and [ly["name"] for ly in cfg["config"]["layers"]][1] == "dense"
    hist = {(s, t): p for s, t, k, p in vals if k == "histo"}
    assert {s for s, _ in hist} == {0, 2}                      # epochs 0 and 2 (freq 2)
    assert {t for _, t in hist} == {"dense/kernel_0", "dense/bias_0", "dense_1/kernel_0", "dense_1/bias_0",
                                    "dense_2/kernel_0", "dense_2/bias_0", "dense_3/kernel_0", "dense_3/bias_0"}
    w = m.get_weights()
    h = hist[(2, "dense/kernel_0")]
    assert h["num"] == w[0].size and sum(h["bucket"]) == w[0].size
    np.testing.assert_allclose([h["min"], h["max"], h["sum"]], [w[0].min(), w[0].max(), w[0].sum()], rtol=1e-5)
    imgs = {t: p for s, t, k, p in vals if k == "image" and s == 2}
    im = imgs["dense/kernel_0/image"]
    assert im["height"] == 18 and im["width"] == 14 and im["png"].startswith(b"\x89PNG")
    assert imgs["dense/bias_0/image"]["height"] == 1
    with pytest.raises(TypeError):
        TensorBoard(str(tmp_path), not_an_argument=1)
    with pytest.warns(UserWarning):
        TensorBoard(str(tmp_path), profile_batch=2)
