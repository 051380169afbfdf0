"""Reference-compatible CLIs (C18): arity/usage, in-process runs, and a multi-process
broker -> train -> model store -> predict -> result-topic pipeline over TCP + SASL PLAIN."""
import os
import subprocess
import sys
import time

import numpy as np
import pytest

from streamml.cli.__main__ import main as cli

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_usage_errors(capsys):
    assert cli(["cardata-v3", "a", "b"]) == 1
    assert "<servers> <topic> <offset> <result_topic> <mode> <model-file> <project>" in capsys.readouterr().out
    assert cli(["lstm-v2", "a", "b", "c", "d", "e"]) == 1
    assert cli(["cardata-v1", "a"]) == 1
    assert cli(["cardata-v3", "s", "t", "0", "r", "bogus", "m.h5", "p"]) == 1
    assert "Mode is invalid" in capsys.readouterr().out
    assert cli(["no-such-command"]) == 1


def test_cardata_v3_inprocess(tmp_path, monkeypatch):
    from streamml.kafka import fake_broker
    monkeypatch.setenv("SML_MODEL_STORE", str(tmp_path / "store"))
    base = ["synthetic://21000", "CARS", "0", "preds"]
    common = ["--device", "cpu", "--workdir", str(tmp_path)]
    assert cli(["cardata-v3", *base, "train", "m1.h5", "proj", "--epochs", "2", *common]) == 0
    assert (tmp_path / "store" / "tf-models_proj" / "m1.h5").exists()
    os.unlink(tmp_path / "m1.h5")          # predict must fetch it from the store
    assert cli(["cardata-v3", *base, "predict", "m1.h5", "proj", *common]) == 0
    b = fake_broker("synthetic-CARS")
    assert b.end_offset("preds", 0) == 100 * 100        # batch(100).skip(100).take(100)
    rec = b.read("preds", 0, 0, 1)
    msg = rec[0][2]                                      # (offset, key, value)
    assert msg.startswith(b"[") and msg.endswith(b"]")   # np.array2string row


def test_precision_flag_reaches_the_small_batch_trainer(tmp_path, monkeypatch):
    """``--precision bf16`` on the AE CLIs selects compile(minibatch_precision="bf16") (the
    small-batch trainer's bf16 contractions); the default stays Keras-exact fp32 (None)."""
    from streamml.models.autoencoder import Autoencoder
    seen = []
    orig = Autoencoder.compile

    def spy(self, *a, **kw):
        seen.append(kw.get("minibatch_precision"))
        return orig(self, *a, **kw)

    monkeypatch.setattr(Autoencoder, "compile", spy)
    monkeypatch.setenv("SML_MODEL_STORE", str(tmp_path / "store"))
    base = ["synthetic://12000", "CARSP", "0", "predsp"]
    common = ["--device", "cpu", "--workdir", str(tmp_path), "--epochs", "1", "--take", "10"]
    assert cli(["cardata-v3", *base, "train", "mp.h5", "proj", "--precision", "bf16", *common]) == 0
    assert cli(["cardata-v3", *base, "train", "mq.h5", "proj", *common]) == 0
    assert cli(["creditcard", "--device", "cpu", "--rows", "4000", "--epochs", "1", "--precision", "bf16"]) == 0
    assert seen == ["bf16", None, "bf16"]


def test_lstm_v2_and_v1_inprocess(tmp_path, monkeypatch):
    monkeypatch.setenv("SML_MODEL_STORE", str(tmp_path / "store"))
    base = ["synthetic://2500", "LSTMCARS", "0", "lstm-out"]
    common = ["--device", "cpu", "--workdir", str(tmp_path), "--epochs", "1", "--take", "50"]
    assert cli(["lstm-v2", *base, "train", "lstm.h5", *common]) == 0
    assert (tmp_path / "store" / "car-demo-tensorflow-models" / "lstm.h5").exists()
    assert cli(["lstm-v2", *base, "predict", "lstm.h5", *common]) == 0
    assert cli(["lstm-v1", "synthetic://1500", "LSTM1", "0", "lstm1-out", *common]) == 0


def test_creditcard_and_mnist_inprocess(capsys):
    assert cli(["creditcard", "--device", "cpu", "--rows", "8000", "--epochs", "1", "--evaluate"]) == 0
    out = capsys.readouterr().out
    assert '"roc_auc"' in out
    assert cli(["mnist", "--device", "cpu", "--epochs", "1", "--steps-per-epoch", "300", "--rows", "1200"]) == 0
    assert cli(["mnist", "--device", "cpu", "--epochs", "1", "--rows", "600", "--simplified"]) == 0


def _start_broker(extra):
    env = dict(os.environ, PYTHONPATH=REPO)
    p = subprocess.Popen([sys.executable, "-m", "streamml.cli", "broker", "--port", "0", *extra],
                         stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True, env=env)
    addr = None
    t0 = time.time()
    while time.time() - t0 < 120:
        line = p.stdout.readline()
        if not line:
            break
        if line.startswith("listening "):
            addr = line.split()[1]
            break
    if addr is None:
        p.kill()
        raise RuntimeError("broker did not start")
    return p, addr


@pytest.mark.slow
def test_multiprocess_pipeline_over_tcp_with_sasl(tmp_path):
    broker, addr = _start_broker(["--sasl", "test:test123", "--preload", "SENSOR_DATA_S_AVRO=20500"])
    try:
        env = dict(os.environ, PYTHONPATH=REPO, SML_MODEL_STORE=str(tmp_path / "store"))
        args = [addr, "SENSOR_DATA_S_AVRO", "0", "model-predictions"]
        common = ["--device", "cpu", "--workdir", str(tmp_path / "job"), "--epochs", "1"]
        for mode in ("train", "predict"):
            r = subprocess.run([sys.executable, "-m", "streamml.cli", "cardata-v3", *args, mode, "model1.h5",
                                "demo", *common], env=env, capture_output=True, text=True, timeout=600)
            assert r.returncode == 0, r.stdout + r.stderr
        from streamml.config import REFERENCE_KAFKA_CONFIG
        from streamml.kafka import KafkaClient
        c = KafkaClient(addr, REFERENCE_KAFKA_CONFIG)
        assert c.latest("model-predictions", 0) == 10000
        # wrong credentials are rejected
        with pytest.raises(Exception):
            KafkaClient(addr, [*REFERENCE_KAFKA_CONFIG[:3], "sasl.password=nope", "sasl.mechanisms=PLAIN"]).latest(
                "model-predictions", 0)
    finally:
        broker.terminate()
        broker.wait(timeout=30)


@pytest.mark.gpu
def test_lstm_v2_train_on_gpu_uses_persistent_trainer(tmp_path, monkeypatch, capsys, cuda_device):
    """cardata-v2's job on the GPU: device window views -> LSTMPredictor.fit -> the persistent
    reference-stack kernel (look_back 1, batch 1); the two-layer stack trains on the fused
    kernels with in-place windows; mnist trains on the mlp.hip GEMMs."""
    from streamml.models import lstm as lstm_mod
    engines = []
    orig = lstm_mod.LSTMPredictor.fit

    def spy(self, *a, **kw):
        h = orig(self, *a, **kw)
        engines.append(self.last_fit_engine)
        return h
    monkeypatch.setattr(lstm_mod.LSTMPredictor, "fit", spy)
    monkeypatch.setenv("SML_MODEL_STORE", str(tmp_path / "store"))
    base = ["synthetic://2500", "LSTMGPU", "0", "lstm-gpu-out"]
    common = ["--device", str(cuda_device), "--workdir", str(tmp_path), "--epochs", "2", "--take", "200"]
    assert cli(["lstm-v2", *base, "train", "lstm.h5", *common]) == 0
    assert engines == ["persistent"]
    assert cli(["lstm-v2", *base, "predict", "lstm.h5", *common]) == 0
    assert cli(["mnist", "--device", str(cuda_device), "--epochs", "1", "--steps-per-epoch", "100",
                "--rows", "1200"]) == 0
