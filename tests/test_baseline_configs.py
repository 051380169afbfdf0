"""BASELINE.json configs 1-5 as end-to-end tests, each a
shrunken run of the same entry point the benchmark / CLI uses.

1. Dense AE on testdata/car-sensor-data.csv, CPU only, batch 32 (plumbing).
2. Dense AE bf16, synthetic car-sensor stream, 1x MI355X: ``bench.py``.
3. LSTM predictor seq_len 50, 2 layers, bf16: ``bench/bench_lstm.py``.
4. Dense AE DP: the same ``bench.py`` under torchrun. The multi-rank path runs in
   ``test_bench_dp_gpu.py`` (two ranks sharing GPU 0) and ``test_dp.py`` (gloo,
   CPU). This file checks that the DP JSON contract names the config's metric.
5. Streaming inference: load an .h5 autoencoder, score every event of a keyed
   stream per replica (shard-by-key). ``bench/bench_infer.py`` and the ``serve``
   CLI (``test_serve_cli.py``).
"""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BASELINE = json.load(open(os.path.join(ROOT, "BASELINE.json")))


def _json_line(stdout: str) -> dict:
    lines = [ln for ln in stdout.splitlines() if ln.startswith("{")]
    assert lines, stdout[-2000:]
    return json.loads(lines[-1])


def test_config1_cpu_autoencoder_on_reference_csv():
    """Config 1: the reference's own CSV fixture, CPU, batch 32; the loss goes down."""
    from streamml.data import stream as st
    from streamml.models.autoencoder import Autoencoder
    csv = os.path.join(ROOT, "tests", "fixtures", "car-sensor-data.csv")
    rows = st.csv(csv).filter_normal().take(40)     # reference trains on failure_occurred == "false" rows
    m = Autoencoder(device="cpu", seed=0)
    h = m.fit(rows, epochs=3, batch_size=32, verbose=0)
    losses = h.history["loss"]
    assert len(losses) == 3 and losses[-1] < losses[0]


@pytest.mark.gpu
def test_config2_bench_contract(cuda_device):
    r = subprocess.run([sys.executable, "bench.py", "--steps", "3", "--warmup", "1", "--batch-per-gpu", "1048576",
                        "--dataset-rows", "4194304", "--infer-events", "50"], cwd=ROOT, capture_output=True,
                       text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    out = _json_line(r.stdout)
    assert out["metric"] == BASELINE["metric"]
    assert out["n_gpus"] == 1 and out["steps"] == 3 and out["warmup"] == 1
    assert out["dtype"] == "bf16" and out["higher_is_better"] is True and out["scaling"] == "weak"
    assert out["value"] > 0 and out["ms_per_step"] > 0 and out["p50_infer_us"] > 0
    assert out["config"]["parallelism"] == "dp1"


@pytest.mark.gpu
def test_config3_lstm_bench(cuda_device):
    r = subprocess.run([sys.executable, "bench/bench_lstm.py", "--batch", "4096", "--steps", "2", "--warmup", "1"],
                       cwd=ROOT, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    out = _json_line(r.stdout)
    assert out["seq_len"] == 50 and out["dtype"] == "bf16" and out["value"] > 0
    assert np.isfinite(out["final_loss"])


def test_config4_dp_contract_names_the_metric():
    """Config 4's multi-rank run (driver: torchrun, N = 2/4/8) reports the same metric,
    whole-job value and dpN parallelism; the rank logic itself runs in
    test_bench_dp_gpu.py / test_dp.py."""
    src = open(os.path.join(ROOT, "bench.py")).read()
    assert '"parallelism": f"dp{' in src or "'parallelism': f'dp{" in src
    assert "WORLD_SIZE" in src or "init_from_env" in src


@pytest.mark.gpu
def test_config5_streaming_inference_from_h5(cuda_device, tmp_path):
    from streamml.models.autoencoder import Autoencoder, load_model
    from streamml.ops.serve import ScoringServer
    path = str(tmp_path / "model1.h5")
    Autoencoder(device="cpu", seed=2).save(path)
    m = load_model(path, device=str(cuda_device), input_normalizer="cardata")
    rng = np.random.default_rng(0)
    rows = rng.uniform(0, 40, (300, 18)).astype(np.float32)
    want = m.score(rows)
    srv = ScoringServer(m, device=cuda_device)
    try:
        got = np.array([srv.score(r[None])[0][0] for r in rows[:50]])   # fixed-QPS style: one event at a time
        burst, _ = srv.score(rows)                                       # backlog: many events in flight
        lat = srv.latency_us(rows[:100], qps=10000.0)
    finally:
        srv.close()
    assert np.median(lat) < 50.0
    np.testing.assert_allclose(got, want[:50], rtol=3e-2, atol=1e-3)
    np.testing.assert_allclose(burst, want, rtol=3e-2, atol=1e-3)
