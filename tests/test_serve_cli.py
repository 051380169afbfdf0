"""``serve``: shard-by-key streaming scorer (BASELINE config 5 / the reference's
model-predictions Deployment) on the in-process broker: replicas split the partitions,
every event is scored exactly as ``Autoencoder.score`` scores it, results stay keyed and
ordered per partition, and committed offsets make a restarted replica resume."""
import json

import numpy as np
import pytest

from streamml.cli import serve as serve_cli
from streamml.cli.__main__ import main as cli_main


def test_shard_partitions_cover_each_partition_once():
    for world in (1, 2, 3, 8, 12):
        owned = [p for r in range(world) for p in serve_cli.shard_partitions(10, r, world)]
        assert sorted(owned) == list(range(10))


def _read_topic(servers, topic, parts):
    from streamml.kafka import KafkaClient
    c = KafkaClient(servers)
    out = {}
    for p in range(parts):
        pos, recs = 0, []
        while True:
            b = c.fetch(topic, p, pos, 1 << 22, 10)
            if len(b["offsets"]) == 0:
                break
            vals, vo = b["values"], b["value_offsets"]
            recs += [json.loads(vals[vo[i]:vo[i + 1]]) for i in range(len(vo) - 1)]
            pos = int(b["offsets"][-1]) + 1
        out[p] = recs
    return out


def test_parse_cpus_taskset_syntax():
    assert serve_cli.parse_cpus("4") == {4}
    assert serve_cli.parse_cpus("4-7, 12") == {4, 5, 6, 7, 12}
    for bad in ("", "7-4", "-1"):
        with pytest.raises(ValueError):
            serve_cli.parse_cpus(bad)


def test_serve_replicas_score_every_event_once(tmp_path, capsys):
    from streamml.data.stream import kafka
    from streamml.models.autoencoder import Autoencoder, load_model
    model_file = tmp_path / "model1.h5"
    Autoencoder(device="cpu", seed=3).save(str(model_file))
    n, parts = 3000, 4
    common = ["synthetic://%d" % n, "SENSOR_SERVE", "model-predictions-serve", "model1.h5",
              "--workdir", str(tmp_path), "--device", "cpu", "--synthetic-partitions", str(parts),
              "--idle-timeout", "0.3", "--replicas", "2"]
    summaries = []
    for r in (0, 1):
        assert cli_main(["serve"] + common + ["--replica-index", str(r)]) == 0
        summaries.append(json.loads(capsys.readouterr().out.strip().splitlines()[-1]))
    assert sorted(summaries[0]["partitions"] + summaries[1]["partitions"]) == list(range(parts))
    assert summaries[0]["events"] + summaries[1]["events"] == n

    servers = "fake://synthetic-SENSOR_SERVE"
    res = _read_topic(servers, "model-predictions-serve", parts)
    assert sum(len(v) for v in res.values()) == n
    model = load_model(str(model_file), device="cpu", input_normalizer="cardata")
    for p, recs in res.items():
        assert [r["offset"] for r in recs] == list(range(len(recs)))      # ordered, no gaps
        assert all(r["partition"] == p for r in recs)
        src = next(iter(kafka(servers, [f"SENSOR_SERVE:{p}:0"]).batch(1 << 20)))
        want = model.score(src.x)
        got = np.array([r["score"] for r in recs])
        np.testing.assert_allclose(got, want, rtol=1e-5, atol=1e-6)
        assert [r["car"] for r in recs] == list(src.keys)
        assert all(r["anomaly"] == (r["score"] > 5.0) for r in recs)

    # restart replica 0: committed offsets -> nothing left to score
    assert cli_main(["serve"] + common + ["--replica-index", "0"]) == 0
    again = json.loads(capsys.readouterr().out.strip().splitlines()[-1])
    assert again["events"] == 0


def test_serve_eight_replicas_ten_partitions_balanced(tmp_path, capsys):
    """BASELINE config 5 on the reference's topology (10 partitions) at 8 replicas: the key
    shares give every car to exactly one replica, every event is scored once, and the
    replicas' event counts are balanced (round-robin partitions would give 2:1)."""
    from streamml.models.autoencoder import Autoencoder
    model_file = tmp_path / "model1.h5"
    Autoencoder(device="cpu", seed=3).save(str(model_file))
    n, parts, W = 40000, 10, 8
    common = ["synthetic://%d" % n, "SENSOR_SERVE8", "preds-serve8", "model1.h5", "--workdir", str(tmp_path),
              "--device", "cpu", "--synthetic-partitions", str(parts), "--idle-timeout", "0.3", "--replicas", str(W)]
    events = []
    for r in range(W):
        assert cli_main(["serve"] + common + ["--replica-index", str(r)]) == 0
        s = json.loads(capsys.readouterr().out.strip().splitlines()[-1])
        events.append(s["events"])
        assert 1 <= len(s["partitions"]) <= 3
    assert sum(events) == n
    assert max(events) / min(events) <= 1.15, events
    res = _read_topic("fake://synthetic-SENSOR_SERVE8", "preds-serve8", parts)
    recs = [r for v in res.values() for r in v]
    assert len(recs) == n and len({(r["partition"], r["offset"]) for r in recs}) == n
    # a car's events come from one source partition -> ordered by offset in its result stream
    by_car = {}
    for r in recs:
        by_car.setdefault(r["car"], set()).add(r["partition"])
    assert all(len(v) == 1 for v in by_car.values())


@pytest.mark.gpu
def test_serve_on_gpu_matches_cpu_scores(tmp_path, capsys, cuda_device):
    from streamml.models.autoencoder import Autoencoder, load_model
    from streamml.data.stream import kafka
    model_file = tmp_path / "model1.h5"
    Autoencoder(device="cpu", seed=5).save(str(model_file))
    argv = ["serve", "synthetic://2000", "SENSOR_SERVE_GPU", "preds-gpu", "model1.h5", "--workdir", str(tmp_path),
            "--device", str(cuda_device), "--synthetic-partitions", "2", "--idle-timeout", "0.3", "--emit", "both"]
    assert cli_main(argv) == 0
    summary = json.loads(capsys.readouterr().out.strip().splitlines()[-1])
    assert summary["events"] == 2000
    servers = "fake://synthetic-SENSOR_SERVE_GPU"
    res = _read_topic(servers, "preds-gpu", 2)
    cpu = load_model(str(model_file), device="cpu", input_normalizer="cardata")
    for p, recs in res.items():
        src = next(iter(kafka(servers, [f"SENSOR_SERVE_GPU:{p}:0"]).batch(1 << 20)))
        got = np.array([r["score"] for r in recs])
        np.testing.assert_allclose(got, cpu.score(src.x), rtol=3e-2, atol=1e-3)   # bf16 MFMA vs fp32
        assert all("reconstruction" in r for r in recs)


@pytest.mark.gpu
def test_serve_low_latency_cli(tmp_path, capsys, cuda_device):
    """``serve --low-latency``: the C++ loop on the persistent scorer, two replicas over
    four partitions, every event scored once, keyed and ordered, offsets committed (a
    restarted replica has nothing left)."""
    from streamml.data.stream import kafka
    from streamml.models.autoencoder import Autoencoder, load_model
    model_file = tmp_path / "model1.h5"
    Autoencoder(device="cpu", seed=7).save(str(model_file))
    n, parts = 3000, 4
    common = ["serve", "synthetic://%d" % n, "SENSOR_LL", "preds-ll", "model1.h5", "--workdir", str(tmp_path),
              "--device", str(cuda_device), "--synthetic-partitions", str(parts), "--idle-timeout", "0.3",
              "--low-latency", "--max-wait-ms", "20", "--replicas", "2"]
    summaries = []
    import os
    mask = os.sched_getaffinity(0)
    for r in (0, 1):
        # the loop thread on one CPU (explicit, or one core of an L3 domain), restored after
        pin = ["--cpus", str(min(mask)) if r == 0 else "auto"]
        assert cli_main(common + ["--replica-index", str(r)] + pin) == 0
        assert os.sched_getaffinity(0) == mask
        summaries.append(json.loads(capsys.readouterr().out.strip().splitlines()[-1]))
    assert all(s_["low_latency"] for s_ in summaries)
    assert summaries[0]["events"] + summaries[1]["events"] == n
    servers = "fake://synthetic-SENSOR_LL"
    res = _read_topic(servers, "preds-ll", parts)
    assert sum(len(v) for v in res.values()) == n
    cpu = load_model(str(model_file), device="cpu", input_normalizer="cardata")
    for p, recs in res.items():
        assert [r["offset"] for r in recs] == list(range(len(recs)))
        src = next(iter(kafka(servers, [f"SENSOR_LL:{p}:0"]).batch(1 << 20)))
        assert [r["car"] for r in recs] == list(src.keys)
        np.testing.assert_allclose([r["score"] for r in recs], cpu.score(src.x), rtol=3e-2, atol=1e-3)
    assert cli_main(common + ["--replica-index", "0"]) == 0
    assert json.loads(capsys.readouterr().out.strip().splitlines()[-1])["events"] == 0
