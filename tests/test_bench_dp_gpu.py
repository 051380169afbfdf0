"""bench.py's multi-rank path on the GPU box (one GPU).

``test_bench_two_ranks_shared_gpu``: the driver's plain ``python3 bench.py --gpus 2``
self-launches two torchrun ranks as a child process; they share GPU 0 and all-reduce
over gloo (``SML_SHARE_GPU0=1``; RCCL refuses two ranks on one device).  Exercises exactly the code the driver's 2/4/8-GPU scaling run
executes -- shard-by-key data, broadcast, per-step flat-bucket all-reduce,
barrier-bracketed timing, max-over-ranks -- and checks that the replicas end
bit-identical and rank 0 prints one well-formed JSON line.
"""
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _check_stream_dp(out, n):
    """The stream_dp phase: every rank trained on its own offset ranges of the 10-partition topic."""
    sdp = out["stream_dp"]
    assert "error" not in sdp and "skipped" not in sdp, sdp
    assert sdp["world"] == n and len(sdp["partition_lists"]) == n and all(sdp["partition_lists"]), sdp
    assert sdp["steps_equal"] and sdp["replicas_identical"], sdp
    assert sum(r["rows_read"] for r in sdp["per_rank"]) == sdp["rows"], sdp
    assert sdp["trained_rows"] == sum(r["kept"] for r in sdp["per_rank"]) and sdp["trained_rows_per_s"] > 0, sdp
    assert out["stream_dp_rows_per_s"] == sdp["trained_rows_per_s"]


@pytest.mark.gpu
def test_bench_two_ranks_shared_gpu(tmp_path, cuda_device):
    env = dict(os.environ, SML_SHARE_GPU0="1", OMP_NUM_THREADS="2")
    dump = str(tmp_path / "params")
    # no torchrun prefix: bench.py must launch its own ranks (the driver runs it this way)
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"),
           "--gpus", "2", "--steps", "4", "--warmup", "2", "--batch-per-gpu", "65536",
           "--dataset-rows", "262144", "--infer-events", "2000", "--infer-repeats", "1", "--e2e-events", "0",
           "--lstm-steps", "0", "--batch32-steps", "2000", "--mqtt-clients", "0", "--large-stream-rows", "400000",
           "--stream-dp-rows", "150000", "--stream-dp-batch", "16384", "--dump-params", dump]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=240, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2 and out["steps"] == 4 and out["warmup"] == 2
    assert out["config"]["global_batch"] == 2 * 65536 and out["config"]["parallelism"] == "dp2"
    assert out["value"] > 0 and np.isfinite(out["final_epoch_loss"])
    assert out["backend"] == "gloo" and len(out["per_rank_ms_per_step"]["ranks"]) == 2
    # the record says what it is: two ranks on ONE device, a labelled rehearsal
    assert out["rehearsal"] is True and out["n_distinct_devices"] == 1, out["devices"]
    devs = out["devices"]
    assert devs["world_size"] == 2 and [d["rank"] for d in devs["per_rank"]] == [0, 1]
    assert len({d["pci_bus_id"] for d in devs["per_rank"]}) == 1 and all(d["pid"] > 0 for d in devs["per_rank"])
    # config 5 per replica: both ranks scored their own shard
    assert len(out["infer_per_replica_p50_us"]) == 2 and all(v > 0 for v in out["infer_per_replica_p50_us"])
    coll = out["small_allreduce"]
    assert coll["bucket_bytes"] == 6144 and coll["backend_allreduce_us"] > 0 and coll["p2p_allreduce_us"] > 0, coll
    assert out["keras_batch32_dp"]["replicas_identical"] is True, out["keras_batch32_dp"]
    # rank 0's single-replica side measurements must not call a collective (dp="none"): the
    # other rank has already shut its process group down
    for k in ("fit_batch100", "stream_e2e"):
        assert out[k] and "error" not in out[k], out[k]
        assert out[k]["engine"] == "persistent", out[k]
    big = out["stream_large_batch"]
    assert "error" not in big and big["engine"] == "throughput" and big["trained_rows_per_s"] > 0, big
    assert [c["workers"] for c in big["decode_curve"]] == [1, 2, 4, 8, 16], big
    _check_stream_dp(out, 2)
    p0 = np.load(dump + ".rank0.npy")
    p1 = np.load(dump + ".rank1.npy")
    np.testing.assert_array_equal(p0, p1)


@pytest.mark.gpu
@pytest.mark.parametrize("n", [4, 8])
def test_bench_n_ranks_rehearsal(tmp_path, cuda_device, n):
    """The driver's 4- and 8-GPU scaling run rehearsed on one GPU: ``bench.py --gpus N``
    self-launches N ranks (gloo, all on GPU 0) with EVERY side measurement on, at reduced
    sizes.  The line must carry N replicas' scoring p50s, the small all-reduce, an in-kernel
    P2P DP run with N peers whose replicas end bit-identical, every rank's parameters
    identical, and the per-phase wall clock; the whole job must stay inside its budget."""
    env = dict(os.environ, SML_SHARE_GPU0="1", OMP_NUM_THREADS="2")
    dump = str(tmp_path / "params")
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"),
           "--gpus", str(n), "--steps", "4", "--warmup", "2", "--batch-per-gpu", "65536",
           "--dataset-rows", "262144", "--infer-events", "2000", "--infer-repeats", "1", "--e2e-events", "2000",
           "--batch32-steps", "2000", "--fleet-models", "64", "--dp-steps", "500", "--collective-iters", "50",
           "--fit-epochs", "2", "--fresh-steps", "2", "--fit-rows", "200000", "--stream-rows", "500000",
           "--lstm-steps", "4", "--mqtt-clients", "2000", "--mqtt-interval", "1", "--mqtt-messages", "2",
           "--large-stream-rows", "400000", "--stream-dp-rows", "100000", "--stream-dp-batch", "8192",
           "--budget-s", "240", "--dump-params", dump]
    t0 = __import__("time").time()
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300, env=env, cwd=ROOT)
    wall = __import__("time").time() - t0
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    out = json.loads(lines[0])
    assert out["n_gpus"] == n and out["config"]["parallelism"] == f"dp{n}"
    assert out["config"]["global_batch"] == n * 65536 and len(out["per_rank_ms_per_step"]["ranks"]) == n
    assert len(out["infer_per_replica_p50_us"]) == n and all(v > 0 for v in out["infer_per_replica_p50_us"])
    coll = out["small_allreduce"]
    assert coll.get("backend_allreduce_us", 0) > 0 and coll.get("p2p_allreduce_us", 0) > 0, coll
    dpr = out["keras_batch32_dp"]
    assert dpr.get("replicas_identical") is True and dpr["global_batch"] == 32 * n, dpr
    ph = out["phase_s"]
    for k in ("infer", "small_allreduce", "keras_batch32_dp", "kafka_e2e", "lstm_kafka_e2e", "keras_batch32",
              "fit_large_batch",
              "fresh_rows", "fit_batch100", "stream_e2e", "stream_large_batch", "lstm_seq50", "lstm_ref",
              "lstm_infer", "mqtt_e2e", "stream_dp", "lstm_seq50_dp",
              "total_wall"):
        assert k in ph, (k, ph, out["budget"])
    ldp = out["lstm_seq50_dp"]   # config 3 under DP: every rank its own 65 536 windows, one bucket per step
    assert ldp.get("replica_max_abs_diff") == 0.0 and ldp["global_batch"] == n * 65536, ldp
    assert out["summary"]["lstm_seq50_dp_windows_per_s"] > 0
    assert not out["budget"]["skipped"], out["budget"]
    assert out["mqtt_connections"] == 2000 and out["mqtt_dropped"] == 0, out["mqtt_e2e"]
    _check_stream_dp(out, n)
    assert wall < 300
    ps = [np.load(f"{dump}.rank{i}.npy") for i in range(n)]
    for p in ps[1:]:
        np.testing.assert_array_equal(ps[0], p)


@pytest.mark.gpu
def test_bench_budget_skips_and_still_prints(cuda_device):
    """A budget too small for any side measurement: every phase is skipped and named, the
    headline line still prints."""
    env = dict(os.environ, OMP_NUM_THREADS="2")
    env.pop("SML_SHARE_GPU0", None)
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--steps", "3", "--warmup", "1", "--batch-per-gpu",
           "65536", "--dataset-rows", "131072", "--budget-s", "1"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=240, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    out = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][0])
    assert out["value"] > 0 and out["n_gpus"] == 1
    sk = out["budget"]["skipped"]
    assert "infer" in sk and "kafka_e2e" in sk and "lstm_seq50" in sk, sk


@pytest.mark.gpu
def test_bench_force_pg_rccl_world1(cuda_device):
    """The whole DP bench path on ONE RCCL rank (SML_FORCE_PG=1): nccl communicator,
    per-step all-reduce in the timed loop, P2P exchange + in-kernel DP, collectives."""
    env = dict(os.environ, SML_FORCE_PG="1", OMP_NUM_THREADS="2")
    env.pop("SML_SHARE_GPU0", None)
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "1", "--steps", "4", "--warmup", "2",
           "--batch-per-gpu", "65536", "--dataset-rows", "262144", "--infer-events", "1000", "--infer-repeats", "1",
           "--e2e-events", "0", "--lstm-steps", "0", "--batch32-steps", "2000", "--fit-rows", "0",
           "--stream-rows", "0", "--large-stream-rows", "0", "--dp-steps", "2000", "--collective-iters", "50",
           "--mqtt-clients", "0"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=240, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    out = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][0])
    assert out["n_gpus"] == 1 and out["backend"] == "nccl", out
    assert out["small_allreduce"]["backend"] == "nccl" and out["small_allreduce"]["backend_allreduce_us"] > 0
    assert out["small_allreduce"]["p2p_allreduce_us"] > 0, out["small_allreduce"]
    assert out["keras_batch32_dp"]["replicas_identical"] is True, out["keras_batch32_dp"]


def test_bench_refuses_missing_gpus():
    """--gpus N with fewer visible GPUs (none here) exits non-zero instead of measuring fewer."""
    env = dict(os.environ)
    for k in ("SML_SHARE_GPU0", "WORLD_SIZE"):
        env.pop(k, None)
    import torch
    n = torch.cuda.device_count()
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(max(n + 1, 2)), "--steps", "1"],
                       capture_output=True, text=True, timeout=120, env=env, cwd=ROOT)
    assert r.returncode == 2, r.stdout[-2000:] + r.stderr[-2000:]
    assert "visible" in r.stderr and not r.stdout.strip()
