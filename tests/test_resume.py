"""Checkpoint / resume and failure recovery.

* a job stopped after epoch 2 and restarted from its checkpoint ends with the
  same weights as an uninterrupted run;
* under torchrun (2 ranks, gloo) with a rank crashed mid-epoch by fault
  injection, the survivors error out on the collective, torchrun restarts the
  group, the job resumes from the last checkpoint and again matches the
  uninterrupted run bit for bit.
"""
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
COMMON = ["--device=cpu", "--servers=synthetic://6000", "--batch_size=100", "--take=10", "--seed=3"]


def _env(**kw):
    e = dict(os.environ, PYTHONPATH=REPO, OMP_NUM_THREADS="2", SML_PG_TIMEOUT_S="60")
    for k in ("SML_FAULT_RANK", "SML_FAULT_STEP", "SML_FAULT_MODE"):
        e.pop(k, None)
    e.update({k: str(v) for k, v in kw.items()})
    return e


def _run(args, env, torchrun=0, restarts=0):
    if torchrun:
        s = socket.socket()
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
        s.close()
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={torchrun}",
               f"--max-restarts={restarts}", "--master-addr=127.0.0.1", f"--master-port={port}",
               "-m", "streamml.cli", "train", *args]
    else:
        cmd = [sys.executable, "-m", "streamml.cli", "train", *args]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600, env=env)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith('{"job"')]
    return json.loads(lines[-1]), r


def _weights(path):
    from streamml.models.autoencoder import load_model
    return load_model(path, device="cpu").get_weights()


def test_resume_matches_uninterrupted(tmp_path):
    a, b = tmp_path / "a", tmp_path / "b"
    full, _ = _run([*COMMON, "--epochs=4", f"--ckpt-dir={a}"], _env())
    part, _ = _run([*COMMON, "--epochs=2", f"--ckpt-dir={b}"], _env())
    assert part["resumed_from_epoch"] == 0
    rest, _ = _run([*COMMON, "--epochs=4", f"--ckpt-dir={b}"], _env())
    assert rest["resumed_from_epoch"] == 2
    assert rest["final_loss"] == pytest.approx(full["final_loss"], rel=1e-6)
    for u, v in zip(_weights(str(a / "model1.h5")), _weights(str(b / "model1.h5"))):
        np.testing.assert_array_equal(u, v)
    from streamml.ckpt import resume as rs
    cks = rs.list_checkpoints(str(b))
    assert [os.path.basename(p) for p in cks] == ["ckpt-00002.h5", "ckpt-00003.h5", "ckpt-00004.h5"]
    assert rs.read_state(cks[-1])["epoch"] == 4


@pytest.mark.dist
def test_dp_crash_restart_resumes(tmp_path):
    a, b = tmp_path / "a", tmp_path / "b"
    ref, _ = _run([*COMMON, "--epochs=3", f"--ckpt-dir={a}"], _env(), torchrun=2)
    # rank 1 dies at global step 15 (epoch 2 of 3: 10 steps per epoch), first attempt only
    rec, r = _run([*COMMON, "--epochs=3", f"--ckpt-dir={b}"], _env(SML_FAULT_RANK=1, SML_FAULT_STEP=15),
                  torchrun=2, restarts=1)
    assert "[fault-injection] rank 1 crash at step 15" in r.stderr
    assert rec["resumed_from_epoch"] == 1 and rec["world_size"] == 2
    assert rec["final_loss"] == pytest.approx(ref["final_loss"], rel=1e-6)
    for u, v in zip(_weights(str(a / "model1.h5")), _weights(str(b / "model1.h5"))):
        np.testing.assert_array_equal(u, v)


@pytest.mark.dist
def test_hung_peer_detected_by_collective_timeout(tmp_path):
    """A rank that stops answering (hang, not crash) turns into an error on its peer within the
    process-group timeout instead of a silent stall; torchrun then fails the job."""
    import time
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    env = _env(SML_FAULT_RANK=1, SML_FAULT_STEP=5, SML_FAULT_MODE="hang", SML_PG_TIMEOUT_S=5)
    t0 = time.time()
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
                        "--master-addr=127.0.0.1", f"--master-port={port}", "-m", "streamml.cli", "train", *COMMON,
                        "--epochs=2", f"--ckpt-dir={tmp_path}"], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode != 0
    assert "[fault-injection] rank 1 hang at step 5" in r.stderr
    assert time.time() - t0 < 120
