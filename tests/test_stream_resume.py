"""Continuous training from a partitioned topic with checkpointed stream positions (SURVEY.md 5.3:
consumer offsets committed with checkpoints; reference README.md:124-128, "train from the commit
log").  Two gloo ranks under torchrun follow a 4-partition topic of the shared broker in bounded
segments (cli/train.py ``segment_rows``); rank 1 is killed mid-segment, torchrun restarts the
group, and the job resumes from the last checkpoint's positions: the final parameters equal an
uninterrupted run with the same segment boundaries, and every record is trained exactly once."""
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PARTS, PER_PART, SEG = 4, 2400, 600


def _env(**kw):
    e = dict(os.environ, PYTHONPATH=REPO, OMP_NUM_THREADS="2", SML_PG_TIMEOUT_S="60")
    for k in ("SML_FAULT_RANK", "SML_FAULT_STEP", "SML_FAULT_MODE"):
        e.pop(k, None)
    e.update({k: str(v) for k, v in kw.items()})
    return e


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _run(args, env, ranks=2, restarts=0):
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={ranks}",
           f"--max-restarts={restarts}", "--master-addr=127.0.0.1", f"--master-port={_port()}",
           "-m", "streamml.cli", "train", *args]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600, env=env)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith('{"job"')]
    return json.loads(lines[-1]), r


@pytest.fixture(scope="module")
def broker():
    from streamml.data import stream as S
    from streamml.data.avro import AvroCodec
    from streamml.data.produce import encode_chunk
    from streamml.kafka.client import FakeBroker
    b = FakeBroker(sasl_username="test", sasl_password="test123")   # the reference's SASL/PLAIN config
    b.create_topic("SENSOR_DATA_S_AVRO", PARTS)
    codec = AvroCodec("cardata-v1")
    for p in range(PARTS):
        c = next(iter(S.synthetic(PER_PART, chunk=PER_PART, seed=10 + p, failure_rate=0.0)))
        buf, offs = encode_chunk(codec, c.x, c.label)
        b.append_buffer("SENSOR_DATA_S_AVRO", p, buf, offs)
    yield b
    b.stop()


def _args(b, ckpt, group):
    return ["--device=cpu", f"--servers={b.address}", "--partition=-1", "--offset=0", "--batch_size=100",
            f"--segment-rows={SEG}", "--epochs=4", "--seed=5", f"--group={group}", f"--ckpt-dir={ckpt}"]


def _weights(path):
    from streamml.models.autoencoder import load_model
    return load_model(path, device="cpu").get_weights()


@pytest.mark.dist
def test_continuous_training_crash_resumes_from_checkpointed_positions(tmp_path, broker):
    from streamml.ckpt import resume as rs
    a, b = tmp_path / "a", tmp_path / "b"
    ref, _ = _run(_args(broker, a, "ref"), _env())
    # each rank owns 2 partitions x 600 records per segment = 12 steps of 100 rows: step 27 is in
    # segment 3 (index 2), after the checkpoint of segment 2
    rec, r = _run(_args(broker, b, "crash"), _env(SML_FAULT_RANK=1, SML_FAULT_STEP=27), restarts=1)
    assert "[fault-injection] rank 1 crash at step 27" in r.stderr
    assert ref["resumed_from_epoch"] == 0 and rec["resumed_from_epoch"] == 2 and rec["world_size"] == 2
    # exactly once: every partition consumed to 4 x 600, the resumed run read segments 3 and 4 only
    want = {f"SENSOR_DATA_S_AVRO:{p}": 4 * SEG for p in range(PARTS)}
    assert ref["positions"] == want and rec["positions"] == want
    assert ref["segment_records"] == [2 * SEG] * 4 and rec["segment_records"] == [2 * SEG] * 2
    st2 = rs.read_state(rs.checkpoint_path(str(b), 2))
    assert st2["offsets"] == {f"SENSOR_DATA_S_AVRO:{p}": 2 * SEG for p in range(PARTS)}
    assert rec["final_loss"] == pytest.approx(ref["final_loss"], rel=1e-6)
    for u, v in zip(_weights(str(a / "model1.h5")), _weights(str(b / "model1.h5"))):
        np.testing.assert_array_equal(u, v)
    # the consumer group follows the checkpoints
    from streamml.kafka.client import KafkaClient
    c = KafkaClient(broker.address, ["security.protocol=sasl_plaintext", "sasl.mechanisms=PLAIN",
                                     "sasl.username=test", "sasl.password=test123"])
    assert [c.committed("crash", "SENSOR_DATA_S_AVRO", p) for p in range(PARTS)] == [4 * SEG] * PARTS


@pytest.mark.dist
def test_continuous_training_rescaled_restart(tmp_path, broker):
    """The checkpoint's position map is per partition, so a restart with another world size (1
    rank after 2) still resumes every partition where the last checkpoint left it."""
    d = tmp_path / "c"
    args = _args(broker, d, "rescale")
    first, _ = _run([*args[:-3], "--epochs=2", *args[-2:]], _env())
    assert first["positions"] == {f"SENSOR_DATA_S_AVRO:{p}": 2 * SEG for p in range(PARTS)}
    cmd = [sys.executable, "-m", "streamml.cli", "train", *args]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600, env=_env())
    assert r.returncode == 0, r.stderr[-3000:]
    out = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith('{"job"')][-1])
    assert out["resumed_from_epoch"] == 2 and out["world_size"] == 1
    assert out["positions"] == {f"SENSOR_DATA_S_AVRO:{p}": 4 * SEG for p in range(PARTS)}
    assert out["segment_records"] == [PARTS * SEG] * 2
