"""bench.py's multi-rank path on the GPU box (one GPU): two torchrun ranks share
GPU 0 and all-reduce over gloo (``SML_SHARE_GPU0=1``; RCCL refuses two ranks on
one device).  Exercises exactly the code the driver's 2/4/8-GPU scaling run
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


@pytest.mark.gpu
def test_bench_two_ranks_shared_gpu(tmp_path, cuda_device):
    env = dict(os.environ, SML_SHARE_GPU0="1", OMP_NUM_THREADS="2")
    dump = str(tmp_path / "params")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}", os.path.join(ROOT, "bench.py"),
           "--gpus", "2", "--steps", "4", "--warmup", "2", "--batch-per-gpu", "65536",
           "--dataset-rows", "262144", "--infer-events", "0", "--dump-params", dump]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=240, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2 and out["steps"] == 4 and out["warmup"] == 2
    assert out["config"]["global_batch"] == 2 * 65536 and out["config"]["parallelism"] == "dp2"
    assert out["value"] > 0 and np.isfinite(out["final_epoch_loss"])
    coll = out["small_allreduce"]
    assert coll["bucket_bytes"] == 6144 and coll["backend_allreduce_us"] > 0 and coll["p2p_allreduce_us"] > 0, coll
    assert out["keras_batch32_dp"]["replicas_identical"] is True, out["keras_batch32_dp"]
    # rank 0's single-replica side measurements must not call a collective (dp="none"): the
    # other rank has already shut its process group down
    for k in ("fit_batch100", "stream_e2e"):
        assert out[k] and "error" not in out[k], out[k]
        assert out[k]["engine"] == "persistent", out[k]
    p0 = np.load(dump + ".rank0.npy")
    p1 = np.load(dump + ".rank1.npy")
    np.testing.assert_array_equal(p0, p1)
