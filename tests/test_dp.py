"""Data parallelism (world_size 2 over gloo, launched with torchrun on 127.0.0.1).

Checks the DP contract every model family shares: one flat all-reduce of the
gradient bucket per step with global-batch mean scaling -> replicas stay bit-
identical, and DP training equals single-process training on the concatenated
global batches.
"""
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.fixture(scope="module")
def dp_run(tmp_path_factory):
    out = tmp_path_factory.mktemp("dp")
    env = dict(os.environ, OMP_NUM_THREADS="2")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}",
           os.path.join(HERE, "helpers", "dp_worker.py"), str(out)]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600, env=env)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    return out


def _load(path):
    z = np.load(path)
    return [z[k] for k in z.files if k.startswith("arr_")], z


@pytest.mark.dist
@pytest.mark.parametrize("fam", ["ae", "lstm", "mlp"])
def test_replicas_identical(dp_run, fam):
    a, _ = _load(dp_run / f"{fam}_0.npz")
    b, _ = _load(dp_run / f"{fam}_1.npz")
    for u, v in zip(a, b):
        np.testing.assert_array_equal(u, v)


@pytest.mark.dist
def test_ae_dp_equals_single_process(dp_run):
    from streamml.models.autoencoder import Autoencoder
    rng = np.random.default_rng(0)
    x = rng.uniform(-1, 1, size=(256, 18)).astype(np.float32)
    sh = [x[:128], x[128:]]
    glob = np.concatenate([np.concatenate([sh[0][b * 16:(b + 1) * 16], sh[1][b * 16:(b + 1) * 16]])
                           for b in range(8)])
    ae = Autoencoder(device="cpu", seed=3)
    h = ae.fit(glob, epochs=2, batch_size=32, shuffle=False, verbose=0)
    w, z = _load(dp_run / "ae_0.npz")
    for u, v in zip(w, ae.get_weights()):
        np.testing.assert_allclose(u, v, rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(z["loss"], h.history["loss"], rtol=1e-5)


@pytest.mark.dist
def test_fit_dp_none_is_single_replica_inside_a_group(dp_run):
    """fit(dp="none") on rank 0 alone (its peer already shut down) trains on all of x like a
    process with no group: bench.py's rank-0 side measurements at N > 1 rely on it."""
    from streamml.models.autoencoder import Autoencoder
    x = np.random.default_rng(0).uniform(-1, 1, size=(256, 18)).astype(np.float32)
    ae = Autoencoder(device="cpu", seed=4)
    h = ae.fit(x, epochs=1, batch_size=32, shuffle=False, verbose=0)
    w, z = _load(dp_run / "ae_solo.npz")
    for u, v in zip(w, ae.get_weights()):   # CPU torch thread counts differ: summation order only
        np.testing.assert_allclose(u, v, rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(z["loss"], h.history["loss"], rtol=1e-5)


@pytest.mark.dist
def test_lstm_dp_short_last_batch_is_mean_over_trained_rows(dp_run):
    """Uneven shards (31 / 30 windows) at batch 8: the last step trains 7 + 6 rows, and its
    update must be the mean over those 13 rows -- the single-process step on the concatenated
    rows -- not the average of the two ranks' means."""
    import torch
    from streamml.models.lstm import LSTMPredictor
    from streamml.parallel.dp import shard_range
    rng = np.random.default_rng(0)
    rng.uniform(-1, 1, size=(256, 18))          # the worker's draws before the uneven set
    rng.uniform(-1, 1, size=(64, 4, 18))
    rng.uniform(-1, 1, size=(64, 18))
    xu = rng.uniform(-1, 1, size=(61, 4, 18)).astype(np.float32)
    yu = rng.uniform(-1, 1, size=(61, 18)).astype(np.float32)
    sh = [shard_range(61, r, 2) for r in range(2)]
    m = LSTMPredictor.reference(look_back=4, device="cpu", seed=2)
    m.compile() if hasattr(m, "compile") and not getattr(m, "compiled", True) else None
    for b in range(4):
        idx = np.concatenate([np.arange(s0, s1)[b * 8:(b + 1) * 8] for s0, s1 in sh])
        m.train_step(torch.as_tensor(xu[idx]), torch.as_tensor(yu[idx]))
    a, _ = _load(dp_run / "lstm_uneven_0.npz")
    b_, _ = _load(dp_run / "lstm_uneven_1.npz")
    for u, v in zip(a, b_):
        np.testing.assert_array_equal(u, v)
    for u, v in zip(a, m.fp.get()):
        np.testing.assert_allclose(u, v.detach().cpu().numpy() if hasattr(v, "detach") else v, rtol=1e-5, atol=1e-6)
