"""Keras-granularity data parallelism with the gradient exchange inside the persistent
kernel (csrc/kernels/ae_minibatch.hip + runtime/p2p.cpp).

* in-launch replicas (one process, ``P2PGroup.local``): W workgroups = W ranks, each on its
  own rows; after every step the replicas are bit-identical and equal an fp32 PyTorch
  Keras-Adam run on the concatenated global batch;
* two processes sharing GPU 0 through HIP IPC handles (the same code path as one process
  per GPU over xGMI): replicas bit-identical, equal to the in-launch result, and the
  host-callable one-launch P2P all-reduce is exact.
"""
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest
import torch

from streamml.data.cardata import normalize_affine
from streamml.models.reference import TorchAE, init_dense_weights
from streamml.ops.ae import AESpec
from streamml.ops.ae_fleet import AEFleet
from streamml.parallel.p2p import P2PGroup

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("world,B,nsteps", [(2, 32, 40), (4, 32, 25), (3, 100, 12)])
def test_in_launch_replicas_match_global_batch_oracle(cuda_device, world, B, nsteps):
    spec = AESpec()
    sc, sh = normalize_affine()
    w0 = init_dense_weights(spec.layer_sizes, seed=9)
    fleet = AEFleet(spec, [w0] * world, cuda_device, scale=sc, shift=sh)
    rng = np.random.default_rng(4)
    raw = rng.uniform(0, 40, (world, B * nsteps, 18)).astype(np.float32)
    fleet.attach_rings(torch.from_numpy(raw).to(cuda_device), B)
    group = P2PGroup.local(cuda_device, world)
    half = nsteps // 2
    fleet.train_minibatches(half, dp=group)
    fleet.train_minibatches(nsteps - half, dp=group)    # a second launch continues the tags
    torch.cuda.synchronize()
    p = fleet.params.cpu()
    for r in range(1, world):
        assert torch.equal(p[0], p[r]), f"replica {r} diverged"
    ref = TorchAE(spec.layer_sizes, spec.activations, spec.activity_l1, w0)
    xn = raw * sc + sh
    for s in range(nsteps):
        ref.step(torch.from_numpy(np.concatenate([xn[r, s * B:(s + 1) * B] for r in range(world)])))
    for got, want in zip(fleet.get_weights(0), ref.get_weights()):
        np.testing.assert_allclose(got, want, rtol=2e-4, atol=2e-5)


def test_in_launch_timeout_is_reported(cuda_device):
    """A rank whose peer never runs: the poll gives up, the host raises (no hung GPU)."""
    from streamml.parallel.p2p import P2PTimeout
    spec = AESpec()
    fleet = AEFleet(spec, [init_dense_weights(spec.layer_sizes, seed=1)], cuda_device)
    fleet.attach_rings(torch.rand((32 * 4, 18), device=cuda_device), 32)
    group = P2PGroup.local(cuda_device, 2, timeout_s=0.2)
    kw = group.kernel_args(0)          # rank 0 of 2, rank 1 never launched
    fleet.C.ae_train_minibatches(fleet.ring, fleet.cursor, fleet.scale, fleet.shift, fleet.params, fleet.m,
                                 fleet.v, fleet.iter, fleet.metrics, 32, 3, spec.dims, spec.act_codes,
                                 float(spec.activity_l1), 1e-3, 0.9, 0.999, 1e-7, 1.0 / 64, True, None, None, **kw)
    with pytest.raises(P2PTimeout):
        group.check()


def test_two_processes_ipc_shared_gpu(tmp_path, cuda_device):
    env = dict(os.environ, SML_SHARE_GPU0="1", OMP_NUM_THREADS="2")
    out = str(tmp_path / "p2p")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}",
           os.path.join(ROOT, "tests", "helpers", "p2p_worker.py"), out]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=180, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    info = json.load(open(out + ".json"))
    print("p2p allreduce (2 ranks on one GPU):", info["allreduce_us"], "us per call")
    assert info["allreduce_ok"], info
    assert info["steps"] == 80 and info["iter"] == 80, info
    p0, p1 = np.load(out + ".rank0.npy"), np.load(out + ".rank1.npy")
    np.testing.assert_array_equal(p0, p1)
    assert info["engines"]["p2p"] == "persistent+p2p" and info["engines"]["local_sgd:5"] == "persistent+local_sgd:5"
    assert info["engines"]["stream"] == "persistent+p2p" and info["engines"]["stream_iters"] >= 190
    for tag in ("fit_p2p", "fit_local_sgd5", "fit_stream"):
        np.testing.assert_array_equal(np.load(f"{out}.{tag}.rank0.npy"), np.load(f"{out}.{tag}.rank1.npy"))
    # the same two shards through in-launch replicas give the same parameters
    spec = AESpec()
    sc, sh = normalize_affine()
    fleet = AEFleet(spec, [init_dense_weights(spec.layer_sizes, seed=5)] * 2, cuda_device, scale=sc, shift=sh)
    raw = np.stack([np.random.default_rng(100 + r).uniform(0, 40, (32 * 40, 18)).astype(np.float32)
                    for r in range(2)])
    fleet.attach_rings(torch.from_numpy(raw).to(cuda_device), 32)
    group = P2PGroup.local(cuda_device, 2)
    fleet.train_minibatches(80, dp=group)
    np.testing.assert_array_equal(fleet.params[0].cpu().numpy(), p0)
