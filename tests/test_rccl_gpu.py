"""The DP code path under a real RCCL (``nccl``) process group of ONE rank.

Every multi-rank test on the one-GPU box shares GPU 0 over gloo (RCCL refuses two ranks
on one device), so this is the test that opens an RCCL communicator: ``SML_FORCE_PG=1``
makes ``dp.init_from_env`` create the group at world 1, and the script exercises
``init_process_group(device_id=...)``, ``all_reduce``, ``barrier(device_ids=...)``,
``all_gather_object``, ``P2PGroup.try_create``, one ``step_ring`` whose gradient bucket
goes through the RCCL all-reduce -- compared bit-for-bit with the same step without it --
and a reference-stack LSTM epoch on the fused DP step (flat-gradient all-reduce per step).
Runs in a child process so the group never outlives the test.
"""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

SCRIPT = r'''
import json, sys
import numpy as np
import torch
import torch.distributed as dist
sys.path.insert(0, sys.argv[1])
from streamml.parallel import dp
from streamml.parallel.p2p import P2PGroup
from streamml.ops.ae import AESpec, FusedAE
from streamml.models.reference import init_dense_weights
from streamml.data.cardata import normalize_affine, synthetic_device_tensor

env = dp.init_from_env("cuda")
dev = env.device
res = {"backend": dist.get_backend(), "world": dist.get_world_size(), "is_dist": env.is_dist}
t = torch.arange(1540, dtype=torch.float32, device=dev)
dp.allreduce_sum_(t)
res["allreduce_ok"] = bool(torch.equal(t, torch.arange(1540, dtype=torch.float32, device=dev)))
dp.barrier(dev)
objs = [None]
dist.all_gather_object(objs, {"rank": env.rank})
res["gather"] = objs
g, err = P2PGroup.try_create(dev)
res["p2p"] = g is not None
res["p2p_err"] = repr(err) if err else None
spec = AESpec()
sc, sh = normalize_affine()
w = init_dense_weights(spec.layer_sizes, seed=3)
data = synthetic_device_tensor(1 << 16, dev, seed=3)
a = FusedAE(spec, w, dev, scale=sc, shift=sh)
b = FusedAE(spec, w, dev, scale=sc, shift=sh)
a.attach_ring(data, 1 << 15)
b.attach_ring(data, 1 << 15)
a.step_ring(global_batch=1 << 15, allreduce=dp.allreduce_sum_)
b.step_ring(global_batch=1 << 15)
torch.cuda.synchronize()
res["step_equal"] = bool(torch.equal(a.params, b.params))
res["step_changed"] = not bool(torch.equal(a.params, torch.from_numpy(__import__("streamml.ops.ae", fromlist=["pack_image"]).pack_image(w)).to(dev)))
if g is not None:
    a.attach_ring(data, 32)
    a.train_minibatches(100, dp=g)
    res["p2p_steps_ok"] = bool(torch.isfinite(a.params).all())
# the reference LSTM stack under the group: fused no-autograd steps + the RCCL all-reduce
from streamml.models.lstm import LSTMPredictor
from streamml.data.stream import sliding_windows
rows = torch.tensor(np.random.default_rng(1).uniform(-1, 1, (257, 18)), dtype=torch.float32, device=dev)
X, Y = sliding_windows(rows, 1)
la = LSTMPredictor.reference(look_back=1, device=dev, seed=2)
lb = LSTMPredictor.reference(look_back=1, device=dev, seed=2)
la.fit(X, Y, epochs=1, batch_size=64, verbose=0)
res["lstm_engine"] = la.last_fit_engine
for s in range(0, 256, 64):
    lb.train_step(X[s:s + 64], Y[s:s + 64])
torch.cuda.synchronize()
res["lstm_equal"] = bool(torch.equal(la.fp.flat, lb.fp.flat))
dp.shutdown()
print("RESULT " + json.dumps(res))
'''


@pytest.mark.gpu
def test_dp_path_on_one_rccl_rank(cuda_device):
    env = dict(os.environ, SML_FORCE_PG="1")
    for k in ("SML_SHARE_GPU0", "WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT", "SML_DIST_BACKEND"):
        env.pop(k, None)
    r = subprocess.run([sys.executable, "-c", SCRIPT, ROOT], capture_output=True, text=True, timeout=180, env=env,
                       cwd=ROOT)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    res = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("RESULT ")][0][7:])
    assert res["backend"] == "nccl" and res["world"] == 1 and res["is_dist"], res
    assert res["allreduce_ok"] and res["gather"] == [{"rank": 0}], res
    assert res["p2p"], res
    assert res["p2p_steps_ok"], res
    assert res["step_equal"] and res["step_changed"], res
    assert res["lstm_engine"] == "fused+allreduce" and res["lstm_equal"], res
