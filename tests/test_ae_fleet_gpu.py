"""Fleet mode of the persistent small-batch AE trainer (csrc/kernels/ae_minibatch.hip,
``ops/ae_fleet.py``): M independent models, one workgroup each.

Each fleet model must be BIT-identical to the same model trained alone through
``FusedAE.train_minibatches`` (same kernel instantiation, per-workgroup pointer
rebase only), which test_ae_minibatch_gpu.py pins against an fp32 torch Keras-Adam
oracle.  One fleet model is also checked against that oracle directly."""
import numpy as np
import pytest
import torch

from streamml.data.cardata import normalize_affine
from streamml.models.reference import TorchAE, init_dense_weights
from streamml.ops.ae import AESpec, FusedAE
from streamml.ops.ae_fleet import AEFleet

pytestmark = pytest.mark.gpu


def _alone(spec, w, ring, B, nsteps, launches, lr, scale, shift, dev, offset=0):
    ae = FusedAE(spec, w, dev, lr=lr, scale=scale, shift=shift)
    ae.attach_ring(ring, B)
    ae.cursor.fill_(offset)
    for _ in range(launches):
        ae.train_minibatches(nsteps)
    return ae


@pytest.mark.parametrize("D,B", [(18, 32), (30, 32), (18, 20)])
def test_fleet_per_model_rings_bit_identical(cuda_device, D, B):
    spec = AESpec(input_dim=D)
    M, nsteps, launches = 5, 40, 2
    ws = [init_dense_weights(spec.layer_sizes, seed=100 + i) for i in range(M)]
    lrs = np.array([1e-3, 3e-3, 5e-4, 1e-2, 2e-3], np.float32)
    scale = np.full(D, 1 / 40.0, np.float32)
    shift = np.zeros(D, np.float32)
    rng = np.random.default_rng(7)
    rings = torch.from_numpy(rng.uniform(0, 40, size=(M, B * 16, D)).astype(np.float32)).to(cuda_device)

    fleet = AEFleet(spec, ws, cuda_device, lr=lrs, scale=scale, shift=shift)
    fleet.attach_rings(rings, B)
    for _ in range(launches):
        fleet.train_minibatches(nsteps)
    got = fleet.read_metrics()
    for i in range(M):
        ae = _alone(spec, ws[i], rings[i].contiguous(), B, nsteps, launches, float(lrs[i]), scale, shift, cuda_device)
        assert torch.equal(fleet.params[i], ae.params), f"model {i} params differ from the single-model run"
        assert torch.equal(fleet.m[i], ae.m) and torch.equal(fleet.v[i], ae.v)
        assert int(fleet.iter[i]) == int(ae.iter) == nsteps * launches
        assert int(fleet.cursor[i]) == int(ae.cursor)
        ref = ae.read_metrics()
        assert got[i]["rows"] == ref["rows"]
        np.testing.assert_allclose(got[i]["loss"], ref["loss"], rtol=1e-6)
        np.testing.assert_allclose(got[i]["accuracy"], ref["accuracy"], rtol=1e-6)
    # the models really are independent: different lrs / data -> different weights
    assert not torch.equal(fleet.params[0], fleet.params[1])


def test_fleet_shared_ring_offsets(cuda_device):
    spec = AESpec()
    scale, shift = normalize_affine()
    M, B, nsteps = 4, 32, 30
    w = init_dense_weights(spec.layer_sizes, seed=5)
    rng = np.random.default_rng(9)
    ring = torch.from_numpy(rng.uniform(0, 40, size=(B * 12, 18)).astype(np.float32)).to(cuda_device)
    offs = [0, 3 * B, 7 * B, 11 * B]
    fleet = AEFleet(spec, [w] * M, cuda_device, scale=scale, shift=shift)   # same init, different data windows
    fleet.attach_rings(ring, B, offsets=offs)
    fleet.train_minibatches(nsteps)
    for i in range(M):
        ae = _alone(spec, w, ring, B, nsteps, 1, 1e-3, scale, shift, cuda_device, offset=offs[i])
        assert torch.equal(fleet.params[i], ae.params)
        assert int(fleet.cursor[i]) == int(ae.cursor)
    assert not torch.equal(fleet.params[0], fleet.params[1])


def test_fleet_model_matches_torch_oracle(cuda_device):
    spec = AESpec()
    scale, shift = normalize_affine()
    M, B, nsteps = 3, 32, 50
    ws = [init_dense_weights(spec.layer_sizes, seed=20 + i) for i in range(M)]
    rng = np.random.default_rng(4)
    raw = rng.uniform(0, 40, size=(M, B * 25, 18)).astype(np.float32)
    fleet = AEFleet(spec, ws, cuda_device, scale=scale, shift=shift)
    fleet.attach_rings(torch.from_numpy(raw).to(cuda_device), B)
    fleet.train_minibatches(nsteps)
    i = 2
    xn = (raw[i] * scale + shift).astype(np.float32)
    ref = TorchAE(spec.layer_sizes, spec.activations, spec.activity_l1, ws[i])
    for s in range(nsteps):
        r0 = (s * B) % xn.shape[0]
        ref.step(torch.from_numpy(xn[r0:r0 + B]))
    for got, want in zip(fleet.get_weights(i), ref.get_weights()):
        np.testing.assert_allclose(got, want, rtol=2e-4, atol=2e-5)


def test_fleet_beyond_resident_capacity(cuda_device):
    """More models than resident workgroups (3 per CU x 256 CUs): a second dispatch round."""
    spec = AESpec()
    scale, shift = normalize_affine()
    M, B, nsteps = 1000, 32, 20
    seeds = list(range(M))
    fleet = AEFleet.from_seeds(spec, seeds, cuda_device, scale=scale, shift=shift)
    rng = np.random.default_rng(1)
    ring = torch.from_numpy(rng.uniform(0, 40, size=(B * 64, 18)).astype(np.float32)).to(cuda_device)
    fleet.attach_rings(ring, B, offsets=[(i % 64) * B for i in range(M)])
    fleet.train_minibatches(nsteps)
    torch.cuda.synchronize()
    assert torch.isfinite(fleet.params).all()
    assert (fleet.iter == nsteps).all()
    # M > #CUs runs the 128-VGPR (two models per CU) instantiation: a separately compiled
    # kernel, so equal to the single-model build to fp32 rounding rather than bitwise
    for i in (0, 517, M - 1):
        ae = _alone(spec, init_dense_weights(spec.layer_sizes, seed=i), ring, B, nsteps, 1, 1e-3, scale, shift,
                    cuda_device, offset=(i % 64) * B)
        d = (fleet.params[i] - ae.params).abs().max().item()
        print(f"model {i}: max |fleet - alone| = {d:.3g}")
        torch.testing.assert_close(fleet.params[i], ae.params, rtol=2e-4, atol=2e-5)
    i = 517
    xn = ((ring.cpu().numpy() * scale + shift).astype(np.float32))
    ref = TorchAE(spec.layer_sizes, spec.activations, spec.activity_l1, init_dense_weights(spec.layer_sizes, seed=i))
    for s in range(nsteps):
        r0 = ((i % 64) * B + s * B) % xn.shape[0]
        ref.step(torch.from_numpy(xn[r0:r0 + B]))
    for got, want in zip(fleet.get_weights(i), ref.get_weights()):
        np.testing.assert_allclose(got, want, rtol=2e-4, atol=2e-5)
    # a fleet model exported as a standalone FusedAE scores like the fleet's weights
    x = ring[:256]
    ae = fleet.model(517)
    r_fleet, s_fleet, _ = ae.forward(x)
    assert torch.isfinite(s_fleet).all()


def test_fleet_cli_one_model_per_car(cuda_device, tmp_path):
    """``python -m streamml.cli fleet <csv>``: one AE per car of the reference CSV, saved as Keras HDF5."""
    import json
    import os

    from streamml.cli.__main__ import main
    from streamml.data.cardata import load_csv
    from streamml.models.autoencoder import load_model

    csv = os.path.join(os.path.dirname(__file__), "fixtures", "car-sensor-data.csv")
    out = tmp_path / "fleet"
    assert main(["fleet", csv, "--epochs", "2", "--out", str(out)]) == 0
    index = json.loads((out / "index.json").read_text())
    _, _, cars = load_csv(csv)
    assert sorted(index) == sorted(set(cars.tolist()))
    for name, rec in index.items():
        assert rec["keys"] == [name] and np.isfinite(rec["loss"])
    m = load_model(str(out / index[cars[0]]["file"]), device="cpu")
    assert len(m.get_weights()) == 8


def test_ragged_fleet_each_model_its_own_epoch(cuda_device):
    """Ragged rings: models of different sizes in one flat array, each taking
    its own number of steps per epoch -- model b equals a lone FusedAE on its own rows."""
    from streamml.data.cardata import normalize_affine
    from streamml.models.reference import init_dense_weights
    from streamml.ops.ae import AESpec, FusedAE
    from streamml.ops.ae_fleet import AEFleet, ragged_rings_by_key
    spec = AESpec()
    sc, sh = normalize_affine()
    rng = np.random.default_rng(0)
    sizes = [32 * 3, 32 * 10 + 5, 40]
    keys = np.concatenate([[f"car{i}"] * n for i, n in enumerate(sizes)])
    raw = rng.uniform(0, 40, (len(keys), 18)).astype(np.float32)
    flat, table, members = ragged_rings_by_key(raw, keys, batch=32)
    fleet = AEFleet.from_seeds(spec, [7, 8, 9], cuda_device, scale=sc, shift=sh)
    fleet.attach_ragged(torch.from_numpy(flat).to(cuda_device), 32, table)
    fleet.train_epoch(2)
    torch.cuda.synchronize()
    steps = fleet.epoch_steps() * 2
    np.testing.assert_array_equal(fleet.iter.cpu().numpy(), steps)
    for b in range(3):
        ring = torch.from_numpy(flat[table[b, 0]:table[b, 0] + table[b, 1]]).to(cuda_device)
        one = FusedAE(spec, init_dense_weights(spec.layer_sizes, seed=7 + b), cuda_device, scale=sc, shift=sh)
        one.attach_ring(ring, 32)
        one.train_minibatches(int(steps[b]))
        torch.cuda.synchronize()
        np.testing.assert_array_equal(fleet.params[b].cpu().numpy(), one.params.cpu().numpy())
        assert fleet.read_metrics()[b]["rows"] == steps[b] * 32
