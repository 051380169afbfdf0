"""Numerics of the fused AE HIP kernels vs a plain PyTorch fp32 reference."""
import numpy as np
import pytest
import torch

from streamml.data.cardata import normalize_affine
from streamml.models.reference import KerasAdam, ae_forward_torch, ae_loss_torch, init_dense_weights
from streamml.ops.ae import AESpec, FusedAE, pack_image, unpack_image

pytestmark = pytest.mark.gpu


def _weights(spec, seed=0, bias=True):
    w = init_dense_weights(spec.layer_sizes, seed=seed)
    if bias:
        rng = np.random.default_rng(seed + 1)
        for i in range(1, 8, 2):
            w[i] = rng.uniform(-0.2, 0.2, size=w[i].shape).astype(np.float32)
    return w


def _relerr(a, b):
    a = np.asarray(a, dtype=np.float64)
    b = np.asarray(b, dtype=np.float64)
    return np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-12)


@pytest.mark.parametrize("D,n", [(18, 1000), (18, 4096), (30, 777)])
def test_gradients_match_torch(cuda_device, D, n):
    spec = AESpec(input_dim=D)
    w = _weights(spec)
    rng = np.random.default_rng(5)
    x = rng.uniform(-1, 1, size=(n, D)).astype(np.float32)
    fused = FusedAE(spec, w, cuda_device, max_blocks=64)
    g_fused, metr = fused.gradients(torch.from_numpy(x).to(cuda_device))
    wt = [torch.tensor(a, dtype=torch.float32, requires_grad=True) for a in w]
    xt = torch.from_numpy(x)
    loss, mse, acc = ae_loss_torch(xt, wt, spec.activations, spec.activity_l1)
    g_ref = torch.autograd.grad(loss, wt)
    for gf, gr in zip(g_fused, g_ref):
        assert gf.shape == tuple(gr.shape)
        assert _relerr(gf, gr.numpy()) < 3e-2, (gf, gr)
    sq, ab, corr, rows = metr
    assert rows == n
    assert abs(sq / (n * D) - float(mse)) / float(mse) < 2e-2
    assert abs(corr / n - float(acc)) < 0.03


def test_training_trajectory_matches_torch(cuda_device):
    spec = AESpec()
    w = _weights(spec, seed=3)
    scale, shift = normalize_affine()
    rng = np.random.default_rng(7)
    raw =(rng.uniform(0, 1, size=(4 * 512, 18)) * 40).astype(np.float32)
    xn = (raw * scale + shift).astype(np.float32)
    fused = FusedAE(spec, w, cuda_device, max_blocks=32, scale=scale, shift=shift)
    ref_w = [torch.tensor(a, requires_grad=True) for a in w]
    opt = KerasAdam(ref_w)
    xr_dev = torch.from_numpy(raw).to(cuda_device)
    for s in range(4):
        fused.step(xr_dev[s * 512:(s + 1) * 512])
        xb = torch.from_numpy(xn[s * 512:(s + 1) * 512])
        loss, _, _ = ae_loss_torch(xb, ref_w, spec.activations, spec.activity_l1)
        opt.apply(torch.autograd.grad(loss, ref_w))
    torch.cuda.synchronize()
    got = fused.get_weights()
    assert int(fused.iter.item()) == 4
    for a, b in zip(got, ref_w):
        # Adam steps are ~lr-sized; compare the parameter deltas
        assert np.max(np.abs(a - b.detach().numpy())) < 2e-4
    m = fused.read_metrics()
    assert m["rows"] == 4 * 512


def test_forward_and_score(cuda_device):
    spec = AESpec()
    w = _weights(spec, seed=11)
    rng = np.random.default_rng(2)
    n = 333
    x = rng.uniform(-1, 1, size=(n, 18)).astype(np.float32)
    fused = FusedAE(spec, w, cuda_device)
    r, s, f = fused.forward(torch.from_numpy(x).to(cuda_device), threshold=0.3)
    y, _ = ae_forward_torch(torch.from_numpy(x), [torch.from_numpy(a) for a in w], spec.activations)
    y = y.numpy()
    assert _relerr(r.cpu().numpy(), y) < 2e-2
    score_ref = ((y - x) ** 2).mean(axis=1)
    np.testing.assert_allclose(s.cpu().numpy(), score_ref, rtol=3e-2, atol=3e-3)
    agree = (f.cpu().numpy() == (score_ref > 0.3)).mean()
    assert agree > 0.97


def test_pack_roundtrip_on_device(cuda_device):
    spec = AESpec(input_dim=30)
    w = _weights(spec, seed=4)
    fused = FusedAE(spec, w, cuda_device)
    for a, b in zip(fused.get_weights(), w):
        np.testing.assert_array_equal(a, b)
    np.testing.assert_array_equal(unpack_image(pack_image(w), spec)[0], w[0])
