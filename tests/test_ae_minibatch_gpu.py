"""Persistent small-batch AE trainer (csrc/kernels/ae_minibatch.hip) vs a plain PyTorch
fp32 run of the same Keras steps (batch 32, one Adam update per batch).

The kernel is fp32 end to end, so after many steps the parameters must agree with the
torch oracle to summation-order rounding (no bf16 envelope as in test_ae_kernel_gpu)."""
import numpy as np
import pytest
import torch

from streamml.data.cardata import normalize_affine
from streamml.models.reference import TorchAE, init_dense_weights
from streamml.ops.ae import AESpec, FusedAE

pytestmark = pytest.mark.gpu


def _weights(spec, seed):
    w = init_dense_weights(spec.layer_sizes, seed=seed)
    rng = np.random.default_rng(seed + 1)
    for i in range(1, 8, 2):
        w[i] = rng.uniform(-0.2, 0.2, size=w[i].shape).astype(np.float32)
    return w


def _oracle(spec, w, xn, B, nsteps):
    ref = TorchAE(spec.layer_sizes, spec.activations, spec.activity_l1, w)
    n = xn.shape[0]
    for s in range(nsteps):
        r0 = (s * B) % n
        ref.step(torch.from_numpy(xn[r0:r0 + B]))
    return ref


REF_ACTS = ("tanh", "relu", "tanh", "relu")


@pytest.mark.parametrize("D,B,nsteps,launches,acts", [
    (18, 32, 50, 1, REF_ACTS), (18, 32, 64, 4, REF_ACTS), (30, 32, 40, 2, REF_ACTS), (18, 48, 30, 1, REF_ACTS),
    (18, 7, 25, 1, REF_ACTS), (18, 100, 30, 2, REF_ACTS), (18, 128, 20, 1, REF_ACTS), (18, 77, 12, 1, REF_ACTS),
    (30, 100, 16, 1, REF_ACTS),
    (18, 32, 30, 1, ("sigmoid", "linear", "relu", "sigmoid")),   # runtime-activation instantiation
    (11, 20, 30, 3, ("relu", "tanh", "linear", "tanh")),
])
def test_minibatch_steps_match_torch(cuda_device, D, B, nsteps, launches, acts):
    spec = AESpec(input_dim=D, activations=acts)
    w = _weights(spec, seed=11)
    rng = np.random.default_rng(3)
    ring_rows = B * 20                       # wraps for nsteps > 20
    raw = rng.uniform(0, 40, size=(ring_rows, D)).astype(np.float32)
    if D == 18 and acts == REF_ACTS:
        scale, shift = normalize_affine()
    else:
        scale = (np.full(D, 1 / 40.0)).astype(np.float32)
        shift = np.zeros(D, np.float32)
    xn = (raw * scale + shift).astype(np.float32)

    fused = FusedAE(spec, w, cuda_device, scale=scale, shift=shift)
    fused.attach_ring(torch.from_numpy(raw).to(cuda_device), B)
    per = nsteps // launches
    for _ in range(launches):
        fused.train_minibatches(per)
    torch.cuda.synchronize()
    ref = _oracle(spec, w, xn, B, per * launches)

    assert int(fused.iter.item()) == per * launches
    assert int(fused.cursor.item()) == (per * launches * B) % ring_rows
    for got, want in zip(fused.get_weights(), ref.get_weights()):
        assert got.shape == want.shape
        np.testing.assert_allclose(got, want, rtol=2e-4, atol=2e-5)
    it, m, v = fused.get_optimizer_state()
    for got, want in zip(m, ref.opt.m):
        np.testing.assert_allclose(got, want.numpy(), rtol=2e-3, atol=1e-6)

    mt = fused.read_metrics()
    rm = ref.read_metrics()
    assert mt["rows"] == per * launches * B
    assert abs(mt["loss"] - rm["loss"]) <= 1e-4 * max(1.0, abs(rm["loss"]))
    assert abs(mt["accuracy"] - rm["accuracy"]) < 1e-6


def test_minibatch_matches_launch_per_step_path(cuda_device):
    """Same stream through train_minibatches and step_ring (bf16 MFMA path): close, not equal."""
    spec = AESpec()
    w = _weights(spec, seed=4)
    scale, shift = normalize_affine()
    raw = torch.rand((32 * 16, 18), device=cuda_device) * 40.0
    a = FusedAE(spec, w, cuda_device, scale=scale, shift=shift)
    b = FusedAE(spec, w, cuda_device, scale=scale, shift=shift)
    a.attach_ring(raw, 32)
    b.attach_ring(raw, 32)
    a.train_minibatches(16)
    for _ in range(16):
        b.step_ring()
    torch.cuda.synchronize()
    for ga, gb in zip(a.get_weights(), b.get_weights()):
        assert np.max(np.abs(ga - gb)) < 2 * 1e-3 * 16   # Adam moves each weight <= ~lr per step
    assert int(a.cursor.item()) == int(b.cursor.item()) == 0


def test_minibatch_rejects_bad_batch(cuda_device):
    spec = AESpec()
    fused = FusedAE(spec, init_dense_weights(spec.layer_sizes, seed=0), cuda_device)
    fused.attach_ring(torch.zeros((129 * 4, 18), device=cuda_device), 129)
    with pytest.raises(ValueError):
        fused.train_minibatches(2)


@pytest.mark.parametrize("B,models,D", [(32, 1, 18), (32, 6, 18), (32, 1, 30), (32, 3, 30)])
def test_pipelined_build_bit_identical_to_barrier_kernel(cuda_device, monkeypatch, B, models, D):
    """Keras batch 32 on the reference stack runs the pipelined build (the six parameter tiles
    on their own waves, LDS stage counters instead of the two barriers per step).  Same
    arithmetic in the same order as the two-barrier kernel (SML_MB_PIPE=0): bit-identical
    parameters, moments, cursor and metrics, alone and as a fleet (one model per workgroup);
    for the cardata model (D = 18) and the BASELINE row's creditcard model (D = 30)."""
    from streamml.ops.ae_fleet import AEFleet

    spec = AESpec(D, 14, 7)
    scale, shift = normalize_affine() if D == 18 else (None, None)
    g = torch.Generator(device="cpu").manual_seed(5)
    rings = (torch.rand((models, B * 24, D), generator=g) * (40.0 if D == 18 else 2.0)).to(cuda_device)
    ws = [_weights(spec, seed=20 + i) for i in range(models)]
    runs = []
    for pipe in ("1", "0"):
        monkeypatch.setenv("SML_MB_PIPE", pipe)
        if models == 1:
            ae = FusedAE(spec, ws[0], cuda_device, scale=scale, shift=shift)
            ae.attach_ring(rings[0].contiguous(), B)
        else:
            ae = AEFleet(spec, ws, cuda_device, lr=np.float32(2e-3), scale=scale, shift=shift)
            ae.attach_rings(rings, B)
        ae.train_minibatches(50)
        ae.train_minibatches(37)   # 87 steps: the 24-batch ring wraps, the counters restart per launch
        torch.cuda.synchronize()
        runs.append((ae.params.clone(), ae.m.clone(), ae.v.clone(), ae.cursor.clone(), ae.iter.clone(),
                     ae.read_metrics()))
    (p1, m1, v1, c1, i1, r1), (p0, m0, v0, c0, i0, r0) = runs
    assert torch.equal(p1, p0) and torch.equal(m1, m0) and torch.equal(v1, v0)
    assert torch.equal(c1, c0) and torch.equal(i1, i0)
    assert r1 == r0


@pytest.mark.parametrize("D,B", [(18, 100), (18, 32), (30, 32), (18, 7)])
def test_bf16_phase_a_close_to_fp32(cuda_device, monkeypatch, D, B):
    """SML_MB_BF16=1: phase A's forward / activation-gradient contractions on bf16 MFMAs
    (fp32 accumulation, fp32 weight gradients and Adam).  400 steps from one init stay within
    a few percent of the fp32 kernel's parameters and the same loss to 1e-3 -- and are NOT
    bit-identical (the bf16 path really ran)."""
    spec = AESpec(D, 14, 7)
    if D == 18:
        scale, shift = normalize_affine()
        ring = (torch.rand((B * 40, D), generator=torch.Generator().manual_seed(2)) * 40.0).to(cuda_device)
    else:
        scale = shift = None
        ring = torch.randn((B * 40, D), generator=torch.Generator().manual_seed(2)).to(cuda_device)
    out = {}
    for bf in ("0", "1"):
        monkeypatch.setenv("SML_MB_BF16", bf)
        ae = FusedAE(spec, _weights(spec, seed=3), cuda_device, scale=scale, shift=shift)
        ae.attach_ring(ring, B)
        ae.train_minibatches(400)
        torch.cuda.synchronize()
        out[bf] = (ae.params.clone(), ae.read_metrics())
    (p0, m0), (p1, m1) = out["0"], out["1"]
    assert not torch.equal(p0, p1)
    assert ((p1 - p0).norm() / p0.norm()).item() < 3e-2
    assert abs(m1["loss"] - m0["loss"]) <= 1e-3 * abs(m0["loss"]) + 1e-6


def test_bf16_pipelined_build_bit_identical_to_barrier_kernel(cuda_device, monkeypatch):
    """Under SML_MB_BF16=1 the batch-32 pipelined build and the barrier kernel run the same bf16
    contractions in the same order: bit-identical parameters and metrics."""
    spec = AESpec()
    scale, shift = normalize_affine()
    ring = (torch.rand((32 * 24, 18), generator=torch.Generator().manual_seed(5)) * 40.0).to(cuda_device)
    monkeypatch.setenv("SML_MB_BF16", "1")
    runs = []
    for pipe in ("1", "0"):
        monkeypatch.setenv("SML_MB_PIPE", pipe)
        ae = FusedAE(spec, _weights(spec, seed=21), cuda_device, scale=scale, shift=shift)
        ae.attach_ring(ring, 32)
        ae.train_minibatches(87)
        torch.cuda.synchronize()
        runs.append((ae.params.clone(), ae.m.clone(), ae.v.clone(), ae.read_metrics()))
    (p1, m1, v1, r1), (p0, m0, v0, r0) = runs
    assert torch.equal(p1, p0) and torch.equal(m1, m0) and torch.equal(v1, v0)
    assert r1 == r0


def test_autoencoder_minibatch_precision_option(cuda_device, monkeypatch):
    """Autoencoder.compile(minibatch_precision="bf16") trains fit(batch_size=100) on the bf16
    contractions (close to, not equal to, the fp32 model) and leaves the process default alone."""
    from streamml.models.autoencoder import Autoencoder
    monkeypatch.delenv("SML_MB_BF16", raising=False)
    x = np.random.default_rng(0).uniform(-1, 1, size=(20000, 18)).astype(np.float32)
    ws = {}
    for prec in ("fp32", "bf16"):
        m = Autoencoder(device=cuda_device, seed=4)
        m.compile(minibatch_precision=prec)
        h = m.fit(x, epochs=2, batch_size=100, verbose=0)
        assert h.history["loss"][-1] < h.history["loss"][0]
        ws[prec] = np.concatenate([w.ravel() for w in m.get_weights()])
    import os
    assert "SML_MB_BF16" not in os.environ
    assert not np.array_equal(ws["fp32"], ws["bf16"])
    assert np.linalg.norm(ws["bf16"] - ws["fp32"]) / np.linalg.norm(ws["fp32"]) < 3e-2
    # the choice travels with the model's launches: an explicit "fp32" ignores the
    # process default, an unset precision follows it
    monkeypatch.setenv("SML_MB_BF16", "1")
    for prec, want in (("fp32", "fp32"), (None, "bf16")):
        m = Autoencoder(device=cuda_device, seed=4)
        m.compile(minibatch_precision=prec)
        m.fit(x, epochs=2, batch_size=100, verbose=0)
        np.testing.assert_array_equal(np.concatenate([w.ravel() for w in m.get_weights()]), ws[want])
