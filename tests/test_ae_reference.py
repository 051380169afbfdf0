"""CPU tests: Keras-semantics AE reference, padded parameter image, normalisation."""
import numpy as np
import torch

from streamml.data.cardata import FEATURES, normalize_affine, normalize_np
from streamml.models.reference import KerasAdam, TorchAE, ae_loss_torch, init_dense_weights
from streamml.ops.ae import LAYOUT, NPARAM, AESpec, pack_image, unpack_image


def test_param_counts_match_reference():
    # 571 params (D=18) / 835 params (D=30)
    assert AESpec(input_dim=18).n_params == 571
    assert AESpec(input_dim=30).n_params == 835


def test_pack_unpack_roundtrip():
    for d in (18, 30):
        spec = AESpec(input_dim=d)
        w = init_dense_weights(spec.layer_sizes, seed=1)
        w[1] += 0.5
        img = pack_image(w)
        assert img.shape == (NPARAM,)
        back = unpack_image(img, spec)
        for a, b in zip(w, back):
            np.testing.assert_array_equal(a, b)
        # bias lands in the constant-1 row of each padded block
        off, ip, op, brow = LAYOUT[0]
        np.testing.assert_array_equal(img[off + brow * op: off + brow * op + 14], w[1])


def test_glorot_limits():
    w = init_dense_weights([(18, 14)], seed=0)
    lim = np.sqrt(6.0 / 32)
    assert np.abs(w[0]).max() <= lim and np.abs(w[0]).max() > 0.8 * lim
    assert (w[1] == 0).all()


def test_normalize_affine_matches_reference_formula():
    rng = np.random.default_rng(0)
    raw = rng.uniform(0, 3000, size=(64, 18)).astype(np.float32)
    scale, shift = normalize_affine()
    np.testing.assert_allclose(raw * scale + shift, normalize_np(raw), rtol=1e-6, atol=1e-6)
    zeroed = [FEATURES.index(n) for n in ("coolant_temp", "intake_air_flow_speed", "battery_voltage",
                                          "current_draw")]
    assert (scale[zeroed] == 0).all() and (shift[zeroed] == 0).all()
    # scale_fn(v, lo, hi) at the range ends -> -1, +1
    i = FEATURES.index("speed")
    assert abs(0 * scale[i] + shift[i] + 1) < 1e-12 and abs(50 * scale[i] + shift[i] - 1) < 1e-12


def test_keras_adam_matches_closed_form():
    p = torch.tensor([1.0, -2.0])
    opt = KerasAdam([p], lr=0.1)
    g = torch.tensor([0.5, -0.25])
    opt.apply([g])
    # first step: m = 0.1 g, v = 0.001 g^2, lr_t = 0.1*sqrt(0.001)/0.1
    lr_t = 0.1 * np.sqrt(1 - 0.999) / (1 - 0.9)
    exp = np.array([1.0, -2.0]) - lr_t * (0.1 * g.numpy()) / (np.sqrt(0.001 * g.numpy() ** 2) + 1e-7)
    np.testing.assert_allclose(p.numpy(), exp, rtol=1e-6)


def test_torch_ae_trains_on_cpu():
    spec = AESpec()
    ae = TorchAE(spec.layer_sizes, spec.activations, spec.activity_l1, init_dense_weights(spec.layer_sizes, 0))
    rng = np.random.default_rng(0)
    x = torch.from_numpy(rng.uniform(-0.5, 1, size=(512, 18)).astype(np.float32))
    l0 = float(ae_loss_torch(x, ae.w, spec.activations, spec.activity_l1)[0])
    for _ in range(60):
        for s in range(0, 512, 32):
            ae.step(x[s:s + 32])
    l1 = float(ae_loss_torch(x, ae.w, spec.activations, spec.activity_l1)[0])
    assert l1 < 0.7 * l0
    assert ae.opt.iterations == 60 * 16
