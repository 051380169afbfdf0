"""MNIST family (C10 / K13 / C17 raw-byte producer): CPU path + Kafka round trip."""
import numpy as np
import pytest
import torch

from streamml.data import mnist as mn
from streamml.models.mlp import MLPClassifier, softmax_xent_reference


def test_softmax_xent_reference_matches_autograd():
    g = torch.Generator().manual_seed(0)
    z = torch.randn(37, 10, generator=g, requires_grad=True)
    y = torch.randint(0, 10, (37,), generator=g)
    loss = torch.nn.functional.cross_entropy(z, y, reduction="sum")
    loss.backward()
    l2, corr, d = softmax_xent_reference(z.detach(), y)
    assert float(l2) == pytest.approx(float(loss.detach()), rel=1e-6)
    assert int(corr) == int((z.argmax(1) == y).sum())
    torch.testing.assert_close(d, z.grad)


def test_synthetic_mnist_shapes_and_determinism():
    x, y = mn.synthetic_mnist(500, seed=3)
    assert x.shape == (500, 28, 28) and x.dtype == np.uint8 and y.dtype == np.uint8
    x2, y2 = mn.synthetic_mnist(500, seed=3)
    np.testing.assert_array_equal(x, x2)
    assert set(np.unique(y)) <= set(range(10))


def test_idx_roundtrip(tmp_path):
    x, y = mn.synthetic_mnist(20)
    for name, arr in (("train-images-idx3-ubyte.gz", x), ("train-labels-idx1-ubyte", y),
                      ("t10k-images-idx3-ubyte", x[:5]), ("t10k-labels-idx1-ubyte.gz", y[:5])):
        mn.write_idx(str(tmp_path / name), arr)
    (a, b), (c, d) = mn.load_mnist(str(tmp_path))
    np.testing.assert_array_equal(a, x)
    np.testing.assert_array_equal(d, y[:5])
    with pytest.raises(ValueError):
        (tmp_path / "bad").write_bytes(b"\x01\x02\x03\x04")
        mn.load_idx(str(tmp_path / "bad"))


def test_mlp_cpu_learns_and_roundtrips(tmp_path):
    (xtr, ytr), (xte, yte) = mn.load_mnist(n_synthetic=3000)
    m = MLPClassifier(hidden=64, device="cpu", seed=1)
    assert m.count_params() == 784 * 64 + 64 + 64 * 10 + 10
    h = m.fit(xtr, ytr, epochs=3, batch_size=32, validation_data=(xte, yte), verbose=0)
    assert h.history["loss"][-1] < h.history["loss"][0]
    assert h.history["val_accuracy"][-1] > 0.9
    p = m.predict(xte[:50])
    np.testing.assert_allclose(p.sum(1), 1.0, rtol=1e-5)
    path = str(tmp_path / "mnist.h5")
    m.save(path)
    m2 = MLPClassifier.load(path, device="cpu")
    np.testing.assert_allclose(m2.predict(xte[:50]), p, rtol=1e-5, atol=1e-6)
    assert m2.opt.state()[0] == m.opt.state()[0]


def test_mlp_dropout_variant_config(tmp_path):
    m = MLPClassifier(hidden=512, dropout=0.2, device="cpu")
    x, y = mn.synthetic_mnist(256)
    m.fit(x, y, epochs=1, batch_size=32, verbose=0)
    path = str(tmp_path / "d.h5")
    m.save(path)
    m2 = MLPClassifier.load(path, device="cpu")
    assert m2.dropout == pytest.approx(0.2) and m2.hidden == 512
    kinds = [l["class_name"] for l in m.model_config()["config"]["layers"]]
    assert kinds == ["Flatten", "Dense", "Dropout", "Dense"]


def test_mnist_over_fake_kafka():
    x, y = mn.synthetic_mnist(3000, seed=5)
    srv = "fake://mnist-test"
    assert mn.produce_mnist(srv, x, y) == 3000
    got_x, got_y = [], []
    for cx, cy in mn.kafka_mnist(srv):
        got_x.append(cx)
        got_y.append(cy)
    np.testing.assert_array_equal(np.concatenate(got_x), x)
    np.testing.assert_array_equal(np.concatenate(got_y), y)
    m = MLPClassifier(hidden=32, device="cpu")
    h = m.fit(stream=lambda: mn.kafka_mnist(srv), epochs=1, batch_size=1, steps_per_epoch=200, verbose=0)
    assert h.history["loss"][0] > 0
