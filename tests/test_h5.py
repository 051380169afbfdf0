"""Native HDF5 codec: golden reads of the reference Keras files + write/read round trips."""
import os

import numpy as np
import pytest

from streamml.ckpt import h5

FIX = os.path.join(os.path.dirname(__file__), "fixtures")
F1 = os.path.join(FIX, "autoencoder_sensor_anomaly_detection.h5")
F2 = os.path.join(FIX, "autoencoder_sensor_anomaly_detection_fully_trained_100_epochs.h5")


def test_reference_file_golden_values():
    ck = h5.load_keras_h5(F1)
    assert ck.layer_names == ["input_1", "dense", "dense_1", "dense_2", "dense_3"]
    shapes = [a.shape for a in ck.flat_weights()]
    assert shapes == [(30, 14), (14,), (14, 7), (7,), (7, 7), (7,), (7, 30), (30,)]
    np.testing.assert_allclose(ck.weights["dense"][0][1][0, :4], [-0.05193, 0.03872, -0.81092, 0.02078], atol=1e-5)
    assert ck.optimizer_iterations == 35545
    assert ck.model_config["class_name"] == "Model"
    assert ck.training_config["loss"] == "mean_squared_error"
    assert ck.training_config["optimizer_config"]["config"]["epsilon"] == pytest.approx(1e-7)
    assert len(ck.optimizer_weights) == 17
    assert ck.keras_version == "2.2.4-tf"


def test_reference_quirk_weight_subgroup_name():
    ck = h5.load_keras_h5(F2)
    assert ck.layer_names[0] == "dense_4" or "dense_4" in ck.layer_names
    names = [n for n, _ in ck.weights["dense_4"]]
    assert names == ["dense_4_1/kernel:0", "dense_4_1/bias:0"]
    assert ck.optimizer_iterations == 167132
    assert ck.optimizer_weights[0][0] == "training_2/Adam/iter:0"


def test_resave_reference_roundtrip(tmp_path):
    ck = h5.load_keras_h5(F1)
    out = tmp_path / "resaved.h5"
    h5.save_keras_h5(str(out), ck.model_config, list(ck.weights.items()), ck.training_config, ck.optimizer_weights)
    ck2 = h5.load_keras_h5(str(out))
    assert ck2.layer_names == ck.layer_names
    assert ck2.model_config == ck.model_config and ck2.training_config == ck.training_config
    for (n1, a1), (n2, a2) in zip([w for ws in ck.weights.values() for w in ws],
                                  [w for ws in ck2.weights.values() for w in ws]):
        assert n1 == n2
        np.testing.assert_array_equal(a1, a2)
        assert a1.dtype == a2.dtype
    assert [n for n, _ in ck2.optimizer_weights] == [n for n, _ in ck.optimizer_weights]
    assert ck2.optimizer_iterations == 35545
    # raw structure: same groups / datasets / attribute kinds as the h5py-written original
    r1, r2 = h5.read(F1), h5.read(str(out))

    def walk(g, p=""):
        out = {}
        for k, c in g.children.items():
            if isinstance(c, h5.Group):
                out[p + k + "/"] = sorted(c.attrs)
                out.update(walk(c, p + k + "/"))
            else:
                out[p + k] = (c.value.dtype.str, c.value.shape)
        return out
    assert walk(r1) == walk(r2)
    assert sorted(r1.attrs) == sorted(r2.attrs)


def test_generic_roundtrip_many_children(tmp_path):
    root = h5.Group()
    root.attrs["title"] = "héllo"
    root.attrs["vec"] = np.arange(5, dtype=np.int32)
    root.attrs["names"] = np.array([b"a", b"bcd"], dtype="S3")
    g = root.require_group("many")
    rng = np.random.default_rng(0)
    for i in range(40):  # > 8 per symbol node, several SNODs
        g.create_dataset(f"d{i:02d}", rng.standard_normal((3, i % 5 + 1)).astype(np.float32))
    root.create_dataset("deep/er/x", np.float64(3.5))
    root.create_dataset("ints", np.arange(7, dtype=np.int64))
    p = tmp_path / "t.h5"
    h5.write(str(p), root)
    back = h5.read(str(p))
    assert back.attrs["title"] == "héllo"
    np.testing.assert_array_equal(back.attrs["vec"], np.arange(5))
    assert list(back.attrs["names"]) == [b"a", b"bcd"]
    assert sorted(back["many"].children) == sorted(g.children)
    for k, d in g.children.items():
        np.testing.assert_array_equal(back["many"][k].value, d.value)
    assert float(back["deep/er/x"].value) == 3.5
    np.testing.assert_array_equal(back["ints"].value, np.arange(7))


def test_corrupt_files_raise(tmp_path):
    from streamml.ops import load_io
    io = load_io()
    data = open(F1, "rb").read()
    for cut in (10, 100, 1000, 20000):
        with pytest.raises(Exception):
            io.h5_read_bytes(data[:cut])
    with pytest.raises(Exception):
        io.h5_read_bytes(b"not an hdf5 file at all" * 10)
