"""C14 model store + C16 evaluation: parity vs scikit-learn 1.7 (installed here)."""
import os

import numpy as np
import pytest

from streamml.utils import evaluation as ev
from streamml.utils.model_store import LocalDirStore, autoencoder_store, lstm_store, open_store


def _scores(n=4000, seed=0, ties=False):
    rng = np.random.default_rng(seed)
    y = (rng.random(n) < 0.05).astype(int)
    s = rng.gamma(2.0, 1.0, n) + 3.0 * y
    if ties:
        s = np.round(s, 1)
    return y, s


@pytest.mark.parametrize("ties", [False, True])
def test_roc_pr_match_sklearn(ties):
    sk = pytest.importorskip("sklearn.metrics")
    y, s = _scores(ties=ties)
    for drop in (True, False):
        a = ev.roc_curve(y, s, drop_intermediate=drop)
        b = sk.roc_curve(y, s, drop_intermediate=drop)
        for u, v in zip(a, b):
            np.testing.assert_allclose(u, v)
    assert ev.auc(*ev.roc_curve(y, s)[:2]) == pytest.approx(sk.roc_auc_score(y, s), abs=1e-12)
    assert ev.roc_auc_score(y, s) == pytest.approx(sk.roc_auc_score(y, s), abs=1e-12)
    for u, v in zip(ev.precision_recall_curve(y, s), sk.precision_recall_curve(y, s)):
        np.testing.assert_allclose(u, v)
    pred = (s > 5).astype(int)
    np.testing.assert_array_equal(ev.confusion_matrix(y, pred), sk.confusion_matrix(y, pred))


def test_roc_auc_torch_matches():
    sk = pytest.importorskip("sklearn.metrics")
    y, s = _scores(ties=True)
    assert ev.roc_auc_torch(y, s) == pytest.approx(sk.roc_auc_score(y, s), abs=1e-9)


def test_split_and_scaler_match_sklearn():
    pre = pytest.importorskip("sklearn.preprocessing")
    ms = pytest.importorskip("sklearn.model_selection")
    x = np.random.default_rng(1).normal(3, 2, size=(1001, 3))
    a = ev.train_test_split(x, test_size=0.2, random_state=314)
    b = ms.train_test_split(x, test_size=0.2, random_state=314)
    for u, v in zip(a, b):
        np.testing.assert_array_equal(u, v)
    np.testing.assert_allclose(ev.StandardScaler().fit_transform(x), pre.StandardScaler().fit_transform(x))
    col = x[:, :1]
    sc = ev.StandardScaler().fit(col)
    np.testing.assert_allclose(sc.inverse_transform(sc.transform(col)), col)


def test_classification_summary():
    y, s = _scores()
    rep = ev.classification_summary(y, s, threshold=5.0)
    assert set(rep) >= {"confusion", "precision", "recall", "roc_auc"}
    assert np.sum(rep["confusion"]) == len(y)


def test_local_store_roundtrip(tmp_path):
    src = tmp_path / "model.h5"
    src.write_bytes(b"\x89HDF\r\n\x1a\n" + os.urandom(1000))
    st = autoencoder_store("proj", str(tmp_path / "store"))
    assert st.bucket == "tf-models_proj"
    url = st.upload(str(src), "/model.h5")          # reference passes "/" + model_file
    assert url.startswith("file://") and st.exists("model.h5")
    out = tmp_path / "dl" / "m.h5"
    st.download("/model.h5", str(out))
    assert out.read_bytes() == src.read_bytes()
    assert st.list() == ["model.h5"]
    assert lstm_store(str(tmp_path / "store")).bucket == "car-demo-tensorflow-models"
    # corruption is detected
    with open(os.path.join(st.dir, "model.h5"), "ab") as f:
        f.write(b"x")
    with pytest.raises(IOError):
        st.download("model.h5", str(out))
    with pytest.raises(ValueError):
        st.upload(str(src), "../escape.h5")
    with pytest.raises(FileNotFoundError):
        st.download("missing.h5", str(out))


def test_gcs_store_reports_missing_dependency():
    try:
        import google.cloud.storage  # noqa: F401
        pytest.skip("google-cloud-storage installed")
    except ImportError:
        pass
    with pytest.raises(RuntimeError, match="google-cloud-storage"):
        open_store("bucket", "gs://")
    assert isinstance(open_store("b", "file:///tmp/x"), LocalDirStore)
