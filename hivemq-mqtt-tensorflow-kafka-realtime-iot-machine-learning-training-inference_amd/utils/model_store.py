"""Model store: where trained ``.h5`` files go between the train and predict jobs.

The reference uploads the checkpoint to a Google Cloud Storage bucket after
training and downloads it again before predicting:

* autoencoder: bucket ``tf-models_<project>`` (AUTOENCODER-TensorFlow-IO-Kafka/cardata-v3.py:39-41,
  upload :229-232, download :255-258), object name ``"/" + model_file``;
* LSTM: bucket ``car-demo-tensorflow-models`` (LSTM-TensorFlow-IO-Kafka/cardata-v2.py:19-21,
  upload :213-217, download :240-243), object name ``model_file``.

Here a store is addressed by URL:

* ``file:///some/dir`` or a plain path  -> :class:`LocalDirStore` (one sub-directory per bucket);
* ``gs://``                              -> :class:`GCSStore` (needs ``google-cloud-storage``,
  which is not part of this image: constructing it raises a clear error).

``SML_MODEL_STORE`` picks the default root (``~/.streamml/model-store``).
Writes are atomic (temp file + ``os.replace``) so a predict job never sees a
half-written checkpoint from a concurrent train job.
"""
from __future__ import annotations

import hashlib
import json
import os
import shutil
import tempfile
from typing import List, Optional

DEFAULT_ROOT = os.path.join(os.path.expanduser("~"), ".streamml", "model-store")
AE_BUCKET_PREFIX = "tf-models_"
LSTM_BUCKET = "car-demo-tensorflow-models"


def _clean(name: str) -> str:
    """Object names may carry the reference's leading '/' ("/" + model_file)."""
    name = name.replace("\\", "/").lstrip("/")
    parts = [p for p in name.split("/") if p not in ("", ".")]
    if any(p == ".." for p in parts) or not parts:
        raise ValueError(f"invalid object name {name!r}")
    return "/".join(parts)


def _sha256(path: str) -> str:
    h = hashlib.sha256()
    with open(path, "rb") as f:
        for blk in iter(lambda: f.read(1 << 20), b""):
            h.update(blk)
    return h.hexdigest()


class ModelStore:
    bucket: str

    def upload(self, local_path: str, name: str) -> str:
        raise NotImplementedError

    def download(self, name: str, local_path: str) -> str:
        raise NotImplementedError

    def exists(self, name: str) -> bool:
        raise NotImplementedError

    def list(self) -> List[str]:
        raise NotImplementedError


class LocalDirStore(ModelStore):
    """A directory acting as a bucket; a ``.meta.json`` sidecar records size + sha256."""

    def __init__(self, root: str, bucket: str):
        self.root = os.path.abspath(os.path.expanduser(root))
        self.bucket = bucket
        self.dir = os.path.join(self.root, bucket)

    def _path(self, name: str) -> str:
        return os.path.join(self.dir, _clean(name))

    def upload(self, local_path: str, name: str) -> str:
        dst = self._path(name)
        os.makedirs(os.path.dirname(dst), exist_ok=True)
        fd, tmp = tempfile.mkstemp(dir=os.path.dirname(dst), prefix=".upload-")
        os.close(fd)
        try:
            shutil.copyfile(local_path, tmp)
            os.replace(tmp, dst)
        finally:
            if os.path.exists(tmp):
                os.unlink(tmp)
        meta = {"size": os.path.getsize(dst), "sha256": _sha256(dst), "source": os.path.abspath(local_path)}
        with open(dst + ".meta.json", "w") as f:
            json.dump(meta, f)
        return f"file://{dst}"

    def download(self, name: str, local_path: str) -> str:
        src = self._path(name)
        if not os.path.exists(src):
            raise FileNotFoundError(f"{name!r} not in bucket {self.bucket!r} ({self.dir})")
        meta_path = src + ".meta.json"
        if os.path.exists(meta_path):
            with open(meta_path) as f:
                meta = json.load(f)
            if meta.get("sha256") and meta["sha256"] != _sha256(src):
                raise IOError(f"checksum mismatch for {src}")
        d = os.path.dirname(os.path.abspath(local_path))
        os.makedirs(d, exist_ok=True)
        if os.path.abspath(local_path) != os.path.abspath(src):
            fd, tmp = tempfile.mkstemp(dir=d, prefix=".download-")
            os.close(fd)
            shutil.copyfile(src, tmp)
            os.replace(tmp, local_path)
        return local_path

    def exists(self, name: str) -> bool:
        return os.path.exists(self._path(name))

    def list(self) -> List[str]:
        out = []
        for base, _, files in os.walk(self.dir):
            for f in files:
                if f.endswith(".meta.json") or f.startswith("."):
                    continue
                out.append(os.path.relpath(os.path.join(base, f), self.dir).replace(os.sep, "/"))
        return sorted(out)


class GCSStore(ModelStore):
    """Google Cloud Storage bucket (service-account JSON as in the reference)."""

    def __init__(self, bucket: str, credentials: Optional[str] = "/credentials/credentials.json"):
        try:
            from google.cloud import storage  # type: ignore
        except ImportError as e:  # not shipped in this image
            raise RuntimeError("gs:// model store needs google-cloud-storage, which is not installed; "
                               "use a file:// store (SML_MODEL_STORE)") from e
        client = (storage.Client.from_service_account_json(credentials)
                  if credentials and os.path.exists(credentials) else storage.Client())
        self.bucket = bucket
        self._b = client.get_bucket(bucket)

    def upload(self, local_path: str, name: str) -> str:
        self._b.blob(name).upload_from_filename(local_path)
        return f"gs://{self.bucket}/{name}"

    def download(self, name: str, local_path: str) -> str:
        self._b.blob(name).download_to_filename(local_path)
        return local_path

    def exists(self, name: str) -> bool:
        return self._b.blob(name).exists()

    def list(self) -> List[str]:
        return sorted(b.name for b in self._b.list_blobs())


def open_store(bucket: str, url: Optional[str] = None) -> ModelStore:
    url = url or os.environ.get("SML_MODEL_STORE", DEFAULT_ROOT)
    if url.startswith("gs://"):
        return GCSStore(bucket)
    if url.startswith("file://"):
        url = url[len("file://"):]
    return LocalDirStore(url, bucket)


def autoencoder_store(project: str, url: Optional[str] = None) -> ModelStore:
    """Bucket ``tf-models_<project>`` (cardata-v3.py:41)."""
    return open_store(AE_BUCKET_PREFIX + project, url)


def lstm_store(url: Optional[str] = None) -> ModelStore:
    """Bucket ``car-demo-tensorflow-models`` (LSTM-.../cardata-v2.py:21)."""
    return open_store(LSTM_BUCKET, url)
