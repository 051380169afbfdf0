"""Keras-style callbacks used by the reference: ModelCheckpoint, TensorBoard,
the Kafka prediction sink (OutputCallback, cardata-v3.py:235-252) and a CSV/JSON
history logger.  Metrics are read from the device once per epoch, so callbacks
see epoch-level logs (per-step host syncs would stall the GPU pipeline)."""
from __future__ import annotations

import json
import math
import os
from typing import Dict, List, Optional

import numpy as np


class Callback:
    model = None

    def set_model(self, model) -> None:
        self.model = model

    def on_train_begin(self, logs: Optional[dict] = None): ...
    def on_train_end(self, logs: Optional[dict] = None): ...
    def on_epoch_begin(self, epoch: int, logs: Optional[dict] = None): ...
    def on_epoch_end(self, epoch: int, logs: Optional[dict] = None): ...
    def on_predict_batch_end(self, batch: int, logs: Optional[dict] = None): ...
    def on_predict_end(self, logs: Optional[dict] = None): ...


class History(Callback):
    def __init__(self):
        self.history: Dict[str, List[float]] = {}
        self.epoch: List[int] = []

    def on_epoch_end(self, epoch, logs=None):
        self.epoch.append(epoch)
        for k, v in (logs or {}).items():
            self.history.setdefault(k, []).append(v)


class ModelCheckpoint(Callback):
    """``ModelCheckpoint(filepath, monitor='val_loss', save_best_only=True)``
    (Fraud-Detection-Autoencoder.ipynb:862-864)."""

    def __init__(self, filepath: str, monitor: str = "val_loss", save_best_only: bool = False, mode: str = "min",
                 verbose: int = 0):
        self.filepath, self.monitor, self.save_best_only = filepath, monitor, save_best_only
        self.mode, self.verbose = mode, verbose
        self.best = math.inf if mode == "min" else -math.inf
        self.saved: List[str] = []

    def on_epoch_end(self, epoch, logs=None):
        logs = logs or {}
        path = self.filepath.format(epoch=epoch + 1, **logs)
        if self.save_best_only:
            cur = logs.get(self.monitor)
            if cur is None:
                cur = logs.get(self.monitor.replace("val_", ""))
            if cur is None:
                return
            better = cur < self.best if self.mode == "min" else cur > self.best
            if not better:
                return
            self.best = cur
        self.model.save(path)
        self.saved.append(path)
        if self.verbose:
            print(f"Epoch {epoch + 1}: saved model to {path}")


class TensorBoard(Callback):
    """Keras ``TensorBoard`` (TF 2.0 semantics; Fraud-Detection-Autoencoder.ipynb:866,
    confluent-tensorflow-io-kafka.py:54-55):

    * ``epoch_<metric>`` scalars to ``log_dir/train`` and ``log_dir/validation`` (the TF2 tag
      layout decoded from the reference logs);
    * ``histogram_freq=k``: every k-th epoch, one histogram per weight, tagged as TF2 does
      (``dense/kernel_0``: the weight name with ':' -> '_'), in ``train``;
    * ``write_images``: with the histograms, each weight as a grayscale image
      (``<weight>/image``; kernels [in, out], vectors one row);
    * ``write_graph``: the ``keras`` model summary (the model-config JSON as a string tensor,
      plugin ``graph_keras_model``), written once in ``train`` at step 0.  There is no
      TensorFlow graph to serialise: the model runs as HIP kernels;
    * ``update_freq`` other than ``'epoch'`` and a non-zero ``profile_batch`` are accepted
      with a warning and not honoured: logs are epoch-level (metrics are read from the device
      once per epoch), and kernels are profiled with rocprofv3 (``streamml.obs.profile``)."""

    def __init__(self, log_dir: str = "./logs", histogram_freq: int = 0, write_graph: bool = True,
                 write_images: bool = False, update_freq="epoch", profile_batch=None, embeddings_freq: int = 0,
                 embeddings_metadata=None, **unknown):
        import warnings
        if unknown:
            raise TypeError(f"TensorBoard: unexpected arguments {sorted(unknown)}")
        self.log_dir = log_dir
        self.histogram_freq = int(histogram_freq or 0)
        self.write_graph = bool(write_graph)
        self.write_images = bool(write_images)
        if update_freq != "epoch":
            warnings.warn("TensorBoard(update_freq=...): logs are written per epoch (metrics are read from the "
                          "device once per epoch)", stacklevel=2)
        if profile_batch:   # TF's default (2) is left unset here: only an explicit request warns
            warnings.warn("TensorBoard(profile_batch=...): not traced here; profile kernels with rocprofv3 "
                          "(streamml.obs.profile)", stacklevel=2)
        if embeddings_freq:
            warnings.warn("TensorBoard(embeddings_freq=...): no embedding layers; ignored", stacklevel=2)
        self._w = {}
        self._graph_written = False

    def _writer(self, split: str):
        from ..obs.tfevents import EventFileWriter
        if split not in self._w:
            self._w[split] = EventFileWriter(os.path.join(self.log_dir, split))
        return self._w[split]

    def on_train_begin(self, logs=None):
        if self.write_graph and not self._graph_written and hasattr(self.model, "model_config"):
            self._writer("train").text_tensor("keras", json.dumps(self.model.model_config()), 0,
                                              plugin="graph_keras_model", content=b"1")
            self._graph_written = True

    def on_epoch_end(self, epoch, logs=None):
        for k, v in (logs or {}).items():
            if k.startswith("val_"):
                self._writer("validation").scalar("epoch_" + k[4:], v, epoch)
            elif not k.startswith("_"):
                self._writer("train").scalar("epoch_" + k, v, epoch)
        if self.histogram_freq and epoch % self.histogram_freq == 0:
            w = self._writer("train")
            for name, arr in named_weights(self.model):
                tag = name.replace(":", "_")
                w.histogram(tag, arr, epoch)
                if self.write_images:
                    a = np.asarray(arr)
                    w.image(tag + "/image", a.reshape(1, -1) if a.ndim == 1 else a.reshape(a.shape[0], -1), epoch)
        for w in self._w.values():
            w.flush()

    def on_train_end(self, logs=None):
        for w in self._w.values():
            w.close()
        self._w = {}


def named_weights(model):
    """[(Keras weight name, array)] of a model: 'dense/kernel:0', 'lstm/recurrent_kernel:0', ..."""
    ws = [np.asarray(a) for a in (model.get_weights() if hasattr(model, "get_weights") else model.fp.get())]
    names = getattr(model, "weight_names", None)
    if callable(names):
        names = [n for _, ns in names() for n in ns]
    if names is None and hasattr(model, "_layer_names"):
        names = [f"{ln}/{k}:0" for ln in model._layer_names() for k in ("kernel", "bias")]
    if not names or len(names) != len(ws):
        names = [f"weight_{i}:0" for i in range(len(ws))]
    return list(zip(names, ws))


class JSONLogger(Callback):
    def __init__(self, path: str):
        self.path = path

    def on_epoch_end(self, epoch, logs=None):
        with open(self.path, "a") as f:
            f.write(json.dumps({"epoch": epoch, **(logs or {})}) + "\n")


class KafkaPredictionSink(Callback):
    """Reference ``OutputCallback``: every predicted row is formatted with
    ``np.array2string`` and written at index ``batch * batch_size + i`` to a
    ``KafkaOutputSequence`` (cardata-v3.py:235-252); ``flush()`` at the end.
    Optionally appends the anomaly score (the reference emits reconstructions only)."""

    def __init__(self, batch_size: int, topic: str, servers: str, configuration=None, with_score: bool = False,
                 partition: int = 0):
        from ..kafka import KafkaOutputSequence
        self.batch_size = int(batch_size)
        self.with_score = with_score
        self.sequence = KafkaOutputSequence(topic, servers, configuration, partition=partition)
        self.count = 0

    def on_predict_batch_end(self, batch, logs=None):
        outputs = logs["outputs"]
        scores = logs.get("scores")
        index = batch * self.batch_size
        for i, row in enumerate(np.asarray(outputs)):
            msg = np.array2string(row)
            if self.with_score and scores is not None:
                msg = json.dumps({"reconstruction": msg, "score": float(scores[i])})
            self.sequence.setitem(index, msg)
            index += 1
            self.count += 1

    def flush(self):
        self.sequence.flush()

    def on_predict_end(self, logs=None):
        self.flush()


class EarlyStopping(Callback):
    def __init__(self, monitor: str = "val_loss", patience: int = 0, min_delta: float = 0.0):
        self.monitor, self.patience, self.min_delta = monitor, patience, min_delta
        self.best, self.wait, self.stopped_epoch = math.inf, 0, None

    def on_epoch_end(self, epoch, logs=None):
        cur = (logs or {}).get(self.monitor)
        if cur is None:
            return
        if cur < self.best - self.min_delta:
            self.best, self.wait = cur, 0
        else:
            self.wait += 1
            if self.wait > self.patience:
                self.model.stop_training = True
                self.stopped_epoch = epoch
