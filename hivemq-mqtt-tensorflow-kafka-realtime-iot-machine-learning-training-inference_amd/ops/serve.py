"""Persistent per-event scoring on the GPU (``csrc/kernels/ae_serve.hip``, ``lstm_serve.hip``).

``ScoringServer(model)`` keeps one wave resident on the device that polls a
host-mapped request ring; ``score(rows)`` publishes rows and spins on the
completion counter -- no kernel launch, no hipMemcpy per event.  This is the
low-latency path of BASELINE config 5 (the launch-per-event path is
``Autoencoder.score``).  The kernel exits by itself after ``idle_seconds``
without requests and is relaunched transparently on the next request.

``LSTMScoringServer(model)`` serves an :class:`~streamml.models.lstm.LSTMPredictor` the
same way, per car key: the device keeps each key's last ``look_back`` normalised events
and its latest forecast; every event is scored against the key's previous forecast (MSE)
and a forecast of the key's next event is returned (the reference's per-event LSTM
prediction stream, LSTM-TensorFlow-IO-Kafka/cardata-v2.py:220-273).
"""
from __future__ import annotations

from typing import Optional, Tuple

import numpy as np
import torch

from ._ext import load_c


class ScoringServer:
    def __init__(self, model, threshold: float = 5.0, slots: int = 4096, idle_seconds: float = 2.0,
                 device: Optional[torch.device] = None):
        dev = torch.device(device) if device is not None else model.device
        if dev.type != "cuda":
            raise RuntimeError("ScoringServer needs a ROCm device (use Autoencoder.score on CPU)")
        spec = model.spec
        ws = model.get_weights()
        flat = np.concatenate([np.asarray(w, np.float32).ravel() for w in ws])
        sc, sh = model._normalizer()
        self.D = spec.input_dim
        self.threshold = float(threshold)
        self._s = load_c().AEServe(dev.index if dev.index is not None else torch.cuda.current_device(), int(slots),
                                   flat, [spec.input_dim, spec.encoding_dim, spec.hidden_dim], list(spec.act_codes),
                                   None if sc is None else np.asarray(sc, np.float32),
                                   None if sh is None else np.asarray(sh, np.float32), float(threshold),
                                   float(idle_seconds))

    def score(self, rows) -> Tuple[np.ndarray, np.ndarray]:
        """(scores [k], anomaly flags [k]) for raw rows [k, D]."""
        s, f, _ = self._s.infer(np.ascontiguousarray(np.asarray(rows, np.float32).reshape(-1, self.D)), False, 10.0)
        return s, f.astype(bool)

    def infer(self, rows) -> Tuple[np.ndarray, np.ndarray, np.ndarray]:
        """(scores, flags, reconstructions [k, D])."""
        s, f, r = self._s.infer(np.ascontiguousarray(np.asarray(rows, np.float32).reshape(-1, self.D)), True, 10.0)
        return s, f.astype(bool), r

    def latency_us(self, rows, qps: float = 10000.0, device_breakdown: bool = False):
        """Per-event latency (us) of rows submitted one at a time at ``qps`` (C++ timing loop);
        with ``device_breakdown`` also the on-device processing time of each event (us)."""
        gap = int(1e9 / qps) if qps > 0 else 0
        out = self._s.latency_run(np.ascontiguousarray(np.asarray(rows, np.float32)), gap) / 1e3
        if device_breakdown:   # (host round trip, device total, device row-load, device compute)
            return out[:, 0], out[:, 1], out[:, 2], out[:, 3]
        return out[:, 0]

    @property
    def launches(self) -> int:
        return int(self._s.launches)

    def close(self) -> None:
        if self._s is not None:
            self._s.stop()
            self._s = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def lstm_layer_table(model) -> Tuple[np.ndarray, list]:
    """(flat weights in Keras order, LstmServeLayer tuples) of an LSTMPredictor."""
    from .lstm import ACT
    arrays = [np.asarray(a, np.float32) for a in model.fp.get()]
    offs = np.cumsum([0] + [a.size for a in arrays])
    flat = np.concatenate([a.ravel() for a in arrays]) if arrays else np.zeros(0, np.float32)
    table = []
    for L in model.layers:
        if L["kind"] == "lstm":
            p = L["params"]
            table.append((0, L["in_dim"], L["units"], ACT[L["activation"]], int(L["return_sequences"]), 0,
                          int(offs[p]), int(offs[p + 1]), int(offs[p + 2])))
        elif L["kind"] == "repeat":
            table.append((1, 0, 0, 0, 0, int(L["n"]), 0, 0, 0))
        else:
            p = L["params"]
            table.append((2, L["in_dim"], L["units"], 0, 0, 0, int(offs[p]), 0, int(offs[p + 1])))
    return flat, table


class LSTMScoringServer:
    """Persistent per-event LSTM forecaster; ``nkeys`` car keys (ids in [0, nkeys))."""

    def __init__(self, model, nkeys: int = 100_000, threshold: float = 5.0, slots: int = 4096,
                 idle_seconds: float = 2.0, normalizer: Optional[str] = "cardata", device: Optional[torch.device] = None):
        dev = torch.device(device) if device is not None else model.device
        if dev.type != "cuda":
            raise RuntimeError("LSTMScoringServer needs a ROCm device (use LSTMPredictor.predict on CPU)")
        flat, table = lstm_layer_table(model)
        sc = sh = None
        if normalizer == "cardata":
            from ..data.cardata import normalize_affine
            sc, sh = (np.asarray(a, np.float32) for a in normalize_affine())
        elif normalizer not in (None, "none"):
            raise ValueError(f"unknown normalizer {normalizer!r}")
        self.D, self.T, self.nkeys = int(model.features), int(model.look_back), int(nkeys)
        self.threshold = float(threshold)
        self._s = load_c().LSTMServe(dev.index if dev.index is not None else torch.cuda.current_device(), int(slots),
                                     flat, [list(t) for t in table], self.D, self.T, self.nkeys, sc, sh,
                                     float(threshold), float(idle_seconds))

    def forecast(self, rows, keys) -> Tuple[np.ndarray, np.ndarray, np.ndarray]:
        """Events in order -> (forecast of each key's next event [k, D] (zeros until the key has
        ``look_back`` events), score vs the key's previous forecast [k] (NaN if none),
        flags [k]: 0 normal, 1 score > threshold, 2 no previous forecast)."""
        rows = np.ascontiguousarray(np.asarray(rows, np.float32).reshape(-1, self.D))
        keys = np.ascontiguousarray(np.asarray(keys, np.int64).reshape(-1))
        s, f, r = self._s.infer(rows, True, 10.0, keys)
        return r, s, f

    def latency_us(self, rows, keys, qps: float = 10000.0, device_breakdown: bool = False):
        gap = int(1e9 / qps) if qps > 0 else 0
        out = self._s.latency_run(np.ascontiguousarray(np.asarray(rows, np.float32)), gap,
                                  np.ascontiguousarray(np.asarray(keys, np.int64))) / 1e3
        # device phases of the last run: pick-up -> key state and window gathered ("load"),
        # then the stack over the window ("compute")
        self.last_device_load_us = out[:, 2]
        if device_breakdown:
            return out[:, 0], out[:, 1], out[:, 3]
        return out[:, 0]

    def reset(self) -> None:
        """Forget every key's window and forecast."""
        self._s.reset_keys()

    @property
    def launches(self) -> int:
        return int(self._s.launches)

    def close(self) -> None:
        if self._s is not None:
            self._s.stop()
            self._s = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
