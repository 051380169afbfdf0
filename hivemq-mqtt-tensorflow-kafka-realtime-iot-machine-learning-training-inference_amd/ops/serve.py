"""Persistent per-event anomaly scoring on the GPU (``csrc/kernels/ae_serve.hip``).

``ScoringServer(model)`` keeps one wave resident on the device that polls a
host-mapped request ring; ``score(rows)`` publishes rows and spins on the
completion counter -- no kernel launch, no hipMemcpy per event.  This is the
low-latency path of BASELINE config 5 (the launch-per-event path is
``Autoencoder.score``).  The kernel exits by itself after ``idle_seconds``
without requests and is relaunched transparently on the next request.
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
