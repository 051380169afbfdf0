"""K8 ``normalize_filter`` on the device (``csrc/kernels/preprocess.hip``).

The reference's per-event tf.data graph -- ``normalize_fn`` (cardata-v3.py:78-168)
followed by ``filter(y == "false")`` (cardata-v3.py:212) -- as one order-preserving
stream compaction over raw rows that already sit on the GPU (pinned-ring H2D).
"""
from __future__ import annotations

from typing import Optional, Tuple

import numpy as np
import torch

from ._ext import load_c

KEEP_ALL = -1


def normalize_filter(x: torch.Tensor, labels: Optional[torch.Tensor] = None, keep: int = 0,
                     scale: Optional[np.ndarray] = None, shift: Optional[np.ndarray] = None,
                     want_index: bool = False, D: Optional[int] = None
                     ) -> Tuple[torch.Tensor, Optional[torch.Tensor]]:
    """Rows ``r`` with ``labels[r] == keep`` (all rows when ``keep < 0``), normalised as
    ``x * scale + shift``, in their original order; also their source indices.

    Reads the kept-row count back (one 8-byte device->host copy)."""
    dev = x.device
    D = int(D or x.size(1))
    if x.size(0) == 0:
        return (torch.empty((0, D), dtype=torch.float32, device=dev),
                torch.empty(0, dtype=torch.int64, device=dev) if want_index else None)
    sc = None if scale is None else torch.as_tensor(np.asarray(scale, np.float32), device=dev)
    sh = None if shift is None else torch.as_tensor(np.asarray(shift, np.float32), device=dev)
    if labels is not None:
        labels = labels.to(device=dev, dtype=torch.uint8).contiguous()
    out, idx, total = load_c().normalize_filter(x, D, labels, int(keep if labels is not None else KEEP_ALL),
                                                sc, sh, bool(want_index))
    m = int(total.item())
    return out[:m], (idx[:m] if want_index else None)


def normalize_filter_reference(x: np.ndarray, labels: Optional[np.ndarray], keep: int,
                               scale: Optional[np.ndarray], shift: Optional[np.ndarray]):
    """numpy oracle of :func:`normalize_filter`."""
    x = np.asarray(x, np.float32)
    mask = np.ones(len(x), bool) if labels is None or keep < 0 else (np.asarray(labels) == keep)
    y = x[mask]
    if scale is not None:
        y = y * np.asarray(scale, np.float32) + np.asarray(shift, np.float32)
    return y.astype(np.float32), np.nonzero(mask)[0]
