"""Offline anomaly-score evaluation.

The fraud-detection notebooks score the test split with the per-row
reconstruction MSE and then evaluate it with scikit-learn
(Python-Tensorflow-2.0-Keras-Fraud-Detection-Autoencoder.ipynb: ``StandardScaler`` on
Time/Amount, ``train_test_split(test_size=0.2, random_state=314)``, ``roc_curve`` + ``auc``,
``precision_recall_curve``, fixed ``threshold_fixed = 5`` -> ``confusion_matrix``).

These are numpy re-implementations with the same outputs as scikit-learn 1.7
(tests compare against sklearn directly), so the scoring pipeline has no
sklearn dependency.  Scores for millions of rows come from the fused HIP
forward kernel (:meth:`streamml.models.autoencoder.Autoencoder.score`); for
very large score vectors :func:`roc_auc_torch` sorts on the device instead.
"""
from __future__ import annotations

import math
from typing import Optional, Tuple

import numpy as np


def _binary_clf_curve(y_true, y_score) -> Tuple[np.ndarray, np.ndarray, np.ndarray]:
    """Cumulative (fps, tps, thresholds) at each distinct score, scores descending."""
    y_true = np.asarray(y_true).ravel()
    y_score = np.asarray(y_score, dtype=np.float64).ravel()
    if y_true.shape != y_score.shape:
        raise ValueError("y_true and y_score must have the same length")
    y_true = (y_true == 1) if y_true.dtype != bool else y_true
    order = np.argsort(y_score, kind="mergesort")[::-1]
    y_score = y_score[order]
    y_true = y_true[order].astype(np.float64)
    distinct = np.where(np.diff(y_score))[0]
    idx = np.r_[distinct, y_true.size - 1]
    tps = np.cumsum(y_true)[idx]
    fps = 1 + idx - tps
    return fps, tps, y_score[idx]


def roc_curve(y_true, y_score, drop_intermediate: bool = True):
    """(fpr, tpr, thresholds); thresholds[0] = +inf (sklearn >= 1.3 convention)."""
    fps, tps, thr = _binary_clf_curve(y_true, y_score)
    if drop_intermediate and len(fps) > 2:
        keep = np.where(np.r_[True, np.logical_or(np.diff(fps, 2), np.diff(tps, 2)), True])[0]
        fps, tps, thr = fps[keep], tps[keep], thr[keep]
    tps = np.r_[0, tps]
    fps = np.r_[0, fps]
    thr = np.r_[np.inf, thr]
    fpr = fps / fps[-1] if fps[-1] > 0 else np.full(fps.shape, np.nan)
    tpr = tps / tps[-1] if tps[-1] > 0 else np.full(tps.shape, np.nan)
    return fpr, tpr, thr


def auc(x, y) -> float:
    """Trapezoidal area under a monotone curve (either direction)."""
    x = np.asarray(x, dtype=np.float64)
    y = np.asarray(y, dtype=np.float64)
    if x.shape[0] < 2:
        raise ValueError("need at least 2 points to compute an area")
    dx = np.diff(x)
    direction = 1.0
    if np.any(dx < 0):
        if np.all(dx <= 0):
            direction = -1.0
        else:
            raise ValueError("x is neither increasing nor decreasing")
    return float(direction * np.trapezoid(y, x))


def roc_auc_score(y_true, y_score) -> float:
    fpr, tpr, _ = roc_curve(y_true, y_score, drop_intermediate=True)
    return auc(fpr, tpr)


def precision_recall_curve(y_true, probas_pred, drop_intermediate: bool = False):
    """(precision, recall, thresholds) with the final (1, 0) point appended."""
    fps, tps, thr = _binary_clf_curve(y_true, probas_pred)
    if drop_intermediate and len(fps) > 2:
        keep = np.where(np.r_[True, np.logical_or(np.diff(tps[:-1]), np.diff(tps[1:])), True])[0]
        fps, tps, thr = fps[keep], tps[keep], thr[keep]
    ps = tps + fps
    precision = np.zeros_like(tps)
    np.divide(tps, ps, out=precision, where=(ps != 0))
    recall = np.ones_like(tps) if tps[-1] == 0 else tps / tps[-1]
    return np.hstack((precision[::-1], 1)), np.hstack((recall[::-1], 0)), thr[::-1]


def confusion_matrix(y_true, y_pred, labels: Optional[np.ndarray] = None) -> np.ndarray:
    y_true = np.asarray(y_true).ravel()
    y_pred = np.asarray(y_pred).ravel()
    if labels is None:
        labels = np.unique(np.concatenate([y_true, y_pred]))
    labels = np.asarray(labels)
    index = {v.item() if hasattr(v, "item") else v: i for i, v in enumerate(labels)}
    n = len(labels)
    ti = np.array([index.get(v.item() if hasattr(v, "item") else v, -1) for v in y_true])
    pi = np.array([index.get(v.item() if hasattr(v, "item") else v, -1) for v in y_pred])
    ok = (ti >= 0) & (pi >= 0)
    cm = np.zeros((n, n), dtype=np.int64)
    np.add.at(cm, (ti[ok], pi[ok]), 1)
    return cm


def classification_summary(y_true, scores, threshold: float = 5.0) -> dict:
    """The notebook's final report: AUC, confusion at the fixed threshold, precision / recall."""
    y_true = np.asarray(y_true).astype(int)
    pred = (np.asarray(scores) > threshold).astype(int)
    cm = confusion_matrix(y_true, pred, labels=np.array([0, 1]))
    tn, fp, fn, tp = cm.ravel()
    out = {"threshold": float(threshold), "confusion": cm.tolist(),
           "precision": float(tp / (tp + fp)) if tp + fp else 0.0,
           "recall": float(tp / (tp + fn)) if tp + fn else 0.0}
    if 0 < y_true.sum() < len(y_true):
        out["roc_auc"] = roc_auc_score(y_true, scores)
    return out


class StandardScaler:
    """``StandardScaler().fit_transform`` (population std, zero-variance columns left unscaled)."""

    def fit(self, x):
        x = np.asarray(x, dtype=np.float64)
        x2 = x.reshape(len(x), -1)
        self.mean_ = x2.mean(axis=0)
        var = x2.var(axis=0)
        self.var_ = var
        scale = np.sqrt(var)
        scale[scale < 10 * np.finfo(np.float64).eps] = 1.0
        self.scale_ = scale
        return self

    def transform(self, x):
        x = np.asarray(x, dtype=np.float64)
        shp = x.shape
        return ((x.reshape(len(x), -1) - self.mean_) / self.scale_).reshape(shp)

    def fit_transform(self, x):
        return self.fit(x).transform(x)

    def inverse_transform(self, x):
        x = np.asarray(x, dtype=np.float64)
        shp = x.shape
        return (x.reshape(len(x), -1) * self.scale_ + self.mean_).reshape(shp)


def train_test_split(*arrays, test_size: float = 0.25, random_state: Optional[int] = None, shuffle: bool = True):
    """Same split as sklearn's ``train_test_split`` (ShuffleSplit over a legacy RandomState)."""
    if not arrays:
        raise ValueError("at least one array required")
    n = len(arrays[0])
    if any(len(a) != n for a in arrays):
        raise ValueError("arrays must have the same length")
    n_test = int(math.ceil(test_size * n)) if isinstance(test_size, float) else int(test_size)
    n_train = n - n_test
    if shuffle:
        perm = np.random.RandomState(random_state).permutation(n)
        test_idx, train_idx = perm[:n_test], perm[n_test:n_test + n_train]
    else:
        train_idx, test_idx = np.arange(n_train), np.arange(n_train, n)
    out = []
    for a in arrays:
        if hasattr(a, "iloc"):
            out += [a.iloc[train_idx], a.iloc[test_idx]]
        else:
            a = np.asarray(a)
            out += [a[train_idx], a[test_idx]]
    return out


def roc_auc_torch(y_true, y_score) -> float:
    """ROC AUC for very long score vectors: sort + cumsum on the scores' device (ties averaged)."""
    import torch
    s = torch.as_tensor(y_score).double().flatten()
    y = torch.as_tensor(y_true, device=s.device).flatten().double()
    s_sorted, order = torch.sort(s, descending=True, stable=True)
    y = y[order]
    last = torch.ones_like(s_sorted, dtype=torch.bool)
    last[:-1] = s_sorted[1:] != s_sorted[:-1]
    tps = torch.cumsum(y, 0)[last]
    fps = torch.cumsum(1 - y, 0)[last]
    P, N = tps[-1], fps[-1]
    if P == 0 or N == 0:
        return float("nan")
    tpr = torch.cat([tps.new_zeros(1), tps / P])
    fpr = torch.cat([fps.new_zeros(1), fps / N])
    return float(torch.trapezoid(tpr, fpr))
