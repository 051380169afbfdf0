"""Persistent Keras-step trainer for the reference LSTM stack (``lstm_ref_train.hip``).

LSTM-TensorFlow-IO-Kafka/cardata-v2.py:172-209 fits the 4-LSTM + RepeatVector +
TimeDistributed(Dense) stack at ``look_back = 1`` with ``batch_size = 1``: one Adam
update per event.  ``train_steps`` runs ``nsteps`` of those Keras steps in ONE launch
(one workgroup, parameters in LDS, Adam moments in registers) and returns the per-step
``[loss, correct]`` on the device; parameters, moments and the Adam iteration counter
of the model's :class:`~streamml.ops.adam.FlatParams` are updated in place.

At look_back = 1 every LSTM starts from h0 = c0 = 0, so the recurrent kernels and the
forget-gate columns get exactly zero gradient and Keras leaves them unchanged; the
kernel skips them (``check_inactive`` verifies their moments are zero).
"""
from __future__ import annotations

from typing import Optional

import torch

from ._ext import load_c

ACT = {"relu": 1, "tanh": 2}
MAX_BATCH = 32
UNITS = (32, 16, 16, 32)


def supported(model) -> bool:
    """The model is the reference stack (18 features, LSTM 32/16/16/32, one activation,
    RepeatVector, TimeDistributed Dense 18) at look_back 1, on a ROCm device."""
    if model.device.type != "cuda" or model.look_back != 1 or model.features != 18:
        return False
    kinds = [L["kind"] for L in model.layers]
    if kinds != ["lstm", "lstm", "repeat", "lstm", "lstm", "dense"]:
        return False
    lstms = [L for L in model.layers if L["kind"] == "lstm"]
    if tuple(L["units"] for L in lstms) != UNITS or len({L["activation"] for L in lstms}) != 1:
        return False
    if lstms[0]["activation"] not in ACT:
        return False
    head = model.layers[-1]
    return head["units"] == 18 and head["td"] and model.layers[2]["n"] == 1


def _inactive_mask(model) -> torch.Tensor:
    """Flat mask of the parameters the look_back-1 kernel never touches (U, forget columns)."""
    fp = model.fp
    mask = torch.zeros(fp.n_pad, dtype=torch.bool)
    for L in model.layers:
        if L["kind"] != "lstm":
            continue
        u, i0 = L["units"], L["params"]
        w0, w1 = fp.offsets[i0], fp.offsets[i0 + 1]
        mask[w0:w1].view(-1, 4 * u)[:, u:2 * u] = True           # W forget columns
        mask[fp.offsets[i0 + 1]:fp.offsets[i0 + 2]] = True       # U
        b0 = fp.offsets[i0 + 2]
        mask[b0 + u:b0 + 2 * u] = True                          # forget bias
    return mask.to(fp.device)


def check_inactive(model) -> bool:
    """True when every skipped parameter has zero Adam moments (always the case for a
    look_back-1 model; false only for optimizer state imported from elsewhere)."""
    fp = model.fp
    mask = _inactive_mask(model)
    return bool((fp.m[mask].abs().sum() + fp.v[mask].abs().sum()).item() == 0.0)


def train_steps(model, x: torch.Tensor, y: torch.Tensor, batch: int, nsteps: int, row0: int = 0,
                order: Optional[torch.Tensor] = None) -> torch.Tensor:
    """``nsteps`` Keras steps of ``batch`` rows each from sample ``row0`` on (the last one
    partial if the samples run out).  ``x`` / ``y``: [n, 18] row views (any row stride)
    or [n, 1, 18] windows.  Returns the device tensor [nsteps, 2] = (mean loss, correct)."""
    if x.dim() == 3:
        x = x[:, 0]
    if y.dim() == 3:
        y = y[:, 0]
    act = ACT[model.layers[0]["activation"]]
    fp, hp = model.fp, model.hp
    return load_c().lstm_ref_train(fp.flat, fp.m, fp.v, fp.iter, x.float(), y.float(), order, int(row0), int(batch),
                                   int(nsteps), act, hp["lr"], hp["beta_1"], hp["beta_2"], hp["epsilon"])
