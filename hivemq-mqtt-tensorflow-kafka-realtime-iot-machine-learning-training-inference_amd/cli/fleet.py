"""``fleet``: one anomaly autoencoder per car (or per key group), trained concurrently.

The reference trains a single model on the whole stream (cardata-v3.py:187-203,
``fit(batch_size=32)``).  ``fleet`` keys the same rows by car id (the CSV's ``car``
column / the record key that the KSQL REKEY step produces) and trains one model per
key with the same Keras-batch semantics, all models at once on one GPU
(``ops/ae_fleet.py``).  It then writes every model as a Keras HDF5 file plus an
``index.json`` {name -> file, keys, final loss}.

  fleet <csv|synthetic> [--models N] [--epochs E] [--batch 32] [--lr 1e-3] [--out DIR]
"""
from __future__ import annotations

import argparse
import json
import os
import re
from typing import Sequence


def parse_args(argv: Sequence[str]):
    p = argparse.ArgumentParser(prog="fleet", description=__doc__,
                                formatter_class=argparse.RawDescriptionHelpFormatter)
    p.add_argument("source", help="car-sensor CSV (time,car,...) or 'synthetic'")
    p.add_argument("--models", type=int, default=None, help="hash keys onto N models (default: one per key)")
    p.add_argument("--epochs", type=int, default=5)
    p.add_argument("--batch", type=int, default=32)
    p.add_argument("--lr", type=float, default=1e-3)
    p.add_argument("--out", default="fleet_models")
    p.add_argument("--device", default="cuda:0")
    p.add_argument("--seed", type=int, default=0)
    p.add_argument("--synthetic-rows", type=int, default=1 << 20)
    p.add_argument("--synthetic-devices", type=int, default=1000)
    return p.parse_args(list(argv))


def model_name(members, i: int, used=None) -> str:
    """File stem of model ``i``: its key when it owns exactly one, else ``modelNNNNN``.
    ``used`` (a set) de-duplicates stems that sanitise alike (``car/1`` vs ``car_1``, or a
    key literally named ``model00003``): a later collision gets ``-<i>`` appended."""
    stem = re.sub(r"[^A-Za-z0-9_.-]", "_", str(members[i][0])) if len(members[i]) == 1 else f"model{i:05d}"
    if used is not None:
        if stem in used:
            stem = f"{stem}-{i}"
        used.add(stem)
    return stem


def training_rows(ns):
    """(raw rows, car keys) of NORMAL events only: the reference trains its anomaly model on
    ``failure_occurred == "false"`` rows (cardata-v3.py:211-212); the CSV has no failure
    column, so every CSV row counts as normal."""
    import numpy as np

    from ..data.cardata import SyntheticCarSource, load_csv
    if ns.source == "synthetic":
        src = SyntheticCarSource(seed=ns.seed, n_devices=ns.synthetic_devices)
        raw, fail, dev_id, _ = src.generate(ns.synthetic_rows)
        raw, dev_id = raw[~fail], dev_id[~fail]
        return raw, np.array([f"electric-vehicle-{d:05d}" for d in dev_id])
    raw, _, keys = load_csv(ns.source)
    return raw, keys


def main(argv: Sequence[str]) -> int:
    ns = parse_args(argv)
    import numpy as np
    import torch

    from ..data.cardata import normalize_affine
    from ..models.autoencoder import Autoencoder
    from ..ops.ae import AESpec
    from ..ops.ae_fleet import AEFleet, ragged_rings_by_key

    raw, keys = training_rows(ns)
    flat, table, members = ragged_rings_by_key(raw, keys, batch=ns.batch, n_models=ns.models)
    M = len(members)
    spec = AESpec(input_dim=raw.shape[1])
    scale, shift = normalize_affine()
    dev = torch.device(ns.device)
    fleet = AEFleet.from_seeds(spec, [ns.seed + i for i in range(M)], dev, lr=ns.lr, scale=scale, shift=shift)
    fleet.attach_ragged(torch.from_numpy(flat).to(dev), ns.batch, table)
    steps = fleet.epoch_steps()
    print(f"fleet: {M} models, {len(flat)} rows, {int(steps.min())}-{int(steps.max())} steps of {ns.batch} rows "
          f"per model per epoch", flush=True)
    ms = []
    for ep in range(ns.epochs):
        fleet.reset_metrics()
        fleet.train_epoch()
        ms = fleet.read_metrics()
        losses = np.array([m["loss"] for m in ms])
        print(f"Epoch {ep + 1}/{ns.epochs} - loss mean {losses.mean():.4f} min {losses.min():.4f} "
              f"max {losses.max():.4f}", flush=True)
    os.makedirs(ns.out, exist_ok=True)
    index, used = {}, set()
    for i in range(M):
        name = model_name(members, i, used)
        path = os.path.join(ns.out, name + ".h5")
        am = Autoencoder(input_dim=spec.input_dim, device="cpu")
        am.compile(learning_rate=ns.lr)   # the saved training_config records the rate actually used
        am.set_weights(fleet.get_weights(i))
        am.save(path, include_optimizer=False)
        index[name] = {"file": os.path.basename(path), "keys": [str(k) for k in members[i]],
                       "loss": ms[i]["loss"] if ms else None}
    with open(os.path.join(ns.out, "index.json"), "w") as f:
        json.dump(index, f, indent=1)
    print(f"wrote {M} models to {ns.out}", flush=True)
    return 0
