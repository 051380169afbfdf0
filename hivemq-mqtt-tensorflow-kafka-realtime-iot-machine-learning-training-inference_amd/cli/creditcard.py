"""Credit-card fraud autoencoder front end (autoencoder-anomaly-detection/).

``creditcard [servers]``: the Kafka consumer + training script
(Sensor-Kafka-Consumer-and-TensorFlow-Model-Training.py:33-50): read
``creditcard:0`` (group ``creditcard``, eof), batch 32, decode the CSV records,
train the D = 30 autoencoder for 5 epochs.  The reference passes ``(x, Class)``
to ``fit`` of an x -> x model (a shape bug); here the autoencoder target is x.

``--evaluate`` adds the notebook's offline evaluation (Python-Tensorflow-2.0-Keras-
Fraud-Detection-Autoencoder.ipynb): StandardScaler on Time / Amount, 80/20 split
with ``random_state=314``, train on ``Class == 0``, score the test split with the
fused HIP scoring kernel and report ROC AUC, precision / recall and the
confusion matrix at ``threshold_fixed = 5``.

Without a server (or with ``synthetic://[rows]``) synthetic data of the Kaggle
shape is produced into an in-process broker first.
"""
from __future__ import annotations

import json
import time
from typing import Sequence

import numpy as np

from . import common

USAGE = "Usage: python3 creditcard.py [servers] [--evaluate]"


def _flags(p):
    p.add_argument("--epochs", type=int, default=5)
    p.add_argument("--batch-size", type=int, default=32)
    p.add_argument("--rows", type=int, default=50000)
    p.add_argument("--csv", default=None, help="creditcard.csv to produce instead of synthetic data")
    p.add_argument("--evaluate", action="store_true")
    p.add_argument("--threshold", type=float, default=5.0)
    p.add_argument("--save", default=None, help="write the trained model (.h5)")
    p.add_argument("--precision", default=None, choices=["fp32", "bf16"],
                   help="small-batch trainer contractions: fp32 (Keras-exact, default) or bf16 MFMAs")


def main(argv: Sequence[str]) -> int:
    common.print_options(argv)
    ns = common.parse(argv, USAGE, ["servers"], n_optional=1, add_flags=_flags)
    from ..data import creditcard as cc
    from ..models.autoencoder import Autoencoder
    from ..utils import evaluation as ev

    servers = ns.servers or "synthetic://"
    cfg = common.kafka_config(servers, ns.kafka_config)
    if servers.startswith(("synthetic://", "fake://")):
        rest = servers.split("://", 1)[1]
        n = int(rest) if servers.startswith("synthetic://") and rest else ns.rows
        if ns.csv:
            x, y = cc.load_csv(ns.csv)
        else:
            x, y = cc.synthetic_creditcard(n, seed=ns.synthetic_seed)
        servers = "fake://creditcard"
        print(cc.produce_creditcard(servers, x, y), "records has been produced in 'creditcard'", flush=True)
    chunks = list(cc.kafka_creditcard(servers, config=cfg))
    x = np.concatenate([c[0] for c in chunks]) if chunks else np.zeros((0, cc.NUM_FEATURES))
    y = np.concatenate([c[1] for c in chunks]) if chunks else np.zeros(0, np.int64)
    print(f"consumed {len(x)} records ({int(y.sum())} fraud)", flush=True)

    ae = Autoencoder(input_dim=30, encoding_dim=14, hidden_dim=7, device=ns.device, seed=ns.seed)
    ae.compile(metrics=["accuracy"], loss="mean_squared_error", optimizer="adam", minibatch_precision=ns.precision)
    if not ns.evaluate:
        t0 = time.perf_counter()
        ae.fit(x.astype(np.float32), epochs=ns.epochs, batch_size=ns.batch_size, shuffle=False, verbose=2)
        print(f"Training complete ({time.perf_counter() - t0:.2f}s)", flush=True)
    else:
        xs, _ = cc.standardize_time_amount(x)
        x_train, x_test, y_train, y_test = ev.train_test_split(xs, y, test_size=0.2, random_state=314)
        x_train = x_train[y_train == 0].astype(np.float32)
        ae.fit(x_train, epochs=ns.epochs, batch_size=ns.batch_size, shuffle=True,
               validation_data=(x_test.astype(np.float32),), verbose=2)
        scores = ae.score(x_test.astype(np.float32))
        rep = ev.classification_summary(y_test, scores, threshold=ns.threshold)
        print(json.dumps(rep), flush=True)
    if ns.save:
        ae.save(ns.save)
    return 0


if __name__ == "__main__":
    import sys
    sys.exit(common.run(main))
