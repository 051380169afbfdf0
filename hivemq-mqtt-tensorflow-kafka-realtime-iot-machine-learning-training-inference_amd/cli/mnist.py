"""MNIST front end (python-scripts/tensorflow-kafka-mnist*.py, confluent-tensorflow-io-kafka*.py).

``mnist [servers]``: produce the training set as raw bytes to ``xx`` / ``yy``
(reference producer), consume both topics, zip, ``batch(1)`` and fit
Flatten -> Dense(128, relu) -> Dense(10, softmax) with sparse CE + Adam for
``--epochs`` x ``--steps-per-epoch`` (reference: 5 x 12000, or 1 x 1000 with a
TensorBoard callback).  ``--simplified`` is confluent-tensorflow-io-kafka-simplified.py:
Dense(512) + Dropout(0.2), arrays, batch 32, validation on the test split.
Without real MNIST IDX files (``--mnist-dir``) a synthetic digit set is used.
"""
from __future__ import annotations

import time
from typing import Sequence

from . import common

USAGE = "Usage: python3 tensorflow-kafka-mnist.py [servers]"


def _flags(p):
    p.add_argument("--epochs", type=int, default=5)
    p.add_argument("--steps-per-epoch", type=int, default=12000)
    p.add_argument("--batch-size", type=int, default=1)
    p.add_argument("--rows", type=int, default=60000)
    p.add_argument("--mnist-dir", default=None)
    p.add_argument("--simplified", action="store_true")
    p.add_argument("--no-produce", action="store_true", help="topics xx / yy are already filled")
    p.add_argument("--log-dir", default=None, help="TensorBoard event directory")
    p.add_argument("--save", default=None)


def main(argv: Sequence[str]) -> int:
    common.print_options(argv)
    ns = common.parse(argv, USAGE, ["servers"], n_optional=1, add_flags=_flags)
    from ..data import mnist as mn
    from ..models.mlp import MLPClassifier
    from ..nn.callbacks import TensorBoard

    (xtr, ytr), (xte, yte) = mn.load_mnist(ns.mnist_dir, seed=ns.synthetic_seed, n_synthetic=ns.rows)
    print("train: ", (xtr.shape, ytr.shape), flush=True)
    cbs = [TensorBoard(ns.log_dir)] if ns.log_dir else []
    t0 = time.perf_counter()
    if ns.simplified:
        model = MLPClassifier(hidden=512, dropout=0.2, device=ns.device, seed=ns.seed)
        model.fit(xtr, ytr, epochs=ns.epochs, batch_size=32 if ns.batch_size == 1 else ns.batch_size,
                  validation_data=(xte, yte), callbacks=cbs, verbose=2)
    else:
        servers = ns.servers or "fake://mnist"
        cfg = common.kafka_config(servers, ns.kafka_config)
        if servers.startswith("synthetic://"):
            servers = "fake://mnist"
        if not ns.no_produce:
            print("count(x, y): ", mn.produce_mnist(servers, xtr, ytr, config=cfg), flush=True)
        model = MLPClassifier(hidden=128, device=ns.device, seed=ns.seed)
        model.fit(stream=lambda: mn.kafka_mnist(servers, config=cfg), epochs=ns.epochs, batch_size=ns.batch_size,
                  steps_per_epoch=ns.steps_per_epoch, callbacks=cbs, verbose=2)
    loss, acc = model.evaluate(xte, yte)
    print(f"test loss {loss:.4f} accuracy {acc:.4f} ({time.perf_counter() - t0:.1f}s)", flush=True)
    if ns.save:
        model.save(ns.save)
    return 0


if __name__ == "__main__":
    import sys
    sys.exit(common.run(main))
