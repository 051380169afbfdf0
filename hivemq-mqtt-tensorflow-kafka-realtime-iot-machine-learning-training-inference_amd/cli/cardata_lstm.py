"""LSTM front ends: ``lstm-v2`` (train | predict + model store) and ``lstm-v1`` (train then predict).

``lstm-v2 <servers> <topic> <offset> <result_topic> <mode> <model-file>``
(LSTM-TensorFlow-IO-Kafka/cardata-v2.py:152-273): KafkaDataset ``<topic>:0:<offset>``
(group ``cardata-v1``) -> normalize_fn -> ``window(look_back=1, shift=1)`` as x and
``skip(look_back)`` as the next-event target y -> ``zip.batch(1).take(1000)`` ->
``fit(epochs=5)`` -> save + upload to bucket ``car-demo-tensorflow-models``; predict
downloads the model and streams ``dataset_x.batch(1).skip(1000).take(200)``
predictions to ``<result_topic>``.

``lstm-v1 <servers> <topic> <offset> [result_topic]`` (LSTM-.../cardata-v1.py:146-230):
train then predict in one run, no model store.

Model: the reference 5-block stack (18 642 parameters) on the fused HIP LSTM
kernels; ``--stack two-layer --look-back 50`` selects the BASELINE config-3 variant.
"""
from __future__ import annotations

import time
from typing import Sequence

import numpy as np

from . import common

V2_USAGE = "Usage: python3 cardata-v1.py <servers> <topic> <offset> <result_topic> <mode> <model-file>"
V1_USAGE = "Usage: python3 cardata-v1.py <servers> <topic> <offset> [result_topic]"


def _flags(p):
    p.add_argument("--epochs", type=int, default=5)
    p.add_argument("--batch-size", type=int, default=1)
    p.add_argument("--look-back", type=int, default=1)
    p.add_argument("--take", type=int, default=1000, help="training batches per epoch (.take(1000))")
    p.add_argument("--skip", type=int, default=1000, help="predict skips this many windows")
    p.add_argument("--predict-take", type=int, default=200)
    p.add_argument("--stack", choices=["reference", "two-layer"], default="reference")
    p.add_argument("--schema", default="cardata-v1")
    p.add_argument("--group", default="cardata-v1")
    p.add_argument("--predict-engine", choices=["auto", "persistent", "batch"], default="auto",
                   help="persistent: events one at a time through the resident GPU forecaster "
                        "(lstm_serve.hip); batch: model.predict over the windows; auto: persistent on ROCm")


def _rows(ns, servers, cfg) -> np.ndarray:
    """Bounded (eof) read of the partition, normalised with normalize_fn -> [n, 18]."""
    from ..data import stream as st
    s = st.kafka(servers, [f"{ns.topic}:0:{int(ns.offset)}"], schema=ns.schema, group=ns.group, eof=True,
                 config=cfg).normalize()
    return s.collect().x.astype(np.float32)


def _windows(rows: np.ndarray, look_back: int) -> np.ndarray:
    n = len(rows) - look_back + 1
    if n <= 0:
        return np.zeros((0, look_back, rows.shape[1]), np.float32)
    idx = np.arange(n)[:, None] + np.arange(look_back)[None, :]
    return rows[idx]


def _build(ns):
    from ..models.lstm import LSTMPredictor
    if ns.stack == "two-layer":
        return LSTMPredictor.two_layer(look_back=ns.look_back, device=ns.device, seed=ns.seed)
    return LSTMPredictor.reference(look_back=ns.look_back, device=ns.device, seed=ns.seed)


def _train(ns, rows, model):
    T = ns.look_back
    if model.device.type == "cuda":
        # windows as strided views over the device-resident rows, read in place by the
        # fused LSTM kernels (no [n, T, F] materialisation)
        import torch
        from ..data.stream import sliding_windows
        x, y = sliding_windows(torch.as_tensor(np.ascontiguousarray(rows, np.float32), device=model.device), T)
    else:
        x = _windows(rows, T)[:len(rows) - T]      # zip(dataset_x, dataset.skip(T)) drops the last window
        y = rows[T:]
    print("DATASET: ", f"windows={len(x)} look_back={T} batch={ns.batch_size} take={ns.take}", flush=True)
    t0 = time.perf_counter()
    model.fit(x, y, epochs=ns.epochs, batch_size=ns.batch_size, take=ns.take, verbose=2)
    print(f"Training complete ({time.perf_counter() - t0:.2f}s)", flush=True)


def _predict_persistent(model, rows: np.ndarray, first: int, count: int) -> np.ndarray:
    """Forecasts of windows [first, first + count) by streaming the events one at a time
    through the resident forecaster: the window ending at event i is window i - T + 1, so
    events 0 .. first + count + T - 2 are fed (one key: the reference windows the partition's
    event sequence, not per car) and the forecasts at the matching events returned."""
    from ..ops.serve import LSTMScoringServer
    T = model.look_back
    end = min(len(rows), first + count + T - 1)
    if end < first + T:
        return np.zeros((0, model.features), np.float32)
    with LSTMScoringServer(model, nkeys=1, normalizer=None) as srv:   # rows are normalised already
        pred, _, _ = srv.forecast(rows[:end], np.zeros(end, np.int64))
    return pred[first + T - 1:end]


def _predict(ns, servers, cfg, rows, model, result_topic):
    from ..nn.callbacks import KafkaPredictionSink
    xw = _windows(rows, ns.look_back)
    b0 = ns.skip * ns.batch_size
    xw = xw[b0:b0 + ns.predict_take * ns.batch_size]
    cbs = [KafkaPredictionSink(ns.batch_size, result_topic, servers, cfg)] if result_topic else []
    engine = ns.predict_engine
    # the forecaster emits each window's LAST step only: it serves stacks whose output is one
    # step per window (the reference at look_back 1); a sequence-output stack (RepeatVector(R)
    # with R > 1) keeps the batch engine under "auto", so both engines return the same shape
    shape = np.shape(model.predict(np.zeros((1, ns.look_back, model.features), np.float32)))[1:]
    one_step = int(np.prod(shape)) == model.features
    if engine == "auto":
        engine = "persistent" if model.device.type == "cuda" and one_step else "batch"
    if engine == "persistent":
        out = _predict_persistent(model, rows, b0, len(xw))
        if one_step:
            out = out.reshape((len(out),) + tuple(shape))
        for cb in cbs:   # the reference OutputCallback, per batch_size forecasts
            cb.set_model(model)
            for bi, s0 in enumerate(range(0, len(out), ns.batch_size)):
                cb.on_predict_batch_end(bi, {"outputs": out[s0:s0 + ns.batch_size]})
            cb.on_predict_end()
        print(f"predict {len(out)} windows (persistent forecaster) -> {result_topic}", flush=True)
        print("Predict complete", flush=True)
        return out
    out = model.predict(xw, batch_size=ns.batch_size, callbacks=cbs)
    print(f"predict {len(xw)} windows -> {result_topic}", flush=True)
    print("Predict complete", flush=True)
    return out


def main_v2(argv: Sequence[str]) -> int:
    common.print_options(argv)
    ns = common.parse(argv, V2_USAGE, ["servers", "topic", "offset", "result_topic", "mode", "model_file"],
                      add_flags=_flags)
    mode = ns.mode.strip().lower()
    if mode not in ("train", "predict"):
        print("Mode is invalid, must be either 'train' or 'predict':", mode)
        return 1
    from ..models.lstm import LSTMPredictor
    from ..utils.model_store import lstm_store

    servers = common.prepare_servers(ns.servers, ns.topic, seed=ns.synthetic_seed, schema=ns.schema)
    cfg = common.kafka_config(ns.servers, ns.kafka_config)
    store = lstm_store(ns.store)
    path = common.model_path(ns.workdir, ns.model_file)
    rows = _rows(ns, servers, cfg)
    if mode == "train":
        print("Running training", flush=True)
        model = _build(ns)
        _train(ns, rows, model)
        model.save(path)
        store.upload(path, ns.model_file)
        print("Model stored successfully ", ns.model_file, flush=True)
    else:
        print("Downloading model", ns.model_file, flush=True)
        store.download(ns.model_file, path)
        print("Loading model", flush=True)
        model = LSTMPredictor.load(path, device=ns.device)
        ns.look_back = model.look_back
        _predict(ns, servers, cfg, rows, model, ns.result_topic)
    return 0


def main_v1(argv: Sequence[str]) -> int:
    common.print_options(argv)
    ns = common.parse(argv, V1_USAGE, ["servers", "topic", "offset", "result_topic"], n_optional=1,
                      add_flags=_flags)
    servers = common.prepare_servers(ns.servers, ns.topic, seed=ns.synthetic_seed, schema=ns.schema)
    cfg = common.kafka_config(ns.servers, ns.kafka_config)
    rows = _rows(ns, servers, cfg)
    model = _build(ns)
    _train(ns, rows, model)
    _predict(ns, servers, cfg, rows, model, ns.result_topic)
    return 0


if __name__ == "__main__":
    import sys
    sys.exit(common.run(main_v2))
