"""Autoencoder front ends: ``cardata-v3`` (train | predict + model store) and ``cardata-v1`` (train then predict).

``cardata-v3 <servers> <topic> <offset> <result_topic> <mode> <model-file> <project>``
(AUTOENCODER-TensorFlow-IO-Kafka/cardata-v3.py):

* train   -- KafkaDataset ``<topic>:0:<offset>`` (group ``cardata-autoencoder``, eof) ->
  normalize_fn -> keep ``failure_occurred == "false"`` -> batch(100).take(100) ->
  ``fit(epochs=20, verbose=2)`` -> save ``<model-file>`` -> upload to bucket
  ``tf-models_<project>`` (:203-232);
* predict -- download + load the model, ``batch(100).skip(100).take(100)`` over
  every event -> ``predict`` with the Kafka output callback writing
  ``np.array2string(reconstruction)`` to ``<result_topic>`` (:235-280).

``cardata-v1 <servers> <topic> <offset> [result_topic]``
(AUTOENCODER-TensorFlow-IO-Kafka/cardata-v1.py): 5 epochs x batch 32 x take(100),
save / reload ``path_to_my_model.h5``, predict ``batch(32).skip(100).take(100)``.

Normalisation is not a host stage: the model is built with
``input_normalizer="cardata"`` so the reference ``normalize_fn`` runs as the
fused affine map inside the HIP kernels' first load.
"""
from __future__ import annotations

import time
from typing import Sequence

from . import common

V3_USAGE = "Usage: python3 cardata-v1.py <servers> <topic> <offset> <result_topic> <mode> <model-file> <project>"
V1_USAGE = "Usage: python3 cardata-v1.py <servers> <topic> <offset> [result_topic]"


def _flags(p):
    p.add_argument("--epochs", type=int, default=None)
    p.add_argument("--batch-size", type=int, default=None)
    p.add_argument("--take", type=int, default=100, help="batches per epoch (.take(100))")
    p.add_argument("--skip", type=int, default=100, help="predict skips this many batches (.skip(100))")
    p.add_argument("--predict-take", type=int, default=100)
    p.add_argument("--schema", default="cardata-v1")
    p.add_argument("--with-score", action="store_true", help="also emit the per-event anomaly score")
    p.add_argument("--group", default="cardata-autoencoder")
    p.add_argument("--partitions", default=None,
                   help="partitions to read: '0' (the reference, cardata-v3.py:46), 'all', or a comma list; "
                        "default 0, or all under torchrun (WORLD_SIZE > 1)")
    p.add_argument("--assign", default="auto", choices=["auto", "split", "partitions"],
                   help="under torchrun: each rank's share of the partitions (streamml.kafka.assign)")
    p.add_argument("--native-feed", action="store_true", help="ROCm: the C++ partition-parallel feed")
    p.add_argument("--feed-workers", type=int, default=4)
    p.add_argument("--precision", default=None, choices=["fp32", "bf16"],
                   help="small-batch trainer contractions (Keras batch <= 128): fp32 (Keras-exact, default) or "
                        "bf16 MFMAs with fp32 master weights / Adam (compile(minibatch_precision=...))")


def _world() -> int:
    import os
    return int(os.environ.get("WORLD_SIZE", "1"))


def _stream(ns, servers, cfg, shard=None):
    from ..data import stream as st
    parts = ns.partitions or ("all" if _world() > 1 else "0")
    specs = ([f"{ns.topic}:*:{int(ns.offset)}"] if parts == "all" else
             [f"{ns.topic}:{int(p)}:{int(ns.offset)}" for p in parts.split(",") if p != ""])
    native = bool(ns.native_feed) and shard is not None
    return st.kafka(servers, specs, schema=ns.schema, group=ns.group, eof=True, config=cfg, shard=shard,
                    assign=ns.assign, native=native, workers=ns.feed_workers)


def _train(ns, servers, cfg, epochs, batch_size, out_path):
    """Under torchrun every rank trains on its own share of the partitions (one process per
    GPU, gradients all-reduced per step); rank 0 writes the model."""
    from ..models.autoencoder import Autoencoder
    from ..parallel.dp import init_from_env, sync_model_from_rank0
    env = init_from_env(None if ns.device == "auto" else ("cuda" if ns.device.startswith("cuda") else "cpu"))
    device = ns.device if env.world_size == 1 else env.device
    ae = Autoencoder(input_dim=18, encoding_dim=14, hidden_dim=7, input_normalizer="cardata", device=device,
                     seed=ns.seed)
    ae.compile(metrics=["accuracy"], loss="mean_squared_error", optimizer="adam", minibatch_precision=ns.precision)
    sync_model_from_rank0(ae)
    if env.rank == 0:
        ae.summary()
    # filter(y == "false") (cardata-v3.py:212): on a GPU the K8 kernel compacts on the device
    training = _stream(ns, servers, cfg, shard="auto" if env.world_size > 1 else None).filter_normal(device=True)
    t0 = time.perf_counter()
    ae.fit(training, epochs=epochs, batch_size=batch_size, steps_per_epoch=ns.take, verbose=2 if env.rank == 0 else 0)
    if env.rank == 0:
        print(f"Training complete ({time.perf_counter() - t0:.2f}s)", flush=True)
        ae.save(out_path)
    ae.dist_rank = env.rank
    return ae


def _predict(ns, servers, cfg, model, batch_size, result_topic):
    from ..nn.callbacks import KafkaPredictionSink
    data = _stream(ns, servers, cfg).batch(batch_size).skip(ns.skip).take(ns.predict_take)
    cbs = []
    if result_topic:
        sink = KafkaPredictionSink(batch_size, result_topic, servers, cfg, with_score=ns.with_score)
        cbs.append(sink)
    out = model.predict(data, batch_size=batch_size, callbacks=cbs)
    print(f"predict {out.shape[0]} events -> {result_topic}", flush=True)
    print("Predict complete", flush=True)
    return out


def main_v3(argv: Sequence[str]) -> int:
    common.print_options(argv)
    ns = common.parse(argv, V3_USAGE, ["servers", "topic", "offset", "result_topic", "mode", "model_file",
                                       "project"], add_flags=_flags)
    mode = ns.mode.strip().lower()
    if mode not in ("train", "predict"):
        print("Mode is invalid, must be either 'train' or 'predict':", mode)
        return 1
    from ..models.autoencoder import load_model
    from ..utils.model_store import autoencoder_store

    servers = common.prepare_servers(ns.servers, ns.topic, seed=ns.synthetic_seed, schema=ns.schema)
    cfg = common.kafka_config(ns.servers, ns.kafka_config)
    store = autoencoder_store(ns.project, ns.store)
    path = common.model_path(ns.workdir, ns.model_file)
    batch_size = ns.batch_size or 100
    if mode == "train":
        ae = _train(ns, servers, cfg, ns.epochs or 20, batch_size, path)
        if ae.dist_rank == 0:
            url = store.upload(path, "/" + ns.model_file)
            print("Model stored successfully", ns.model_file, url, flush=True)
        from ..parallel.dp import shutdown
        shutdown()
    else:
        print("Downloading model", ns.model_file, flush=True)
        store.download("/" + ns.model_file, path)
        print("Loading model", flush=True)
        model = load_model(path, device=ns.device, input_normalizer="cardata")
        _predict(ns, servers, cfg, model, batch_size, ns.result_topic)
    return 0


def main_v1(argv: Sequence[str]) -> int:
    common.print_options(argv)
    ns = common.parse(argv, V1_USAGE, ["servers", "topic", "offset", "result_topic"], n_optional=1,
                      add_flags=_flags)
    from ..models.autoencoder import load_model

    servers = common.prepare_servers(ns.servers, ns.topic, seed=ns.synthetic_seed, schema=ns.schema)
    cfg = common.kafka_config(ns.servers, ns.kafka_config)
    path = common.model_path(ns.workdir, "path_to_my_model.h5")
    batch_size = ns.batch_size or 32
    ae = _train(ns, servers, cfg, ns.epochs or 5, batch_size, path)
    from ..parallel.dp import shutdown
    shutdown()
    if ae.dist_rank == 0:   # predict runs once, on rank 0
        model = load_model(path, device=ns.device, input_normalizer="cardata")   # "recreate purely from the file"
        _predict(ns, servers, cfg, model, batch_size, ns.result_topic)
    return 0


if __name__ == "__main__":
    import sys
    sys.exit(common.run(main_v3))
