"""Config-driven, restartable training job.

    python -m streamml.cli train --config job.yaml [--key=value ...]
    torchrun --nproc-per-node 8 --max-restarts 3 -m streamml.cli train --ckpt-dir /ckpt ...

Settings come from :class:`streamml.config.Config` (YAML/JSON file, then
``SML_*`` environment variables, then ``--key=value`` flags) plus the job keys
below.  The job checkpoints every ``ckpt_every`` epochs (rank 0 writes, sidecar
with the training position) and, when started with a checkpoint directory that
already holds one, resumes from it -- weights, Adam moments and iteration count
from the ``.h5``, the epoch from the sidecar, rank 0's state broadcast to every
replica.  Under ``torchrun --max-restarts`` a crashed or hung rank therefore
costs at most one epoch of work (see :mod:`streamml.parallel.fault`).

Data: ``servers=synthetic://N`` (default) trains on N synthetic car events
(deterministic, rank-sharded inside ``fit``); a Kafka bootstrap / ``fake://``
source streams the topic (``partition=-1``: every partition), each rank its own share
(``assign``: split | partitions, :mod:`streamml.kafka.assign`) through the native feed,
with no collect.  Prints one JSON summary line on rank 0.

Continuous training (``segment_rows=N``, autoencoder): the job follows the topic instead of
re-reading a bounded snapshot per epoch.  Each of ``epochs`` segments trains, on every rank, the
next <= N records of each partition it owns (``p % world == rank``), from the positions of the
last checkpoint (:class:`streamml.kafka.assign.SegmentPlan`); after the segment the positions
advance, and every ``ckpt_every`` segments the checkpoint's sidecar stores every partition's
position next to the model (committed to the consumer group too).  A restart -- e.g. by
``torchrun --max-restarts`` after a crashed rank -- resumes from those positions: every record is
trained exactly once, in the same step boundaries as an uninterrupted run
(tests/test_stream_resume.py).
"""
from __future__ import annotations

import json
import os
import sys
import time
from typing import Sequence


JOB_KEYS = {"ckpt_dir": None, "ckpt_every": 1, "rows": 200000, "stack": "two_layer", "metrics_port": 0,
            "segment_rows": 0, "precision": ""}


def _split(argv):
    job, rest = dict(JOB_KEYS), []
    cfg_path = None
    i = 0
    while i < len(argv):
        tok = argv[i]
        if tok == "--config":
            cfg_path = argv[i + 1]
            i += 2
            continue
        if tok.startswith("--config="):
            cfg_path = tok.split("=", 1)[1]
            i += 1
            continue
        key = tok[2:].split("=", 1)[0].replace("-", "_") if tok.startswith("--") else None
        if key in JOB_KEYS:
            if "=" in tok:
                val = tok.split("=", 1)[1]
                i += 1
            else:
                val = argv[i + 1]
                i += 2
            job[key] = type(JOB_KEYS[key])(val) if JOB_KEYS[key] is not None else val
            continue
        rest.append(tok)
        i += 1
    return cfg_path, job, rest


def main(argv: Sequence[str]) -> int:
    from ..config import Config
    cfg_path, job, rest = _split(list(argv))
    cfg = Config.load(cfg_path, env=True, argv=rest)
    import numpy as np
    import torch
    from ..ckpt import resume as rs
    from ..parallel.dp import init_from_env, shutdown, sync_model_from_rank0

    device_type = None if cfg.device == "auto" else ("cuda" if cfg.device.startswith("cuda") else "cpu")
    env = init_from_env(device_type)
    rank, world = env.rank, env.world_size
    if job["metrics_port"] and rank == 0:
        from ..obs.metrics import REGISTRY
        REGISTRY.serve(int(job["metrics_port"]), "0.0.0.0")
    dev = env.device
    ckpt_dir = job["ckpt_dir"]

    # ---------------------------------------------------------------- model
    model, state = (None, None)
    if ckpt_dir:
        if cfg.model == "autoencoder":
            from ..models.autoencoder import load_model as loader
            kw = {"device": dev, "input_normalizer": "cardata"}
        elif cfg.model == "lstm":
            from ..models.lstm import LSTMPredictor
            loader, kw = LSTMPredictor.load, {"device": dev}
        else:
            raise ValueError(f"train: unsupported model {cfg.model!r}")
        model, state = rs.load_latest(ckpt_dir, loader, **kw)
    start_epoch = int(state["epoch"]) if state else 0
    if model is None:
        if cfg.model == "autoencoder":
            from ..models.autoencoder import Autoencoder
            model = Autoencoder(cfg.input_dim, cfg.encoding_dim, cfg.hidden_dim, activity_l1=cfg.activity_l1,
                                device=dev, seed=cfg.seed, input_normalizer="cardata")
            model.compile(learning_rate=cfg.learning_rate, beta_1=cfg.beta_1, beta_2=cfg.beta_2,
                          epsilon=cfg.epsilon, minibatch_precision=job["precision"] or None)
        else:
            from ..models.lstm import LSTMPredictor
            ctor = LSTMPredictor.two_layer if job["stack"] == "two_layer" else LSTMPredictor.reference
            model = ctor(look_back=cfg.look_back, device=dev, seed=cfg.seed)
    sync_model_from_rank0(model)

    # ---------------------------------------------------------------- data
    servers = cfg.servers
    plan = None
    if servers.startswith("synthetic://"):
        from ..data.stream import synthetic
        n = int(servers[len("synthetic://"):] or job["rows"])
        chunk = synthetic(n, chunk=1 << 16, seed=cfg.seed).collect()
        x = chunk.x
        if cfg.model == "lstm":
            from ..data.cardata import normalize_np
            xn = normalize_np(x).astype(np.float32)
            T = cfg.look_back
            idx = np.arange(len(xn) - T)[:, None] + np.arange(T)[None, :]
            data = (xn[idx], xn[np.arange(len(xn) - T) + T])
        else:
            data = (x[chunk.label == 0],)
    else:
        # every rank streams its own share of the topic's partitions (kafka/assign.py: equal
        # contiguous offset ranges, resolved on one log snapshot per epoch) straight into fit --
        # no rank reads another's records and nothing is collected first
        from ..data import stream as st
        part = "*" if cfg.partition < 0 else str(cfg.partition)
        if int(job["segment_rows"]) > 0:
            if cfg.model != "autoencoder":
                raise ValueError("train: segment_rows (continuous training) supports the autoencoder")
            from ..kafka.assign import SegmentPlan
            from ..kafka.client import parse_topic_spec
            # positions of every partition from the checkpoint (any world size: the map is per
            # partition), else the configured offset / the log start
            plan = SegmentPlan([parse_topic_spec(f"{cfg.topic}:{part}:{cfg.offset}")], rank, world,
                               int(job["segment_rows"]), (state or {}).get("offsets"))
        # continuous mode reads with the ORDERED parallel reader (fetch + decode threads, batches in
        # cursor order): the row order -- and so a replay after a restart -- is deterministic; the
        # native feed hands slabs over in completion order
        s = st.kafka(servers, [f"{cfg.topic}:{part}:{cfg.offset}"], schema=cfg.schema, group=cfg.group,
                     eof=True, config=cfg.kafka_config if not servers.startswith("fake://") else None,
                     shard="auto", assign=cfg.assign,
                     native=cfg.native_feed and dev.type == "cuda" and plan is None,
                     workers=cfg.feed_workers, plan=plan, ordered=plan is not None)
        data = (s.filter_normal(device=True),) if cfg.model == "autoencoder" else (s, None)

    # ---------------------------------------------------------------- train
    from ..nn.callbacks import Callback

    class _Ckpt(Callback):
        def on_epoch_end(self, epoch, logs=None):
            if ckpt_dir and (epoch + 1) % int(job["ckpt_every"]) == 0:
                rs.save_checkpoint(self.model, ckpt_dir, epoch + 1, extra={"loss": (logs or {}).get("loss")})

    t0 = time.perf_counter()
    if plan is not None:   # continuous: one bounded segment per "epoch", positions checkpointed
        hist = _continuous(model, data[0], plan, cfg, job, ckpt_dir, start_epoch, rank, world, rs)
    elif cfg.model == "autoencoder":
        hist = model.fit(data[0], epochs=cfg.epochs, batch_size=cfg.batch_size, verbose=1 if rank == 0 else 0,
                         callbacks=[_Ckpt()], shuffle=True, seed=cfg.seed, initial_epoch=start_epoch,
                         steps_per_epoch=cfg.take)
    else:
        hist = model.fit(data[0], data[1], epochs=cfg.epochs, batch_size=cfg.batch_size, take=cfg.take,
                         verbose=1 if rank == 0 else 0, callbacks=[_Ckpt()], shuffle=True, seed=cfg.seed,
                         initial_epoch=start_epoch)
    dt = time.perf_counter() - t0
    if ckpt_dir and rank == 0:
        model.save(os.path.join(ckpt_dir, cfg.model_file))
    if rank == 0:
        losses = hist.history.get("loss", [])
        line = {"job": "train", "model": cfg.model, "world_size": world, "resumed_from_epoch": start_epoch,
                "epochs": cfg.epochs, "final_loss": losses[-1] if losses else None,
                "seconds": round(dt, 3), "ckpt_dir": ckpt_dir}
        if plan is not None:
            line["positions"] = getattr(hist, "positions", {})
            line["segment_records"] = hist.history.get("records", [])
            line["segment_loss"] = losses
        print(json.dumps(line), flush=True)
    shutdown()
    return 0


def _continuous(model, data, plan, cfg, job, ckpt_dir, start_seg, rank, world, rs):
    """Segments ``start_seg .. cfg.epochs - 1``: train the next bounded segment of every owned
    partition (every record of it: no ``take`` cap, no shuffle -- the step boundaries are a pure
    function of the positions), advance the positions, checkpoint them with the model."""
    from ..nn.callbacks import History
    from ..parallel.dp import _pg_active
    hist = History()
    hist.history = {"loss": [], "records": []}
    for seg in range(start_seg, cfg.epochs):
        h = model.fit(data, epochs=seg + 1, initial_epoch=seg, batch_size=cfg.batch_size, verbose=0,
                      shuffle=False, seed=cfg.seed)
        n = plan.segment_records()
        plan.advance()
        hist.history["loss"].extend(h.history.get("loss", []))
        hist.history["records"].append(n)
        offsets = plan.offsets()
        if _pg_active():   # every rank's partitions: one map (the ranks' partitions are disjoint)
            import torch.distributed as dist
            parts = [None] * world
            dist.all_gather_object(parts, offsets)
            offsets = {k: v for d in parts for k, v in d.items()}
        if ckpt_dir and (seg + 1) % int(job["ckpt_every"]) == 0:
            loss = h.history.get("loss", [None])[-1]
            rs.save_checkpoint(model, ckpt_dir, seg + 1, offsets=offsets, extra={"loss": loss, "segment_rows":
                                                                                int(job["segment_rows"])})
            if cfg.group:   # Kafka semantics too: the group's committed offsets follow the checkpoints
                try:
                    from ..kafka.client import KafkaClient
                    c = KafkaClient(cfg.servers, cfg.kafka_config if not cfg.servers.startswith("fake://") else None)
                    for k, v in plan.offsets().items():
                        t, p = k.rsplit(":", 1)
                        c.commit(cfg.group, t, int(p), int(v))
                except Exception as e:  # noqa: BLE001 - advisory; the checkpoint is the source of truth
                    print(f"[train] group commit failed: {e!r}", file=sys.stderr)
        hist.positions = offsets
    if not hasattr(hist, "positions"):
        hist.positions = plan.offsets()
    return hist


if __name__ == "__main__":
    sys.exit(main(sys.argv[1:]))
