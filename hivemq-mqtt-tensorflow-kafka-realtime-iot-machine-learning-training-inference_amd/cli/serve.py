"""``serve``: long-running, sharded streaming anomaly scorer (BASELINE config 5).

The reference scales inference by running ``cardata-v3.py ... predict`` as a K8s
Deployment that K8s restarts after every bounded run (python-scripts/README.md:24,
AUTOENCODER-TensorFlow-IO-Kafka/model-predictions.yaml). Each run reads partition 0
only (cardata-v3.py:46) and writes reconstructions (cardata-v3.py:243-249). Here:

* one replica per GPU. Replica ``r`` of ``W`` owns the Kafka partitions ``p`` with
  ``p % W == r``. The producers (MQTT bridge, ``produce``) partition by murmur2(car key),
  so this is shard-by-key: every car's events reach the same GPU, in order;
* the replica follows the log (no eof) and commits its offsets to the consumer group
  after each produced batch. A restarted replica resumes where it stopped, with no K8s
  restart loop and no re-scoring;
* every event is scored on the GPU (reconstruction MSE, K12), flagged with the
  notebook's fixed threshold (``threshold_fixed = 5``), and written to the result
  topic keyed by car: ``{"car", "partition", "offset", "score", "anomaly"}``, plus the
  reconstruction with ``--emit both`` (what the reference streams).

``--low-latency``: the whole per-event path runs in one C++ thread per replica
(:class:`streamml.kafka.scoreloop.LowLatencyScorer`): long-poll fetch -> Avro decode (or,
``--source-format json``, the bridge's JSON events) -> the persistent GPU scorer
(:class:`streamml.ops.serve.ScoringServer`; ``--model lstm``: the per-car forecaster
:class:`~streamml.ops.serve.LSTMScoringServer`, car key -> device slot in C++), no launch
per event -> the same result records formatted in C++ -> one produce per fetch -> commit.

Replica identity comes from ``--replica-index/--replicas``, else torchrun's
``RANK/WORLD_SIZE``, else ``REPLICA_INDEX/REPLICAS`` (a StatefulSet ordinal), else 0/1.
"""
from __future__ import annotations

import json
import os
import time
from typing import List, Sequence, Tuple

import numpy as np

from ..kafka.assign import HASH_SPACE
from ..ops._ext import load_io
from ..utils.affinity import parse_cpus, resolve_cpus  # noqa: F401  (serve.parse_cpus)
from . import common

USAGE = ("python -m streamml.cli serve <servers> <topic> <result_topic> <model-file> "
         "[--project P] [--replicas W --replica-index R] [--threshold 5] [--max-events N]")


def shard_partitions(n_partitions: int, rank: int, world: int) -> List[int]:
    """Whole partitions round-robin (``p % world == rank``): Kafka consumer-group semantics,
    skewed when ``world`` does not divide the partition count (8 replicas over the reference's
    10 partitions: 2 vs 1).  ``serve`` uses :func:`serve_shares` instead."""
    return [p for p in range(int(n_partitions)) if p % int(world) == int(rank)]


def serve_shares(n_partitions: int, rank: int, world: int):
    """Replica ``rank``'s ``(partition, hash_lo, hash_hi)`` key shares (kafka/assign.py "keys"):
    the partitions laid on a line, each replica owning ``P / W`` of it; where a cut falls
    inside a partition, its car keys are split by a 32-bit key hash.  Every car is scored by
    exactly one replica, in order, and the replicas' loads are equal at any ``W``."""
    from ..kafka.assign import key_shares
    return key_shares(n_partitions, rank, world)


def replica_identity(ns) -> Tuple[int, int]:
    if ns.replicas is not None:
        return int(ns.replica_index or 0), int(ns.replicas)
    for r_key, w_key in (("RANK", "WORLD_SIZE"), ("REPLICA_INDEX", "REPLICAS")):
        if w_key in os.environ:
            return int(os.environ.get(r_key, "0")), int(os.environ[w_key])
    return 0, 1


def _flags(p) -> None:
    p.add_argument("--project", default="car-demo", help="model store bucket suffix (cardata-v3 <project>)")
    p.add_argument("--group", default="streamml-serve", help="consumer group for committed offsets")
    p.add_argument("--replicas", type=int, default=None)
    p.add_argument("--replica-index", type=int, default=None)
    p.add_argument("--partitions", type=int, default=None, help="partition count (default: broker metadata)")
    p.add_argument("--from-beginning", action="store_true",
                   help="ignore committed offsets and start at the earliest record")
    p.add_argument("--threshold", type=float, default=5.0)
    p.add_argument("--emit", choices=["score", "both"], default="score")
    p.add_argument("--max-batch", type=int, default=1 << 16, help="rows per device scoring call")
    p.add_argument("--max-events", type=int, default=0, help="stop after this many events (0 = run forever)")
    p.add_argument("--idle-timeout", type=float, default=None, help="stop after this many idle seconds")
    p.add_argument("--synthetic-partitions", type=int, default=8)
    p.add_argument("--metrics-port", type=int, default=0)
    p.add_argument("--schema", default="cardata-v1")
    p.add_argument("--low-latency", action="store_true",
                   help="C++ fetch/decode/score/format/produce loop on the persistent GPU scorer")
    p.add_argument("--max-wait-ms", type=int, default=100, help="long-poll bound of the low-latency loop")
    p.add_argument("--spin-us", type=int, default=0,
                   help="low-latency loop: busy-poll each broker response this long before blocking")
    p.add_argument("--cpus", default=None,
                   help="--low-latency: CPUs for the loop thread, e.g. '4' or '4-7,12', or 'auto' (one core of "
                        "an L3 domain, a different one per replica); a loopback hop across core "
                        "complexes costs microseconds (profiles/r04 SUMMARY §7)")
    p.add_argument("--model", choices=["autoencoder", "lstm"], default="autoencoder",
                   help="lstm: per-car forecaster (look_back events per car on the device, each event "
                        "scored against the car's previous forecast; lstm_serve.hip)")
    p.add_argument("--max-keys", type=int, default=200_000, help="--model lstm: car keys held on the device")
    p.add_argument("--source-format", choices=["avro", "json"], default="avro",
                   help="--low-latency: json follows the MQTT bridge's JSON events (sensor-data, KSQL "
                        "SENSOR_DATA_S) directly instead of the Avro stream")


def seed_group_offsets(client, topic: str, base: str, group: str, partitions, max_world: int = 16) -> dict:
    """Rescaled serving: the consumer group of a replica that shares partitions is tied to the
    replica count (``<base>.<rank>-of-<world>``), so after a rescale it starts with no committed
    positions.  For every partition the group has no commit for, seed it with the MINIMUM position
    committed by the base group or any ``<base>.<r>-of-<w>`` group of ANOTHER replica count
    (w <= ``max_world``): at-least-once -- records between that minimum and another replica's
    position are scored again, none is skipped.  The sibling groups of the current
    count are not candidates: each tracks only ITS key share of a shared partition, so a sibling
    that already ran would otherwise make this replica skip its own share.
    Returns {partition: seeded offset}."""
    seeded = {}
    cur = group.rsplit("-of-", 1)[1] if "-of-" in group else None
    cands = [base] + [f"{base}.{r}-of-{w}" for w in range(2, max_world + 1) for r in range(w) if str(w) != cur]
    for p in partitions:
        if client.committed(group, topic, p) >= 0:
            continue
        pos = [o for o in (client.committed(g, topic, p) for g in cands if g != group) if o >= 0]
        if pos:
            client.commit(group, topic, p, min(pos))
            seeded[int(p)] = min(pos)
    return seeded


def _serve_low_latency(ns, servers, cfg, model, mine, result_parts, summary, rank: int = 0,
                       hash_ranges=None) -> int:
    """One C++ loop per replica over the resident scorer: the autoencoder's, or -- ``--model
    lstm`` -- the per-car forecaster, whose car key -> device slot map lives in the loop
    (cardata-v2.py:220-273 streams one LSTM prediction per event)."""
    from ..kafka.scoreloop import LowLatencyScorer
    from ..obs.metrics import ENGINE
    from ..ops.serve import LSTMScoringServer, ScoringServer

    if model.device.type != "cuda":
        raise SystemExit("--low-latency needs a ROCm device (the persistent scorer)")
    scorer = (LSTMScoringServer(model, nkeys=ns.max_keys, threshold=ns.threshold) if ns.model == "lstm"
              else ScoringServer(model, threshold=ns.threshold))
    with scorer as srv:
        starts = None
        if ns.from_beginning:
            from ..kafka import KafkaClient
            c = KafkaClient(servers, cfg)
            starts = [c.earliest(ns.topic, p) for p in mine]
        loop = LowLatencyScorer(servers, ns.topic, ns.result_topic, mine, srv, schema=ns.schema, group=ns.group,
                                starts=starts, result_partitions=[p % result_parts for p in mine],
                                emit_recon=ns.emit == "both", config=cfg, max_batch=min(ns.max_batch, 4096),
                                max_wait_ms=ns.max_wait_ms, spin_us=ns.spin_us, source_format=ns.source_format,
                                hash_ranges=hash_ranges)
        mask = os.sched_getaffinity(0)
        cpus = resolve_cpus(ns.cpus, slot=rank)
        if cpus:
            os.sched_setaffinity(0, cpus)   # this (the loop's) thread
        try:
            st = loop.run(max_events=ns.max_events, idle_timeout_s=ns.idle_timeout)
        finally:
            os.sched_setaffinity(0, mask)
    ENGINE.infer_rows.inc(st["events"], model=model.name)
    ENGINE.anomaly_events.inc(st["anomalies"], model=model.name)
    if ns.model == "lstm":
        summary.update(model="lstm", keys=st["keys"])
    summary.update(events=st["events"], anomalies=st["anomalies"], skipped=st["skipped"], foreign=st["foreign"],
                   keys_dropped=st["keys_dropped"],
                   events_per_s=st["events"] / st["wall_s"] if st["wall_s"] > 0 else 0.0, low_latency=True,
                   stages_s={k: st[k] for k in ("fetch_s", "decode_s", "score_s", "format_s", "produce_s",
                                                 "commit_s")})
    print(json.dumps(summary), flush=True)
    return 0


def main(argv: Sequence[str]) -> int:
    common.print_options(argv)
    ns = common.parse(argv, USAGE, ["servers", "topic", "result_topic", "model_file"], add_flags=_flags)
    from ..data.stream import LABEL_MISSING, kafka
    from ..kafka import KafkaClient, KafkaOutputSequence
    from ..models.autoencoder import load_model
    from ..obs.metrics import ENGINE, REGISTRY
    from ..utils.model_store import autoencoder_store

    rank, world = replica_identity(ns)
    servers = common.prepare_servers(ns.servers, ns.topic, seed=ns.synthetic_seed, schema=ns.schema,
                                     partitions=ns.synthetic_partitions)
    cfg = common.kafka_config(ns.servers, ns.kafka_config)
    device = ns.device
    if device == "auto":
        import torch
        device = f"cuda:{int(os.environ.get('LOCAL_RANK', '0'))}" if torch.cuda.is_available() else "cpu"

    path = common.model_path(ns.workdir, ns.model_file)
    if not os.path.exists(path):
        if ns.model == "lstm":
            from ..utils.model_store import lstm_store
            lstm_store(ns.store).download(ns.model_file, path)
        else:
            autoencoder_store(ns.project, ns.store).download("/" + ns.model_file, path)
    if ns.model == "lstm":
        from ..models.lstm import LSTMPredictor
        model = LSTMPredictor.load(path, device=device)
    else:
        model = load_model(path, device=device, input_normalizer="cardata")
    if ns.metrics_port and rank == 0:
        REGISTRY.serve(ns.metrics_port, addr="0.0.0.0")

    meta = KafkaClient(servers, cfg).partitions()
    n_parts = ns.partitions or meta.get(ns.topic, 1)
    if ns.result_topic not in meta and servers.startswith("fake://"):
        from ..kafka import fake_broker
        try:   # the reference creates model-predictions with the source topic's partition count
            fake_broker(servers[len("fake://"):] or "default").create_topic(ns.result_topic, n_parts)
        except Exception:
            pass   # another replica created it first
        meta = KafkaClient(servers, cfg).partitions()
    result_parts = max(1, meta.get(ns.result_topic, 1))
    shares = serve_shares(n_parts, rank, world)
    mine = [p for p, _, _ in shares]
    partial = any(not (lo == 0 and hi == HASH_SPACE) for _, lo, hi in shares)
    base_group = ns.group
    if partial:   # a shared partition's position is per replica: its own consumer group
        ns.group = f"{ns.group}.{rank}-of-{world}"
    if not ns.from_beginning:
        seed_group_offsets(KafkaClient(servers, cfg), ns.topic, base_group, ns.group, [p for p, _, _ in shares])
    print(f"replica {rank}/{world}: partitions {mine} of {n_parts} on {device}", flush=True)
    summary = {"replica": rank, "replicas": world, "partitions": mine, "events": 0, "anomalies": 0,
               "key_shares": [[p, lo / HASH_SPACE, hi / HASH_SPACE] for p, lo, hi in shares], "group": ns.group}
    if not mine:
        print(json.dumps(summary), flush=True)
        return 0

    if ns.source_format == "json" and not ns.low_latency:
        raise SystemExit("--source-format json needs --low-latency (the C++ loop decodes the JSON events)")
    if ns.low_latency:
        return _serve_low_latency(ns, servers, cfg, model, mine, result_parts, summary, rank,
                                  [(lo, hi) for _, lo, hi in shares])
    forecaster, key_ids = None, {}
    if ns.model == "lstm":
        if model.device.type != "cuda":
            raise SystemExit("--model lstm serving needs a ROCm device (the persistent forecaster)")
        from ..ops.serve import LSTMScoringServer
        forecaster = LSTMScoringServer(model, nkeys=ns.max_keys, threshold=ns.threshold)
    start = -2 if ns.from_beginning else 0
    # every partition listed; the plan keeps this replica's key shares (records of a shared
    # partition whose car another replica owns are dropped after decode)
    topics = [f"{ns.topic}:{p}:{start}" for p in range(n_parts)]
    stream = kafka(servers, topics, schema=ns.schema, group=ns.group, eof=False, config=cfg, commit=True,
                   resume=not ns.from_beginning, idle_timeout_s=ns.idle_timeout, shard=(rank, world), assign="keys")
    sinks, next_index = {}, {}
    t0 = time.perf_counter()
    for chunk in stream:
        part = int(chunk.meta.get("partition", 0))
        sink = sinks.get(part)
        if sink is None:   # results keep the source partition: a car's scores stay ordered
            sink = sinks[part] = KafkaOutputSequence(ns.result_topic, servers, cfg, partition=part % result_parts)
            next_index[part] = 0
        ok = chunk.meta.get("ok")                  # undecodable records are skipped, not scored
        ok = (chunk.label != LABEL_MISSING) if ok is None else ok.astype(bool)
        if not ok.all():
            chunk = chunk.select(ok)
        if len(chunk) == 0:
            continue
        t_batch = time.perf_counter()
        recon = None
        if forecaster is not None:
            # car key -> device slot (first come, first served; the table holds --max-keys cars)
            ids = np.empty(len(chunk), np.int64)
            for i, k in enumerate(chunk.keys or [None] * len(chunk)):
                kid = key_ids.get(k)
                if kid is None:
                    if len(key_ids) >= ns.max_keys:
                        raise SystemExit(f"more than --max-keys {ns.max_keys} cars on this replica")
                    kid = key_ids[k] = len(key_ids)
                ids[i] = kid
            pred, scores, fl = forecaster.forecast(chunk.x, ids)
            flags = fl == 1               # 2 = the car has no forecast yet (score NaN)
            if ns.emit == "both":
                recon = pred
        elif ns.emit == "both":
            recon, scores = model.reconstruct_and_score(chunk.x, batch_size=ns.max_batch)
            flags = scores > ns.threshold
        else:
            scores = model.score(chunk.x, batch_size=ns.max_batch)
            flags = scores > ns.threshold
        dt_us = (time.perf_counter() - t_batch) * 1e6 / len(chunk)
        keys = chunk.keys or [None] * len(chunk)
        offs = chunk.offsets if chunk.offsets is not None else np.arange(len(chunk))
        # json.dumps({car, partition, offset, score, anomaly[, reconstruction]}) per event, in C++
        recs = load_io().score_records(list(keys), part, np.asarray(offs, np.int64), np.asarray(scores, np.float32),
                                       np.asarray(flags, np.uint8), recon)
        sink.extend(next_index[part], recs, keys)   # one bulk append, no per-event Python loop
        next_index[part] += len(chunk)
        sink.flush()   # produced before the dataset commits this batch's offsets (at-least-once)
        n_flag = int(flags.sum())
        ENGINE.infer_rows.inc(len(chunk), model=model.name)
        ENGINE.anomaly_events.inc(n_flag, model=model.name)
        ENGINE.infer_latency.observe(dt_us)
        summary["events"] += len(chunk)
        summary["anomalies"] += n_flag
        if ns.max_events and summary["events"] >= ns.max_events:
            break
    for sink in sinks.values():
        sink.flush()
    if forecaster is not None:
        forecaster.close()
        summary["model"] = "lstm"
        summary["keys"] = len(key_ids)
    wall = time.perf_counter() - t0
    summary["events_per_s"] = summary["events"] / wall if wall > 0 else 0.0
    print(json.dumps(summary), flush=True)
    return 0
