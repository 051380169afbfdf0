#!/usr/bin/env python3
"""The reference's own training job on the real entry point: ``Autoencoder.fit``.

cardata-v3 trains ``fit(zip((x, x)).batch(100).take(100), epochs=20)`` on the
label-filtered Kafka stream (AUTOENCODER-TensorFlow-IO-Kafka/cardata-v3.py:176-177,
212-222).  Two numbers:

* ``fit_batch100``: ``fit(array, batch_size=100, shuffle=True)`` -- one Keras Adam
  update per 100 rows, every step on the persistent kernel (rows/s);
* ``stream_e2e``: in-process Kafka broker (``partitions`` partitions of Confluent-framed
  Avro) -> fetch + decode -> pinned ring -> H2D -> K8 filter -> ``fit(batch_size=100)``
  (rows/s of consumed events), plus each host stage alone.

``measure(...)`` is also called by ``bench.py`` for its ``fit_batch100`` / ``stream_e2e``
fields.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def fit_array(device, rows: int = 2_000_000, batch: int = 100, engine: str = "auto", seed: int = 0,
              dp: str = "auto") -> dict:
    import numpy as np
    import torch

    from streamml.data.cardata import SyntheticCarSource
    from streamml.models.autoencoder import Autoencoder

    raw, _, _, _ = SyntheticCarSource.scenario("full", seed=seed, failure_rate=0.0).generate(rows)
    m = Autoencoder(device=device, input_normalizer="cardata", seed=seed)
    m.compile()
    x = torch.as_tensor(np.ascontiguousarray(raw, np.float32), device=device)
    m.fit(x[:batch * 200], epochs=1, batch_size=batch, verbose=0, engine=engine, dp=dp)   # warm-up
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    h = m.fit(x, epochs=1, batch_size=batch, verbose=0, engine=engine, dp=dp)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    steps = -(-rows // batch)
    return {"rows_per_s": rows / dt, "us_per_step": dt / steps * 1e6, "steps": steps, "batch": batch,
            "engine": m.last_fit_engine, "loss": h.history["loss"][-1], "dtype": "fp32"}


def stream_e2e(device, rows: int = 2_000_000, batch: int = 100, partitions: int = 8, workers: int = 8,
               fetch_bytes: int = 4 << 20, failure_rate: float = 0.01, native: bool = True, dp: str = "auto",
               compare_chunks: bool = False) -> dict:
    import torch

    from streamml.data import stream as S
    from streamml.data.avro import AvroCodec
    from streamml.data.produce import encode_chunk
    from streamml.kafka import fake_broker
    from streamml.models.autoencoder import Autoencoder

    name = f"bench-e2e-{rows}-{partitions}-{time.time_ns()}"
    b = fake_broker(name)
    topic = "SENSOR_DATA_S_AVRO"
    b.create_topic(topic, partitions)
    codec = AvroCodec("cardata-v1")
    t0 = time.perf_counter()
    # encode up to 1 M distinct events once, then append that record set round-robin until
    # `rows` events are in the log (a long run without a long Python encode)
    chunk = min(rows, 250_000)
    encoded = []
    for c in S.synthetic(min(rows, 1_000_000), chunk=chunk, seed=0, failure_rate=failure_rate):
        encoded.append(encode_chunk(codec, c.x, c.label) + (len(c.x),))
    t_encode = time.perf_counter() - t0
    left, i = rows, 0
    while left > 0:
        buf, offs, k = encoded[i % len(encoded)]
        if k > left:   # trim the last set to the exact event count
            buf, offs = buf[:offs[left]], offs[:left + 1]
            k = left
        b.append_buffer(topic, i % partitions, buf, offs)
        left -= k
        i += 1
    t_produce = time.perf_counter() - t0
    specs = [f"{topic}:{p}:0" for p in range(partitions)]
    src = S.kafka(f"fake://{name}", specs, max_bytes=fetch_bytes, workers=workers, native=native)
    out = {"rows": rows, "batch": batch, "partitions": partitions, "workers": workers,
           "produce_rows_per_s": rows / t_produce, "encode_s": t_encode, "native_feed": bool(native)}
    # stage 1: fetch + decode alone (host)
    t0 = time.perf_counter()
    n = src.count_rows() if hasattr(src, "count_rows") else sum(len(c) for c in src)
    out["fetch_decode_rows_per_s"] = n / (time.perf_counter() - t0)
    # stage 2: + pinned ring + H2D (+ K8 filter) into device chunks, no training
    m = Autoencoder(device=device, input_normalizer="cardata")
    m.compile()
    training = src.filter_normal(device=True)
    t0 = time.perf_counter()
    kept = 0
    for xd in m._stream_device_chunks(training):
        kept += int(xd.size(0))
    torch.cuda.synchronize()
    out["ingest_h2d_rows_per_s"] = n / (time.perf_counter() - t0)
    feed = getattr(src, "native_feed", None)
    if feed is not None:
        st = feed.last_stats
        out["feed_stats"] = st
        w = max(st.get("workers", 1), 1)
        out["per_worker_fetch_rows_per_s"] = st["records"] / max(st["fetch_s"] / w, 1e-9) / w
        out["per_worker_decode_rows_per_s"] = st["records"] / max(st["decode_s"] / w, 1e-9) / w
    # stage 3: the training kernel alone on the same number of rows (device resident)
    out["train_only"] = fit_array(device, rows=max(kept, batch * 300), batch=batch, dp=dp)
    # end to end
    m.fit(training, epochs=1, batch_size=batch, verbose=0, steps_per_epoch=50, dp=dp)   # warm-up
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    h = m.fit(training, epochs=1, batch_size=batch, verbose=0, dp=dp)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    out.update({"rows_per_s": n / dt, "kept_rows": kept, "trained_rows_per_s": kept / dt,
                "engine": m.last_fit_engine, "loss": h.history["loss"][-1],
                "epoch_launch": "doorbell" if os.environ.get("SML_STREAM_DOORBELL", "1") != "0" else "per-chunk"})
    if compare_chunks:   # the launch-per-chunk streaming epoch on the same log
        os.environ["SML_STREAM_DOORBELL"] = "0"
        try:
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            m.fit(training, epochs=1, batch_size=batch, verbose=0, dp=dp)
            torch.cuda.synchronize()
            out["per_chunk_rows_per_s"] = n / (time.perf_counter() - t0)
        finally:
            os.environ.pop("SML_STREAM_DOORBELL", None)
    return out


def _encode(rows, failure_rate=0.01, distinct=1_000_000):
    """The bench topic's distinct Confluent-Avro events: (buffer, offsets, count) chunks."""
    from streamml.data import stream as S
    from streamml.data.avro import AvroCodec
    from streamml.data.produce import encode_chunk
    codec = AvroCodec("cardata-v1")
    chunk = min(rows, 250_000)
    return [encode_chunk(codec, c.x, c.label) + (len(c.x),)
            for c in S.synthetic(min(rows, distinct), chunk=chunk, seed=0, failure_rate=failure_rate)]


def _fill_topic(b, topic, rows, partitions, failure_rate=0.01, distinct=1_000_000, staged=None):
    """Append ``rows`` Confluent-framed Avro events round-robin over ``partitions`` (up to
    ``distinct`` encoded once, then re-appended).  ``staged`` (a list): receives the encoded
    (buffer, offsets, count) chunks -- the same values, pre-staged in memory."""
    b.create_topic(topic, partitions)
    encoded = _encode(rows, failure_rate, distinct)
    if staged is not None:
        staged.extend(encoded)
    left, i, nbytes = rows, 0, 0
    while left > 0:
        buf, offs, k = encoded[i % len(encoded)]
        if k > left:
            buf, offs = buf[:offs[left]], offs[:left + 1]
            k = left
        b.append_buffer(topic, i % partitions, buf, offs)
        nbytes += int(offs[k])
        left -= k
        i += 1
    return nbytes


def _cpu_quota():
    """CPUs this process may keep busy (cgroup v2 cpu.max / v1 cfs quota), None if unlimited:
    the feed workers AND the in-process broker's connection threads share it."""
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()
        return None if q == "max" else round(int(q) / int(per), 2)
    except (OSError, ValueError):
        pass
    try:
        with open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us") as f:
            q = int(f.read())
        with open("/sys/fs/cgroup/cpu/cpu.cfs_period_us") as f:
            per = int(f.read())
        return None if q <= 0 else round(q / per, 2)
    except (OSError, ValueError):
        return None


def _broker_process(rows: int, partitions: int, cpus):
    """Start bench/broker_proc.py (pinned to ``cpus`` with taskset when given) and wait for its
    address line.  Returns (Popen, info dict)."""
    import json
    import shutil
    import subprocess
    import sys
    script = os.path.join(os.path.dirname(os.path.abspath(__file__)), "broker_proc.py")
    cmd = [sys.executable, script, "--rows", str(rows), "--partitions", str(partitions)]
    if cpus and shutil.which("taskset"):
        cmd = ["taskset", "-c", ",".join(str(c) for c in sorted(cpus))] + cmd
    proc = subprocess.Popen(cmd, stdin=subprocess.PIPE, stdout=subprocess.PIPE, text=True)
    line = proc.stdout.readline()
    if not line:
        proc.kill()
        raise RuntimeError("broker process exited before serving")
    return proc, json.loads(line)


def _split_cpus(broker_share: float = 0.25):
    """This process's CPUs split in two disjoint sets: (consumer, broker).  With a cgroup quota
    the split is sized by the quota (the CPUs both processes may keep busy), not the machine."""
    allowed = sorted(os.sched_getaffinity(0))
    quota = _cpu_quota()
    usable = allowed[:max(4, int(quota))] if quota else allowed
    nb = max(2, int(round(len(usable) * broker_share)))
    if len(usable) <= nb + 1:
        return set(allowed), None
    return set(usable[:-nb]), set(usable[-nb:])


def stream_large_batch(device, rows: int = 32_000_000, partitions: int = 32, batch: int = 1 << 20,
                       workers=(1, 2, 4, 8, 16, 32), train_workers: int = 0, broker: str = "process") -> dict:
    """Fresh rows at large batch: ``partitions`` partitions of Confluent
    Avro -> native C++ feed (one worker per partition group, pinned slabs, H2D in flight) ->
    ``fit(batch_size=batch, engine="throughput")`` over the stream, every epoch re-reading the
    log like the reference (cardata-v3.py:44-75, python-scripts/README.md:116).

    Reports the host fetch + decode rate against the number of feed workers (the slabs are
    recycled uncopied: the decode alone) and the end-to-end trained rows/s at the best
    worker count.  Each row is ~155 bytes on the wire, so 100 M rows/s is 15.5 GB/s of
    loopback Kafka traffic.

    ``broker="process"`` (default) serves the topic from bench/broker_proc.py, a child process on
    CPUs of its own (the reference's brokers are remote pods): the curve then prices the
    consumer's fetch + decode alone; ``"inproc"`` keeps the in-process broker."""
    from streamml.kafka import fake_broker

    name = f"bench-large-{rows}-{partitions}-{time.time_ns()}"
    topic = "SENSOR_DATA_S_AVRO"
    t0 = time.perf_counter()
    quota = _cpu_quota()
    proc, binfo = None, None
    mask0 = os.sched_getaffinity(0)
    if broker == "process":
        # the broker in a child process on CPUs of its own (the reference's brokers are remote pods);
        # this process's feed workers keep the rest
        mine, theirs = _split_cpus()
        proc, binfo = _broker_process(rows, partitions, theirs)
        src_addr = binfo["addr"]
        staged = _encode(rows)
        nbytes = int(binfo["log_bytes"])
        os.sched_setaffinity(0, mine)
    else:
        b = fake_broker(name)
        src_addr = f"fake://{name}"
        staged = []
        nbytes = _fill_topic(b, topic, rows, partitions, staged=staged)
    try:
        out = _stream_large_batch_on(device, src_addr, topic, rows, partitions, batch, workers, train_workers,
                                     staged, nbytes, quota, t0)
    finally:
        os.sched_setaffinity(0, mask0)
        if proc is not None:
            proc.stdin.close()
            try:
                proc.wait(timeout=30)
            except Exception:  # noqa: BLE001
                proc.kill()
    out["broker"] = ({"mode": "separate process", "pid": binfo["pid"], "cpus": binfo["cpus"],
                      "consumer_cpus": sorted(mine), "produce_s": binfo["produce_s"]}
                     if proc is not None else {"mode": "in-process"})
    return out


def _stream_large_batch_on(device, src_addr, topic, rows, partitions, batch, workers, train_workers, staged, nbytes,
                           quota, t0) -> dict:
    import torch

    from streamml.data import stream as S
    from streamml.models.autoencoder import Autoencoder

    import numpy as np

    out = {"rows": rows, "partitions": partitions, "batch": batch, "log_bytes": nbytes,
           "bytes_per_row": nbytes / rows, "produce_s": time.perf_counter() - t0,
           "cpus": os.cpu_count(), "affinity_cpus": len(os.sched_getaffinity(0)), "cpu_quota": quota}
    specs = [f"{topic}:{p}:0" for p in range(partitions)]
    # 1. the decoder alone: the same Avro values pre-staged in memory (as a fetch response holds
    #    them), decoded by W threads into private slabs -- no broker, no socket, no ring
    sizes = [int(s[1][s[2]]) for s in staged]
    buf = np.concatenate([np.frombuffer(s[0], np.uint8)[:n] for s, n in zip(staged, sizes)])
    bases = np.cumsum([0] + sizes[:-1])
    offs = np.concatenate([np.zeros(1, np.int64)] + [np.asarray(s[1][1:s[2] + 1], np.int64) + int(base)
                                                    for s, base in zip(staged, bases)])
    probe = S.kafka(src_addr, specs[:1], native=True).native_feed
    dcurve = []
    for w in tuple(workers) + ((32,) if 32 not in workers else ()):
        r, _ = probe.decode_only(buf, offs, int(w), repeats=2, keep_label=0)
        dcurve.append({"workers": int(w), "rows_per_s": r})
    out["decode_only_curve"] = dcurve
    out["decode_only_rows"] = int(len(offs) - 1)
    # 2. fetch + decode from the broker (its connection threads share this process's CPUs)
    curve = []
    for w in workers:
        src = S.kafka(src_addr, specs, max_bytes=8 << 20, workers=int(w), native=True)
        t1 = time.perf_counter()
        n = src.native_feed.count_rows()
        dt = time.perf_counter() - t1
        st = src.native_feed.last_stats
        curve.append({"workers": int(w), "rows_per_s": n / dt, "gb_per_s": n * out["bytes_per_row"] / dt / 1e9,
                      "fetch_s": st.get("fetch_s"), "decode_s": st.get("decode_s"),
                      "wait_slab_s": st.get("wait_slab_s")})
    out["decode_curve"] = curve
    best = max(curve, key=lambda c: c["rows_per_s"])
    tw = int(train_workers or best["workers"])
    src = S.kafka(src_addr, specs, max_bytes=8 << 20, workers=tw, native=True)
    training = src.filter_normal(device=True)
    m = Autoencoder(device=device, input_normalizer="cardata")
    m.compile()
    m.fit(training, epochs=1, batch_size=batch, verbose=0, steps_per_epoch=4, engine="throughput", dp="none")
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    h = m.fit(training, epochs=1, batch_size=batch, verbose=0, engine="throughput", dp="none")
    torch.cuda.synchronize()
    dt = time.perf_counter() - t1
    kept = int(h.history["_rows"][-1]) if "_rows" in h.history else None
    st = src.native_feed.last_stats
    out.update({"train_workers": tw, "rows_per_s": rows / dt, "trained_rows_per_s": (kept or 0) / dt,
                "kept_rows": kept, "engine": m.last_fit_engine, "loss": h.history["loss"][-1],
                "h2d_gb_per_s": st.get("h2d_bytes", 0) / dt / 1e9,
                "train_stage_s": {"wall": dt, "fetch_sum": st.get("fetch_s"), "decode_sum": st.get("decode_s"),
                                  "wait_slab_sum": st.get("wait_slab_s")}})
    # 3. the consumer side alone: the same values pre-staged in memory (8 copies of the distinct set),
    #    decoded by the feed workers straight into the pinned ring -> H2D -> fit(throughput); no broker
    #    threads on the CPUs ("pre-stage fetched record batches")
    reps = 8
    sbuf = np.tile(buf, reps)
    soffs = np.concatenate([offs[:-1] + k * len(buf) for k in range(reps)] + [np.array([reps * len(buf)], np.int64)])
    staged_runs = []
    for w in sorted({min(8, int(quota or 8)), max(1, min(16, int(quota or 16) - 2))}):
        ssrc = S.kafka(src_addr, specs[:1], workers=int(w), native=True)
        ssrc.native_feed.stage(sbuf, soffs)
        st_train = ssrc.filter_normal(device=True)
        ms = Autoencoder(device=device, input_normalizer="cardata")
        ms.compile()
        ms.fit(st_train, epochs=1, batch_size=batch, verbose=0, steps_per_epoch=2, engine="throughput", dp="none")
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        hs = ms.fit(st_train, epochs=2, batch_size=batch, verbose=0, engine="throughput", dp="none")
        torch.cuda.synchronize()
        dts = time.perf_counter() - t1
        kept_s = int(sum(hs.history["_rows"])) if "_rows" in hs.history else 0
        sst = ssrc.native_feed.last_stats
        staged_runs.append({"workers": int(w), "values": int(len(soffs) - 1) * 2, "trained_rows_per_s": kept_s / dts,
                            "decode_s_sum": sst.get("decode_s"), "wait_slab_s_sum": sst.get("wait_slab_s"),
                            "h2d_gb_per_s": sst.get("h2d_bytes", 0) / dts / 1e9})
    out["staged_train"] = {"runs": staged_runs, "best_trained_rows_per_s": max(r["trained_rows_per_s"]
                                                                                for r in staged_runs),
                           "path": "pre-staged record values -> feed workers decode into the pinned ring -> H2D -> "
                                   "fit(batch_size=1 M, engine=throughput); no broker"}
    # what caps the curve: the decoder alone against the fetch + decode path, within the CPUs
    # this job may keep busy (the feed workers, the broker's connection threads and the
    # training loop all draw on that one quota)
    dbest = max(dcurve, key=lambda c: c["rows_per_s"])
    per_worker = dcurve[0]["rows_per_s"]
    out["cap"] = {
        "decode_only_best": dbest, "fetch_decode_best": best,
        "decode_per_worker_rows_per_s": per_worker,
        "quota_cpus": quota,
        "decode_rows_per_s_at_quota": per_worker * quota if quota else None,
        "resource": ("CPU quota" if quota and dbest["workers"] <= quota * 1.5 else "decoder scaling"),
        "note": "fetch + decode needs ~2 CPUs per worker (decode thread + the broker's connection thread); "
                "the decode-only curve shows the decoder's own scaling on the same CPUs"}
    return out


def stream_dp(device, rank: int, world: int, rows_per_rank: int = 4_000_000, partitions: int = 10,
              batch: int = 1 << 20, workers: int = 4) -> dict:
    """Data-parallel training from ONE partitioned topic (BASELINE config 4 with the reference's
    ingestion path; SURVEY.md 2.4 stream / partition parallelism).  Collective: every rank calls it.

    Rank 0 hosts the in-process Kafka broker (127.0.0.1, reached by every rank over TCP like a
    broker of the cluster) and fills ``partitions`` partitions (the reference's sensor-data has
    10, 01_installConfluentPlatform.sh:180) with ``rows_per_rank x world`` Confluent-Avro car
    events.  Every rank streams its own share -- equal contiguous offset ranges of all
    partitions (kafka/assign.py "split") -- through its native feed (``workers`` threads) into
    ``fit(batch_size=batch, engine="throughput")``: one fused step + one flat RCCL all-reduce
    per batch, every filtered row of every share trained exactly once.  Whole-job trained
    rows/s over the slowest rank's epoch."""
    import torch
    import torch.distributed as dist

    from streamml.data import stream as S
    from streamml.models.autoencoder import Autoencoder
    from streamml.parallel import dp as dpm

    topic = "SENSOR_DATA_S_AVRO"
    broker, info = None, [None]
    if rank == 0:
        try:   # a failure here reaches every rank through the broadcast (no rank left waiting)
            from streamml.kafka import FakeBroker
            broker = FakeBroker()
            t0 = time.perf_counter()
            nbytes = _fill_topic(broker, topic, rows_per_rank * world, partitions)
            info = [{"addr": broker.address, "log_bytes": nbytes, "produce_s": time.perf_counter() - t0}]
        except Exception as e:  # noqa: BLE001
            info = [{"error": repr(e)[:300]}]
    dist.broadcast_object_list(info, src=0)
    info = info[0]
    if "error" in info:
        if broker is not None:
            broker.stop()
        raise RuntimeError(f"stream_dp setup on rank 0: {info['error']}")
    try:
        src = S.kafka(info["addr"], [f"{topic}:*:0"], shard="auto", assign="split", native=True,
                      workers=workers, max_bytes=8 << 20)
        training = src.filter_normal(device=True)
        m = Autoencoder(device=device, input_normalizer="cardata")
        m.compile()
        dpm.sync_model_from_rank0(m)
        m.fit(training, epochs=1, batch_size=batch, verbose=0, steps_per_epoch=2, engine="throughput", dp="rccl")
        torch.cuda.synchronize()
        dpm.barrier(device)
        t1 = time.perf_counter()
        h = m.fit(training, epochs=1, batch_size=batch, verbose=0, engine="throughput", dp="rccl")
        torch.cuda.synchronize()
        dpm.barrier(device)
        dt = dpm.allreduce_max(time.perf_counter() - t1, device)
        shares = [[s.partition, s.start, s.end] for s in src.plan.last]
        st = dict(src.native_feed.last_stats)
        chk = float(m.backend.params.double().sum())
        per_rank = [None] * world
        dist.all_gather_object(per_rank, {"shares": shares, "rows_read": st.get("records"), "kept": st.get("rows"),
                                          "iterations": m.iterations, "param_checksum": chk,
                                          "fetch_s": st.get("fetch_s"), "decode_s": st.get("decode_s")})
    finally:
        dpm.barrier(device)
        if broker is not None:
            broker.stop()
    trained = int(h.history["_rows"][-1])
    return {"trained_rows_per_s": trained / dt, "rows_per_s": rows_per_rank * world / dt, "seconds": dt,
            "rows": rows_per_rank * world, "trained_rows": trained, "partitions": partitions, "batch": batch,
            "global_batch": batch * world, "world": world, "feed_workers_per_rank": workers,
            "engine": m.last_fit_engine, "loss": h.history["loss"][-1], "assign": "split",
            "partition_lists": [sorted({s[0] for s in r["shares"]}) for r in per_rank], "per_rank": per_rank,
            "replicas_identical": len({r["param_checksum"] for r in per_rank}) == 1,
            "steps_equal": len({r["iterations"] for r in per_rank}) == 1, "broker": info,
            "path": "rank 0's in-process broker over TCP -> per-rank native feed (own offset ranges) -> "
                    "fit(throughput) + RCCL all-reduce per step"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=2_000_000)
    ap.add_argument("--batch", type=int, default=100)
    ap.add_argument("--partitions", type=int, default=8)
    ap.add_argument("--workers", default="8", help="comma-separated feed worker counts to sweep")
    ap.add_argument("--python-feed", action="store_true", help="chunk-by-chunk Python Kafka path")
    ap.add_argument("--skip-stream", action="store_true")
    ap.add_argument("--compare-chunks", action="store_true", help="also time the launch-per-chunk stream epoch")
    ap.add_argument("--large-batch", action="store_true", help="only the large-batch streaming measurement")
    args = ap.parse_args()
    if args.large_batch:
        import torch
        print(json.dumps(stream_large_batch(torch.device("cuda", 0), rows=args.rows)))
        return
    import torch
    dev = torch.device("cuda", 0)
    res = {"fit_batch100": fit_array(dev, args.rows, args.batch)}
    res["fit_batch32"] = fit_array(dev, args.rows // 2, 32)
    res["fit_launch_batch100"] = fit_array(dev, args.rows // 10, args.batch, engine="launch")
    if not args.skip_stream:
        res["stream_e2e"] = [stream_e2e(dev, args.rows, args.batch, args.partitions, int(w),
                                        native=not args.python_feed, compare_chunks=args.compare_chunks) for w in str(args.workers).split(",")]
    print(json.dumps(res))


if __name__ == "__main__":
    main()
