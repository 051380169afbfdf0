#!/usr/bin/env python3
"""BASELINE config 5: streaming inference -- load a .h5 autoencoder, per-event MSE anomaly score.

Measures (1) p50 / p99 per-event latency at a fixed offered rate (default the
reference fleet's 10 000 msg/s, scenario.xml: 100 000 cars x 1 msg / 10 s): each
event is copied from pinned host memory, scored by the fused HIP forward kernel
and the score copied back; latency is event-available -> score-on-host.
(2) batched scoring throughput (events/s) for micro-batches of a stream.
With torchrun, every rank serves its own car-key shard (shard-by-key) and rank
0 reports the aggregate.  The reference publishes no latency number.
"""
import argparse
import itertools
import json
import os
import sys
import tempfile
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


_E2E_RUNS = itertools.count()


def _serving_cpus(k: int):
    """``k`` CPUs of this process's affinity set for the spinning serving threads, one per
    physical core where the topology says which CPUs are SMT siblings (None: too few)."""
    cpus = sorted(os.sched_getaffinity(0))
    if len(cpus) < k + 2:   # leave room for the broker's connection threads
        return None
    picked, seen = [], set()
    for c in reversed(cpus):
        try:
            with open(f"/sys/devices/system/cpu/cpu{c}/topology/thread_siblings_list") as f:
                core = f.read().strip()
        except OSError:
            core = str(c)
        if core in seen:
            continue
        seen.add(core)
        picked.append(c)
        if len(picked) == k:
            return picked
    return None


def _l3_cpus(k: int, slot: int = 0):
    """streamml.utils.affinity.l3_cpus: ``k`` distinct cores of one L3 domain (None: unknown)."""
    from streamml.utils.affinity import l3_cpus
    return l3_cpus(k, slot)


def kafka_e2e(m, ev, qps, threshold, events, rank=0, warm=100, spin_us=200, pin=None, make_scorer=None):
    """Kafka append -> result append latency through the real serving path: a paced C++
    producer appends Confluent-Avro car events (one produce request each, keyed by car) to
    an in-process broker at ``qps``; the ``serve --low-latency`` loop (long-poll fetch, C++
    decode, persistent GPU scorer, C++ JSON records, produce acks=1) runs in its own thread.

    Primary latency: the broker's append time (LogAppendTime, same steady clock) of an
    event's result record minus that of the event itself -- Kafka-append -> result
    visible to consumers.  Also reported: producer-send -> result-produce-ack (both client
    legs included).  ``spin_us``: the low-latency socket policy (broker connection threads,
    long polls and the loop's client busy-poll this long before blocking).  ``pin``: ``"l3"``
    (the default where the topology is readable; ``SML_E2E_PIN=0`` turns it off) puts the
    scoring loop, the producer and the broker's connection threads on distinct cores of ONE
    L3 domain -- unpinned, each loopback hop took ~2.3 or ~4.7 us depending on where the
    scheduler placed the threads (profiles/r04); ``"cores"`` pins only the loop and the
    producer (distinct physical cores, any L3); ``False`` leaves placement to the scheduler.
    ``make_scorer``: the resident scorer to serve with (default the autoencoder's
    ``ScoringServer``; e.g. an ``LSTMScoringServer``, whose car keys the loop maps to device
    slots in C++)."""
    import threading

    import numpy as np
    from streamml.data.avro import AvroCodec
    from streamml.data.produce import encode_chunk
    from streamml.kafka import fake_broker
    from streamml.kafka.scoreloop import LowLatencyScorer, paced_produce
    from streamml.ops.serve import ScoringServer

    n = events + warm
    # a fresh broker per call (bench.py re-executes this module per use: the counter alone
    # would repeat, so the name also carries a nanosecond stamp)
    name = f"bench-e2e-{os.getpid()}-{rank}-{spin_us}-{next(_E2E_RUNS)}-{time.time_ns()}"
    b = fake_broker(name)
    b.create_topic("SENSOR_DATA_S_AVRO", 1)
    b.create_topic("model-predictions", 1)
    b.record_append_times(True)
    b.set_spin_us(spin_us)
    if pin is None:
        pin = "l3" if os.environ.get("SML_E2E_PIN", "1") != "0" else False
    cpus = None
    if pin == "l3":
        cpus = _l3_cpus(5, rank)
        if cpus:
            b.set_thread_cpus(cpus[2:])   # before any client connects
    buf, offs = encode_chunk(AvroCodec("cardata-v1"), np.ascontiguousarray(ev[:n], np.float32),
                             np.zeros(n, np.uint8))
    keys = [f"car{i % 1000}" for i in range(n)]
    out = {}
    with (make_scorer() if make_scorer is not None else ScoringServer(m, threshold=threshold, slots=4096)) as srv:
        loop = LowLatencyScorer(f"fake://{name}", "SENSOR_DATA_S_AVRO", "model-predictions", [0], srv, starts=[0],
                                max_wait_ms=100, record_latency=True, spin_us=spin_us)
        if pin and pin != "l3":
            cpus = _serving_cpus(2)

        def serve():
            if cpus:
                os.sched_setaffinity(0, {cpus[0]})   # this thread only (Linux: pid 0 = calling thread)
            out.update(loop.run(max_events=n, idle_timeout_s=10.0))

        th = threading.Thread(target=serve)
        th.start()
        main_mask = os.sched_getaffinity(0)
        if cpus:
            os.sched_setaffinity(0, {cpus[1]})
        try:
            sent = paced_produce(f"fake://{name}", "SENSOR_DATA_S_AVRO", 0, bytes(buf), offs, keys=keys, qps=qps,
                                 spin_us=spin_us)
        finally:
            os.sched_setaffinity(0, main_mask)
        th.join(120)
    b.set_spin_us(0)
    lat = loop.latency_records()
    lat = lat[np.argsort(lat[:, 1])]
    vis = lat[:, 2]
    d_ack = (vis[warm:] - sent[warm:]) / 1e3
    t_in = b.append_times("SENSOR_DATA_S_AVRO", 0, 0, n)
    t_res = b.append_times("model-predictions", 0, 0, n)
    d = (t_res[warm:] - t_in[warm:]) / 1e3
    lw, ti, tr = lat[warm:], t_in[warm:], t_res[warm:]
    med = lambda a: float(np.median(a)) / 1e3   # noqa: E731
    legs = {"append_to_fetched": med(lw[:, 3] - ti), "fetched_to_scored": med(lw[:, 4] - lw[:, 3]),
            "scored_to_formatted": med(lw[:, 5] - lw[:, 4]), "formatted_to_result_append": med(tr - lw[:, 5]),
            "result_append_to_ack": med(lw[:, 2] - tr)}
    st = out
    ev_n = max(st.get("events", 1), 1)
    return {"p50_us": float(np.percentile(d, 50)), "p99_us": float(np.percentile(d, 99)),
            "max_us": float(d.max()), "events": int(len(d)), "offered_qps": qps, "spin_us": spin_us,
            "latency": "broker append time of the event -> broker append time of its result record",
            "send_to_ack_p50_us": float(np.percentile(d_ack, 50)), "send_to_ack_p99_us": float(np.percentile(d_ack, 99)),
            "legs_p50_us": legs, "pinned_cpus": cpus, "pin": pin if cpus else False,
            "results": int(b.end_offset("model-predictions", 0)),
            "batches": st.get("batches"), "events_per_batch": ev_n / max(st.get("batches", 1), 1),
            "per_event_us": {k[:-2]: st[k] / ev_n * 1e6 for k in ("decode_s", "score_s", "format_s",
                                                                 "produce_s", "commit_s") if k in st},
            "path": "paced producer -> broker (long-poll) -> C++ decode -> persistent GPU scorer -> "
                    "C++ JSON -> produce acks=1"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default=None, help=".h5 to load (default: save a fresh 18-dim AE first)")
    ap.add_argument("--events", type=int, default=2000)
    ap.add_argument("--qps", type=float, default=10000.0)
    ap.add_argument("--batch", type=int, default=65536)
    ap.add_argument("--threshold", type=float, default=5.0)
    args = ap.parse_args()
    import numpy as np
    import torch
    from streamml.data.cardata import synthetic_device_tensor
    from streamml.models.autoencoder import Autoencoder, load_model
    from streamml.parallel import dp

    env = dp.init_from_env("cuda")
    dev = env.device
    path = args.model
    if path is None:
        path = os.path.join(tempfile.gettempdir(), f"bench_ae_{os.getpid()}.h5")
        Autoencoder(device="cpu").save(path)   # every rank writes its own copy (same seed -> same weights)
    m = load_model(path, device=dev, input_normalizer="cardata")
    be = m.backend
    ev = synthetic_device_tensor(args.events + 100, dev, seed=env.rank, shard=env.rank,
                                 n_shards=env.world_size).cpu().numpy()
    host = torch.empty((1, 18), dtype=torch.float32).pin_memory()
    out = torch.empty(1, dtype=torch.float32).pin_memory()
    xdev = torch.empty((1, 18), dtype=torch.float32, device=dev)
    lat = []
    period = 1.0 / args.qps
    t_next = time.perf_counter()
    for i in range(args.events + 100):
        while time.perf_counter() < t_next:
            pass
        host.copy_(torch.from_numpy(ev[i:i + 1]))
        t0 = time.perf_counter()
        xdev.copy_(host, non_blocking=True)
        _, s, _ = be.forward(xdev, recon=False, score=True)
        out.copy_(s, non_blocking=True)
        torch.cuda.current_stream().synchronize()
        t1 = time.perf_counter()
        if i >= 100:
            lat.append((t1 - t0) * 1e6)
        t_next += period
    lat = np.asarray(lat)
    # persistent scorer: resident wave polling a host-mapped ring (no launch / copy per event)
    from streamml.ops.serve import ScoringServer
    with ScoringServer(m, threshold=args.threshold, slots=4096) as srv:
        srv.latency_us(ev[:100], qps=args.qps)                  # warm
        launches0 = srv.launches
        plat, pdev, pload, pcomp = srv.latency_us(ev[100:100 + args.events], qps=args.qps, device_breakdown=True)
        relaunches = srv.launches - launches0
        t0 = time.perf_counter()
        for k in range(20):
            srv.score(ev[:4096])
        srv_eps = 20 * 4096 / (time.perf_counter() - t0)
    # Kafka append -> result record visible (serve --low-latency: C++ loop + persistent scorer)
    e2e = kafka_e2e(m, ev, args.qps, args.threshold, args.events, env.rank)
    # batched throughput
    big = synthetic_device_tensor(args.batch * 8, dev, seed=1)
    for _ in range(3):
        be.forward(big[:args.batch], recon=False, score=True, threshold=args.threshold)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(40):
        j = k % 8
        be.forward(big[j * args.batch:(j + 1) * args.batch], recon=False, score=True, threshold=args.threshold)
    torch.cuda.synchronize()
    eps = args.batch * 40 / (time.perf_counter() - t0)
    # whole-job numbers: throughputs summed over the shard-by-key replicas, latency
    # percentiles as the worst replica's (conservative)
    p50, p99 = float(np.percentile(plat, 50)), float(np.percentile(plat, 99))
    eps_all, srv_all = eps, srv_eps
    if env.world_size > 1:
        t = torch.tensor([eps, srv_eps], device=dev, dtype=torch.float64)
        torch.distributed.all_reduce(t)
        eps_all, srv_all = float(t[0].item()), float(t[1].item())
        p50, p99 = dp.allreduce_max(p50, dev), dp.allreduce_max(p99, dev)
    if env.rank == 0:
        print(json.dumps({"metric": "p50 per-event inference latency (AE score)",
                          "value": p50, "unit": "us", "higher_is_better": False,
                          "p99_us": p99, "path": "persistent kernel, host-mapped ring",
                          "launch_path_p50_us": float(np.percentile(lat, 50)),
                          "launch_path_p99_us": float(np.percentile(lat, 99)),
                          "persistent_burst_events_per_s": srv_all,
                          "offered_qps_total": args.qps * env.world_size,
                          "persistent_device_p50_us": float(np.percentile(pdev, 50)),
                          "persistent_device_load_p50_us": float(np.percentile(pload, 50)),
                          "persistent_device_compute_p50_us": float(np.percentile(pcomp, 50)),
                          "persistent_relaunches": relaunches,
                          "offered_qps": args.qps, "events": args.events, "n_gpus": env.world_size,
                          "batched_events_per_s": eps_all, "batch": args.batch, "data": "synthetic",
                          "kafka_e2e_p50_us": e2e["p50_us"], "kafka_e2e_p99_us": e2e["p99_us"],
                          "kafka_e2e": e2e}))
    dp.shutdown()


if __name__ == "__main__":
    main()
