"""End-to-end device-fleet run: MQTT cars -> broker nodes -> Kafka bridge -> GPU scorer -> Kafka.

The reference's defining scale axis is "100000+ IoT connections" (``README.md:157``): the
device simulator connects 100 000 MQTT 5 clients and publishes one car payload per client
every 10 s (``infrastructure/test-generator/scenario.xml:13, 25, 48-49``: 10 000 msg/s) into
a 5-node HiveMQ cluster whose Kafka extension forwards ``vehicles/sensor/data/#`` to the
topic ``sensor-data`` (``infrastructure/hivemq/kafka-config.yaml:20-29``), from which the
model scores each event (``python-scripts/.../cardata-v3.py:235-279``).

:func:`run_fleet` stands the same pipeline up on one host:

* ``brokers`` broker-node processes (:mod:`streamml.mqtt.node`; the C++ epoll broker +
  bridge), each bridging into an in-process Kafka broker;
* ``agents`` simulator processes, agent ``i`` connecting its share of the cars to node
  ``i % brokers`` (each process has its own descriptor limit: 100 000 sockets on the
  client side and 100 000 on the broker side never share one process);
* in this process, one C++ scoring loop per scorer following ``sensor-data`` (the JSON
  events, KSQL's SENSOR_DATA_S) with the persistent GPU scorer(s) -- the autoencoder, and
  optionally the per-car LSTM forecaster -- writing a result record per event.

Every payload carries its CLOCK_MONOTONIC send time (``sent_ns``); the loop records when
each result became visible on the same clock, so the publish -> result latency is exact.
Counts at every hop (published, broker incoming, bridged to Kafka, scored, results) show
whether anything was dropped.
"""
from __future__ import annotations

import json
import os
import subprocess
import sys
import threading
import time
from typing import Dict, List, Optional

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def _spawn(args: List[str], stdin=subprocess.DEVNULL) -> subprocess.Popen:
    """A node / agent child.  Its stderr goes to an unlinked temporary file, never a pipe: a
    child writing more than a pipe buffer of warnings (per-connection errors over 20 000
    sockets) would block on a pipe nobody reads until the run's timeouts."""
    import tempfile
    env = dict(os.environ)
    env["PYTHONPATH"] = ROOT + (os.pathsep + env["PYTHONPATH"] if env.get("PYTHONPATH") else "")
    err = tempfile.TemporaryFile(mode="w+")
    p = subprocess.Popen([sys.executable, "-m", "streamml.mqtt.node"] + args, stdin=stdin,
                         stdout=subprocess.PIPE, stderr=err, cwd=ROOT, env=env, text=True)
    p.err_file = err   # type: ignore[attr-defined]
    return p


def _err_tail(p: subprocess.Popen, n: int = 800) -> str:
    f = getattr(p, "err_file", None)
    if f is None:
        return ""
    try:
        f.flush()
        f.seek(0)
        return f.read()[-n:]
    except (OSError, ValueError):
        return ""


def _json_line(p: subprocess.Popen, timeout_s: float) -> dict:
    """Next JSON line on a child's stdout (bounded wait)."""
    box: Dict[str, object] = {}

    def rd():
        for ln in p.stdout:
            if ln.startswith("{"):
                box["d"] = json.loads(ln)
                return

    t = threading.Thread(target=rd, daemon=True)
    t.start()
    t.join(timeout_s)
    if "d" not in box:
        raise RuntimeError(f"fleet child gave no JSON line within {timeout_s:.0f} s (rc={p.poll()}): {_err_tail(p)}")
    return box["d"]   # type: ignore[return-value]


def _rss_mb(pid: int) -> float:
    try:
        with open(f"/proc/{pid}/status") as f:
            for ln in f:
                if ln.startswith("VmRSS:"):
                    return int(ln.split()[1]) / 1024.0
    except OSError:
        pass
    return 0.0


def plan_processes(clients: int, per_process_max: int = 20_000) -> int:
    """Processes per side (broker nodes = simulator agents) for ``clients`` connections: each
    process holds one socket per car, so its share must fit the descriptor hard limit (which
    children inherit) and, per (source, broker port) pair, the ~28k loopback ephemeral ports."""
    import resource
    hard = resource.getrlimit(resource.RLIMIT_NOFILE)[1]
    cap = per_process_max if hard == resource.RLIM_INFINITY else max(64, min(per_process_max, int(hard) - 256))
    return max(1, -(-int(clients) // cap))


def _pct(a: np.ndarray, q: float) -> Optional[float]:
    return float(np.percentile(a, q)) if len(a) else None


def _windows(sent_ns: np.ndarray, us: np.ndarray, window_s: float, offered_per_s: float) -> List[dict]:
    """Per window of send time: events scored vs offered, p50 / p99 / max publish -> result us."""
    if not len(sent_ns):
        return []
    t = (sent_ns - sent_ns.min()) / 1e9
    idx = (t // window_s).astype(np.int64)
    out = []
    for w in range(int(idx.max()) + 1):
        u = us[idx == w]
        out.append({"t_s": w * window_s, "scored": int(len(u)), "offered": int(round(offered_per_s * window_s)),
                    "p50_us": _pct(u, 50), "p99_us": _pct(u, 99), "max_us": float(u.max()) if len(u) else None})
    return out


def run_fleet(scorer, clients: int = 10_000, interval_s: float = 1.0, messages: int = 10,
              brokers: Optional[int] = None, agents: Optional[int] = None, partitions: int = 10,
              threads: int = 4, qos: int = 0, lstm_scorer=None,
              name: str = "fleet", start_delay_s: Optional[float] = None, sources_per_agent: int = 1,
              max_wait_ms: int = 5, drain_timeout_s: float = 30.0, sample_s: float = 5.0,
              window_s: Optional[float] = None, retention_ms: int = 100_000) -> dict:
    """Run ``clients`` cars x ``messages`` events at ``clients / interval_s`` msg/s end to end.

    ``scorer``: a :class:`~streamml.ops.serve.ScoringServer` (or ``_io.EchoScorer`` on CPU);
    ``lstm_scorer``: optionally a :class:`~streamml.ops.serve.LSTMScoringServer` scoring the
    same events per car in a second loop.  Returns connections, connect time, offered and
    achieved rates, per-hop counts, drops and publish -> result latency percentiles (us).
    ``brokers`` / ``agents`` default to (and are raised to) what the descriptor limit needs
    (:func:`plan_processes`).

    Over time (a sustained run): every ``sample_s`` the broker nodes', agents' and this
    process's resident memory is sampled (``timeline.samples``), and the scored events are cut
    into ``window_s`` windows of result time (default: the send interval) with each window's
    count against the offered count and its p50 / p99 / max latency (``timeline.<scorer>``).

    The topics keep the reference's ``retention.ms=100000`` (01_installConfluentPlatform.sh:180,
    183; ``retention_ms``, -1 = unbounded): a sustained run's in-process Kafka log stays bounded
    (``timeline.samples[].kafka_log_mb``), as the reference's brokers keep theirs."""
    from ..kafka import fake_broker
    from ..kafka.scoreloop import LowLatencyScorer

    need = plan_processes(clients)
    brokers = max(int(brokers or 0), need)
    agents = max(int(agents or 0), brokers)
    t_begin = time.time()
    name = f"{name}-{os.getpid()}-{time.time_ns()}"   # a fresh in-process Kafka per run
    kb = fake_broker(name)
    topic, results, lresults = "sensor-data", "model-predictions", "lstm-predictions"
    for t in (topic, results) + ((lresults,) if lstm_scorer is not None else ()):
        kb.create_topic(t, partitions, retention_ms=retention_ms)
    total = clients * messages
    nodes = [_spawn(["broker", "--kafka", f"127.0.0.1:{kb.port}"], stdin=subprocess.PIPE) for _ in range(brokers)]
    agents_p: List[subprocess.Popen] = []
    try:
        ports = [_json_line(p, 60.0)["port"] for p in nodes]
        loops, outs, ths = [], [], []
        for sc, res in [(scorer, results)] + ([(lstm_scorer, lresults)] if lstm_scorer is not None else []):
            lp = LowLatencyScorer(f"fake://{name}", topic, res, list(range(partitions)), sc, starts=[0] * partitions,
                                  result_partitions=list(range(partitions)), max_wait_ms=max_wait_ms,
                                  record_latency=True, source_format="json", json_stamp="sent_ns")
            out: Dict[str, object] = {}
            th = threading.Thread(target=lambda lp=lp, out=out: out.update(lp.run(max_events=total)), daemon=True)
            th.start()
            loops.append(lp)
            outs.append(out)
            ths.append(th)
        samples: List[dict] = []
        stop_sampler = threading.Event()

        def sampler():
            while True:
                samples.append({"t_s": round(time.time() - t_begin, 2),
                                "broker_rss_mb": round(sum(_rss_mb(p.pid) for p in nodes), 1),
                                "agents_rss_mb": round(sum(_rss_mb(p.pid) for p in agents_p), 1),
                                "scorer_rss_mb": round(_rss_mb(os.getpid()), 1),
                                # the per-event latency records (the measurement, kept for the
                                # percentiles): 56 B per scored event and scorer
                                "latency_records_mb": round(sum(lp.latency_bytes() for lp in loops) / 1e6, 1),
                                "kafka_log_mb": round(kb.log_bytes() / 1e6, 1),
                                "kafka_deleted_records": int(kb.deleted_records)})
                if stop_sampler.wait(sample_s):
                    return

        sth = threading.Thread(target=sampler, daemon=True)
        sth.start()
        per = [clients * i // agents for i in range(agents + 1)]
        if start_delay_s is None:   # interpreter start + every agent's connects (~100 us each, serial per thread)
            start_delay_s = 3.0 + 2.0 * (max(per[i + 1] - per[i] for i in range(agents)) / max(threads, 1)) * 150e-6
        start_at = time.time() + start_delay_s
        for i in range(agents):
            n = per[i + 1] - per[i]
            srcs = ",".join(f"127.0.{1 + i}.{1 + s}" for s in range(sources_per_agent)) if sources_per_agent > 1 else ""
            agents_p.append(_spawn(["agent", "--port", str(ports[i % brokers]), "--clients", str(n), "--messages",
                                    str(messages), "--interval", str(interval_s), "--qos", str(qos), "--threads",
                                    str(threads), "--id-offset", str(per[i]), "--paced", "--start-at", repr(start_at),
                                    "--stamp", "--source-ips", srcs, "--seed", "7"]))
        run_s = start_delay_s + messages * interval_s + 120.0
        sims = [_json_line(p, run_s) for p in agents_p]
        for p in agents_p:
            p.wait(30)
        for p in nodes:       # stdin EOF: flush the bridge, print the node's counters
            p.stdin.close()
        nstats = [_json_line(p, 60.0) for p in nodes]
        for p in nodes:
            p.wait(30)
        published = sum(int(s["published"]) for s in sims)
        t_drain = time.time() + drain_timeout_s
        while time.time() < t_drain and any(th.is_alive() for th in ths):
            if all(int(o.get("events", 0) or 0) >= published for o in outs):
                break
            time.sleep(0.05)
        for lp in loops:
            lp.stop()
        for th in ths:
            th.join(10)
        stop_sampler.set()
        sth.join(10)
    finally:
        for p in agents_p + nodes:
            if p.poll() is None:
                p.kill()
    connected = sum(int(s["connected"]) for s in sims)
    out = {
        "clients": clients, "connections": connected, "connect_failed": sum(int(s["connect_failed"]) for s in sims),
        "brokers": brokers, "agents": agents, "kafka_partitions": partitions,
        "connect_s": max(float(s["connect_s"]) for s in sims),
        "offered_msgs_per_s": clients / interval_s, "messages_per_client": messages,
        "published": published, "publish_failed": sum(int(s["publish_failed"]) for s in sims),
        "publish_msgs_per_s": published / max(max(float(s["publish_s"]) for s in sims), 1e-9),
        "max_send_lag_ms": max(float(s["max_lag_ms"]) for s in sims),
        "sends_late_10ms": sum(int(s["late_10ms"]) for s in sims),
        "broker_incoming": sum(int(s["incoming_publish"]) for s in nstats),
        "bridged_to_kafka": sum(int(s["kafka_sent"]) for s in nstats),
        "bridge_failed": sum(int(s["kafka_failed"]) for s in nstats),
        "bridge_flushed": all(bool(s.get("flushed")) for s in nstats),
        "wall_s": time.time() - t_begin, "kafka": f"fake://{name}",
    }
    rss = [x["broker_rss_mb"] for x in samples if x["broker_rss_mb"] > 0]
    out["broker_rss_mb"] = {"first": rss[0] if rss else None, "last": rss[-1] if rss else None,
                            "max": max(rss) if rss else None}
    net = [x["scorer_rss_mb"] - x["latency_records_mb"] for x in samples]
    out["scorer_rss_mb"] = {"first": samples[0]["scorer_rss_mb"] if samples else None,
                            "last": samples[-1]["scorer_rss_mb"] if samples else None,
                            "last_less_latency_records": round(net[-1], 1) if net else None}
    logmb = [x["kafka_log_mb"] for x in samples]
    out["kafka_log"] = {"retention_ms": retention_ms, "max_mb": max(logmb) if logmb else None,
                        "last_mb": logmb[-1] if logmb else None,
                        "deleted_records": samples[-1]["kafka_deleted_records"] if samples else 0}
    out["timeline"] = {"samples": samples, "window_s": float(window_s or interval_s)}
    for tag, lp, o in zip(("ae", "lstm"), loops, outs):
        lat = lp.latency_records()
        ok = lat[:, 6] > 0
        us = (lat[ok, 2] - lat[ok, 6]) / 1e3
        to_fetch = (lat[ok, 3] - lat[ok, 6]) / 1e3
        vis = np.sort(lat[:, 2])
        rate = (len(vis) - 1) / ((vis[-1] - vis[0]) * 1e-9) if len(vis) > 1 and vis[-1] > vis[0] else None
        out[tag] = {"scored": int(o.get("events", 0) or 0), "skipped": int(o.get("skipped", 0) or 0),
                    "keys": int(o.get("keys", 0) or 0), "anomalies": int(o.get("anomalies", 0) or 0),
                    "results_msgs_per_s": rate,
                    "publish_to_result_p50_us": _pct(us, 50), "publish_to_result_p99_us": _pct(us, 99),
                    "publish_to_result_max_us": float(us.max()) if len(us) else None,
                    "publish_to_fetched_p50_us": _pct(to_fetch, 50),
                    "fetched_to_result_p50_us": _pct(us - to_fetch, 50)}
        out["timeline"][tag] = _windows(lat[ok, 6], us, float(window_s or interval_s), clients / interval_s)
    out["dropped"] = published - out["ae"]["scored"]
    return out
