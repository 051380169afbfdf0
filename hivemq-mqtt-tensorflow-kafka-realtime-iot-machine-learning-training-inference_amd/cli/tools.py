"""Operational front ends: a standalone broker and the test-data producer.

``broker [--port 9092] [--sasl test:test123] [--preload TOPIC=ROWS ...]``
    Runs the native in-process Kafka-protocol broker as its own process so
    separate producer / train / predict processes can talk to it over TCP
    exactly as they would to the reference's Confluent cluster (which used
    SASL PLAIN ``test/test123``, cardata-v3.py:7-15).  ``--preload`` fills a
    topic with synthetic car events (KSQL Avro, Confluent-framed).

``produce <servers> <topic> [--source synthetic:N | csv:PATH | jsonl:PATH]``
    The reference's feeders: the HiveMQ simulator -> MQTT -> Kafka -> KSQL Avro
    chain (scenario.xml, 01_installConfluentPlatform.sh:242-249), the
    ``kafka-avro-console-producer`` of JSON lines (LSTM-.../cardata-v1.sh:6) and
    the CSV producer (testdata/Test-Load-csv).  Records are Confluent-framed Avro
    keyed by car id; ``--partitions P`` spreads keys over P partitions.
"""
from __future__ import annotations

import argparse
import signal
import sys
import threading
import time
from typing import Sequence

from . import common


def main_broker(argv: Sequence[str]) -> int:
    p = argparse.ArgumentParser(prog="broker")
    p.add_argument("--port", type=int, default=9092)
    p.add_argument("--sasl", default="", help="user:password enables SASL PLAIN")
    p.add_argument("--preload", action="append", default=[], help="TOPIC=ROWS synthetic car events")
    p.add_argument("--schema", default="cardata-v1")
    p.add_argument("--duration", type=float, default=None, help="exit after this many seconds")
    p.add_argument("--retention", type=int, default=-1, help="records kept per partition (-1 = all)")
    ns = p.parse_args(list(argv))
    from ..data import produce as prod
    from ..data import stream as st
    from ..kafka import FakeBroker, client as kclient

    user, _, pw = ns.sasl.partition(":")
    b = FakeBroker(ns.port, user, pw, ns.retention)
    # register so in-process producers can reach it as fake://broker without SASL plumbing
    with kclient._FAKES_LOCK:
        kclient._FAKES["broker"] = b
    for spec in ns.preload:
        topic, _, rows = spec.partition("=")
        b.create_topic(topic, 1)
        n = prod.produce(st.synthetic(int(rows or common.SYNTHETIC_DEFAULT_ROWS), chunk=8192), "fake://broker",
                         topic, schema=ns.schema, create=False,
                         config=[f"security.protocol=sasl_plaintext", f"sasl.username={user}",
                                 f"sasl.password={pw}", "sasl.mechanisms=PLAIN"] if user else None)
        print(f"preloaded {n} events into {topic}", flush=True)
    print(f"listening {b.address}", flush=True)
    stop = threading.Event()
    for sig in (signal.SIGINT, signal.SIGTERM):
        signal.signal(sig, lambda *_: stop.set())
    t_end = None if ns.duration is None else time.monotonic() + ns.duration
    while not stop.is_set() and (t_end is None or time.monotonic() < t_end):
        stop.wait(0.2)
    b.stop()
    return 0


def main_produce(argv: Sequence[str]) -> int:
    common.print_options(argv)
    usage = "Usage: produce <servers> <topic> [--source synthetic:N|csv:PATH|jsonl:PATH]"

    def flags(p):
        p.add_argument("--source", default="synthetic:20000")
        p.add_argument("--schema", default="cardata-v1")
        p.add_argument("--partitions", type=int, default=None)
        p.add_argument("--scenario", default="full")
        p.add_argument("--failure-rate", type=float, default=0.01)

    ns = common.parse(argv, usage, ["servers", "topic"], add_flags=flags)
    from ..data import produce as prod
    from ..data import stream as st

    kind, _, arg = ns.source.partition(":")
    if kind == "synthetic":
        src = st.synthetic(int(arg or common.SYNTHETIC_DEFAULT_ROWS), chunk=4096, seed=ns.synthetic_seed,
                           scenario=ns.scenario, failure_rate=ns.failure_rate)
    elif kind == "csv":
        src = st.csv(arg)
    elif kind == "jsonl":
        src = st.json_lines(arg)
    else:
        print(usage)
        return 1
    cfg = common.kafka_config(ns.servers, ns.kafka_config)
    t0 = time.perf_counter()
    n = prod.produce(src, ns.servers, ns.topic, schema=ns.schema, partitions=ns.partitions, config=cfg)
    dt = time.perf_counter() - t0
    print(f"{n} records produced into '{ns.topic}' ({n / max(dt, 1e-9):.0f} records/s)", flush=True)
    return 0



def main_ksql(argv: Sequence[str]) -> int:
    """``ksql <servers> <source_topic> <target_topic> [--window 300]``: the reference's
    SENSOR_DATA_EVENTS_PER_5MIN_T table (01_installConfluentPlatform.sh:256) as a job."""
    common.print_options(argv)
    usage = "Usage: ksql <servers> <source_topic> <target_topic> [--window SECONDS]"

    def flags(p):
        p.add_argument("--window", type=int, default=300)
        p.add_argument("--grace", type=int, default=None)
        p.add_argument("--follow", action="store_true", help="keep consuming (persistent query) instead of "
                                                              "stopping at the partition end")

    ns = common.parse(argv, usage, ["servers", "source", "target"], add_flags=flags)
    from ..data.ksql import run_events_per_window
    cfg = common.kafka_config(ns.servers, ns.kafka_config)
    n = run_events_per_window(ns.servers, ns.source, ns.target, ns.window, config=cfg, grace_s=ns.grace,
                              eof=not ns.follow)
    print(f"{n} window counts produced into '{ns.target}'", flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(common.run(main_produce))
