"""Child-process entry points of a device-fleet run (``python -m streamml.mqtt.node ...``).

The reference runs its MQTT tier as separate pods: a 5-node HiveMQ cluster
(``infrastructure/hivemq/hivemq-crd.yaml:10``) fed by 6 device-simulator agents
(``infrastructure/test-generator/run_scenario.sh:13``, ``kube-cli.sh:347-428``).  A fleet
run (:mod:`streamml.mqtt.fleet`) starts the same shape as processes on one host -- every
process has its own descriptor limit, so 100 000 connected cars fit where one process's
limit would not.  Neither role imports torch or touches a GPU.

``broker --kafka HOST:PORT [--port 0]``
    one broker node with the Kafka bridge; prints ``{"port": P}`` once listening, runs until
    its stdin closes (or SIGTERM), then flushes the bridge and prints its counters as JSON.
``agent --host H --port P --clients N --messages M --interval S [--paced ...]``
    one simulator agent; prints the simulator's stats as JSON.
"""
from __future__ import annotations

import argparse
import json
import signal
import sys
import threading


def _broker(ns) -> int:
    from . import MqttBroker, raise_nofile_limit
    limit = raise_nofile_limit()
    b = MqttBroker(ns.port, kafka=ns.kafka, bridge_batch=ns.bridge_batch, bridge_linger_ms=ns.bridge_linger_ms,
                   metrics=False)
    print(json.dumps({"port": b.port, "nofile": limit}), flush=True)
    done = threading.Event()
    signal.signal(signal.SIGTERM, lambda *_: done.set())
    threading.Thread(target=lambda: (sys.stdin.read(), done.set()), daemon=True).start()
    done.wait()
    flushed = b.flush(30.0)
    st = dict(b.stats())
    st["flushed"] = bool(flushed)
    b.stop()
    print(json.dumps(st), flush=True)
    return 0


def _agent(ns) -> int:
    from . import Scenario, simulate
    sc = Scenario(clients=ns.clients, messages_per_client=ns.messages, interval_s=ns.interval, ramp_s=0.0,
                  qos=ns.qos, version=5)
    st = simulate(sc, ns.host, ns.port, threads=ns.threads, seed=ns.seed, failure_rate=ns.failure_rate,
                  id_offset=ns.id_offset, paced=ns.paced, start_at_unix=ns.start_at, stamp_ns=ns.stamp,
                  source_ips=[a for a in ns.source_ips.split(",") if a])
    print(json.dumps(st), flush=True)
    return 0


def main(argv=None) -> int:
    p = argparse.ArgumentParser(prog="streamml.mqtt.node")
    sub = p.add_subparsers(dest="role", required=True)
    b = sub.add_parser("broker")
    b.add_argument("--kafka", required=True)
    b.add_argument("--port", type=int, default=0)
    b.add_argument("--bridge-batch", type=int, default=1024)
    # 0: no linger -- each produce carries whatever queued during the previous one (the
    # batch grows with the load by itself; a linger only adds latency at 2 k msg/s a node)
    b.add_argument("--bridge-linger-ms", type=int, default=0)
    a = sub.add_parser("agent")
    a.add_argument("--host", default="127.0.0.1")
    a.add_argument("--port", type=int, required=True)
    a.add_argument("--clients", type=int, required=True)
    a.add_argument("--messages", type=int, default=1)
    a.add_argument("--interval", type=float, default=10.0)
    a.add_argument("--qos", type=int, default=0)
    a.add_argument("--threads", type=int, default=4)
    a.add_argument("--seed", type=int, default=0)
    a.add_argument("--failure-rate", type=float, default=0.01)
    a.add_argument("--id-offset", type=int, default=0)
    a.add_argument("--paced", action="store_true")
    a.add_argument("--start-at", type=float, default=0.0)
    a.add_argument("--stamp", action="store_true")
    a.add_argument("--source-ips", default="")
    ns = p.parse_args(argv)
    return _broker(ns) if ns.role == "broker" else _agent(ns)


if __name__ == "__main__":
    sys.exit(main())
