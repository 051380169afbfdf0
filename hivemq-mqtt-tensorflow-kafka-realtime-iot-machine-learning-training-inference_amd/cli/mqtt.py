"""MQTT front ends: the broker + Kafka bridge, the device simulator, the KSQL Avro job.

``mqtt-broker [--port 1883] [--kafka SERVERS] [--kafka-extension kafka-config.yaml] ...``
    The HiveMQ cluster + Kafka extension (infrastructure/hivemq/setup.sh,
    hivemq-crd.yaml, kafka-config.yaml).  ``--kafka-extension`` reads the
    reference's own ConfigMap / XML for the topic mappings; ``--kafka`` overrides
    its bootstrap servers (``fake://name`` = an in-process Kafka broker started here).

``devsim run -s scenario.xml [--broker host:port] [--clients N] [--messages M] ...``
    ``kubectl devsim run -s scenario.xml`` (infrastructure/test-generator/kube-cli.sh,
    scenario.xml / scenario_evaluation.xml): connects every simulated car and
    publishes its sensor payloads; the scaling flags shrink the 100 000-car
    scenario for a single host.

``ksql-avro <servers> [--source sensor-data] [--target SENSOR_DATA_S_AVRO] [--rekey ...]``
    KSQL's JSON -> Avro -> PARTITION BY CAR streams (01_installConfluentPlatform.sh:235-249).

``connect <servers> --config connector.json [--sink-store DIR|gs://bucket] [--follow]``
    The Kafka Connect sinks (infrastructure/kafka-connect/): MongoSinkConnector ->
    digital-twin document store, GcsSinkConnector -> Avro data lake.
"""
from __future__ import annotations

import argparse
import json
import signal
import sys
import threading
import time
from typing import Sequence

from . import common


def main_broker(argv: Sequence[str]) -> int:
    p = argparse.ArgumentParser(prog="mqtt-broker")
    p.add_argument("--port", type=int, default=1883)
    p.add_argument("--user", default="")
    p.add_argument("--password", default="")
    p.add_argument("--max-qos", type=int, default=2)
    p.add_argument("--kafka", default=None, help="Kafka bootstrap list or fake://name (default: from the extension "
                                                   "config, else no bridge)")
    p.add_argument("--kafka-extension", default=None, help="HiveMQ kafka-configuration XML or its ConfigMap YAML")
    p.add_argument("--mapping", action="append", default=[], help="FILTER=KAFKA_TOPIC (repeatable)")
    p.add_argument("--kafka-config", default="auto")
    p.add_argument("--partitions", type=int, default=10, help="partitions of auto-created fake:// topics "
                                                                "(the reference creates sensor-data with 10)")
    p.add_argument("--duration", type=float, default=None)
    p.add_argument("--metrics-port", type=int, default=0, help="serve Prometheus /metrics on this port (0 = off)")
    ns = p.parse_args(list(argv))
    from ..kafka import fake_broker
    from ..mqtt import MqttBroker, TopicMapping, load_topic_mappings

    maps, cluster = [], {}
    if ns.kafka_extension:
        maps, cluster = load_topic_mappings(ns.kafka_extension)
    for spec in ns.mapping:
        flt, _, topic = spec.partition("=")
        maps.append(TopicMapping(topic, [flt], topic))
    kafka = ns.kafka or cluster.get("bootstrap")
    cfg = None
    if kafka:
        cfg = common.kafka_config(kafka, ns.kafka_config)
        if cluster.get("username") and ns.kafka_config == "auto" and not kafka.startswith("fake://"):
            cfg = ["security.protocol=sasl_plaintext", "sasl.mechanisms=PLAIN",
                   f"sasl.username={cluster['username']}", f"sasl.password={cluster.get('password', '')}"]
        if kafka.startswith("fake://"):
            kb = fake_broker(kafka[len("fake://"):] or "default")
            for m in maps or [TopicMapping("sensor-data", ["vehicles/sensor/data/#"], "sensor-data")]:
                kb.create_topic(m.kafka_topic, ns.partitions)
            print(f"in-process Kafka broker listening 127.0.0.1:{kb.port}", flush=True)
    b = MqttBroker(ns.port, kafka=kafka, mappings=maps or None, username=ns.user, password=ns.password,
                   max_qos=ns.max_qos, kafka_config=cfg)
    print(f"MQTT broker listening {b.port} (bridge: {kafka or 'off'}; mappings: "
          f"{[(m.filters, m.kafka_topic) for m in b.mappings]})", flush=True)
    if ns.metrics_port:
        from ..obs.metrics import REGISTRY
        REGISTRY.serve(ns.metrics_port, addr="0.0.0.0")
    stop = threading.Event()
    for sig in (signal.SIGINT, signal.SIGTERM):
        signal.signal(sig, lambda *_: stop.set())
    t_end = None if ns.duration is None else time.monotonic() + ns.duration
    last = 0.0
    while not stop.is_set() and (t_end is None or time.monotonic() < t_end):
        stop.wait(0.2)
        if time.monotonic() - last > 10:
            last = time.monotonic()
            print(json.dumps(b.stats()), flush=True)
    b.flush(10.0)
    print(json.dumps(b.stats()), flush=True)
    b.stop()
    return 0


def main_devsim(argv: Sequence[str]) -> int:
    argv = list(argv)
    if argv and argv[0] == "run":
        argv = argv[1:]
    p = argparse.ArgumentParser(prog="devsim run")
    p.add_argument("-s", "--scenario", required=True)
    p.add_argument("--broker", default=None, help="host:port (default: the scenario's broker)")
    p.add_argument("--clients", type=int, default=None)
    p.add_argument("--messages", type=int, default=None)
    p.add_argument("--interval", type=float, default=None, help="seconds between a car's messages")
    p.add_argument("--ramp", type=float, default=None)
    p.add_argument("--threads", type=int, default=8)
    p.add_argument("--agents", type=int, default=1, help="split the fleet over this many simulator processes")
    p.add_argument("--agent-index", type=int, default=0, help="which share of the fleet this process runs")
    p.add_argument("--seed", type=int, default=0)
    p.add_argument("--failure-rate", type=float, default=0.01)
    p.add_argument("--user", default="")
    p.add_argument("--password", default="")
    ns = p.parse_args(argv)
    from ..mqtt import Scenario, simulate

    sc = Scenario.from_xml(ns.scenario).scaled(ns.clients, ns.messages, ns.interval, ns.ramp)
    host, port = sc.broker
    if ns.broker:
        host, _, ps = ns.broker.rpartition(":")
        port = int(ps)
    print(f"scenario: {sc.clients} cars x {sc.messages_per_client} msgs @ 1/{sc.interval_s:g}s QoS {sc.qos} "
          f"MQTT {'5' if sc.version == 5 else '3.1.1'} -> {host}:{port}", flush=True)
    if not 0 <= ns.agent_index < ns.agents:
        raise SystemExit("--agent-index must be in [0, --agents)")
    lo = sc.clients * ns.agent_index // ns.agents
    hi = sc.clients * (ns.agent_index + 1) // ns.agents
    st = simulate(sc.scaled(clients=hi - lo), host, port, threads=ns.threads, seed=ns.seed,
                  failure_rate=ns.failure_rate, username=ns.user, password=ns.password, id_offset=lo)
    st["msgs_per_s"] = st["published"] / max(st["elapsed_s"], 1e-9)
    print(json.dumps(st), flush=True)
    return 0 if st["connect_failed"] == 0 and st["publish_failed"] == 0 else 2


def main_ksql_avro(argv: Sequence[str]) -> int:
    common.print_options(argv)
    usage = "Usage: ksql-avro <servers> [--source sensor-data] [--target SENSOR_DATA_S_AVRO] [--rekey TOPIC|'']"

    def flags(p):
        p.add_argument("--source", default="sensor-data")
        p.add_argument("--target", default="SENSOR_DATA_S_AVRO")
        p.add_argument("--rekey", default="SENSOR_DATA_S_AVRO_REKEY")
        p.add_argument("--follow", action="store_true", help="keep consuming (no eof)")
        p.add_argument("--idle-timeout", type=float, default=None)

    ns = common.parse(argv, usage, ["servers"], add_flags=flags)
    from ..data.ksql import run_json_to_avro
    cfg = common.kafka_config(ns.servers, ns.kafka_config)
    st = run_json_to_avro(ns.servers, ns.source, ns.target, ns.rekey or None, config=cfg, eof=not ns.follow,
                          idle_timeout_s=ns.idle_timeout)
    print(json.dumps(st), flush=True)
    return 0


def main_connect(argv: Sequence[str]) -> int:
    common.print_options(argv)
    usage = "Usage: connect <servers> --config connector.json [--sink-store DIR|gs://bucket] [--follow]"

    def flags(p):
        p.add_argument("--config", required=True, help="connector JSON or the ConfigMap that carries it")
        p.add_argument("--sink-store", default="./connect-sink", help="local root or gs://bucket")
        p.add_argument("--schema", default="ksql-cardata-v1")
        p.add_argument("--follow", action="store_true")
        p.add_argument("--idle-timeout", type=float, default=None)

    ns = common.parse(argv, usage, ["servers"], add_flags=flags)
    from ..connect import load_connector_config, run_sink
    cfg = common.kafka_config(ns.servers, ns.kafka_config)
    st = run_sink(load_connector_config(ns.config), ns.servers, ns.sink_store, eof=not ns.follow, kafka_config=cfg,
                  schema=ns.schema, idle_timeout_s=ns.idle_timeout)
    print(json.dumps(st), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(common.run(main_broker))
