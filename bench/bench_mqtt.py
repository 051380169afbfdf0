#!/usr/bin/env python3
"""The reference's scale axis end to end: an MQTT device fleet -> broker nodes + Kafka bridge ->
Kafka -> persistent GPU scorer(s) -> result topic (streamml.mqtt.fleet.run_fleet).

Default = the reference's full scenario rate (infrastructure/test-generator/scenario.xml:13,
48-49): 100 000 cars, one car payload per car every 10 s (10 000 msg/s), here for
``--messages`` rounds, over 5 broker nodes (hivemq-crd.yaml:10) and 6 simulator agents
(run_scenario.sh:13).  Prints one JSON line: connections, connect time, offered / achieved
msg/s, per-hop counts, drops, publish -> result latency p50/p99 (us) for the autoencoder
scorer and (``--lstm``) the per-car LSTM forecaster on the same events.

``--device cpu`` swaps the GPU scorers for the C++ echo scorer (pipeline check without a GPU).
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


SCENARIOS = {   # infrastructure/test-generator/scenario*.xml
    "full": {"clients": 100_000, "interval_s": 10.0, "messages": 3000, "qos": 0},       # scenario.xml:13, 48-49
    "evaluation": {"clients": 25, "interval_s": 5.0, "messages": 40, "qos": 1},         # scenario_evaluation.xml:13, 47-48
}


def measure(device="cuda", clients=100_000, interval_s=10.0, messages=3, brokers=None, agents=None, partitions=10,
            threads=4, lstm=True, name="bench-fleet", sources_per_agent=1, qos=0, window_s=None):
    """One fleet run; scorers built here (the AE at random init, the reference LSTM stack at
    look_back 1 -- cardata-v2.py:172-183 -- with one device slot per car)."""
    from streamml.mqtt.fleet import run_fleet
    from streamml.ops._ext import load_io
    if str(device) == "cpu":
        sc = load_io().EchoScorer(18, 5.0)
        lsc = load_io().EchoScorer(18, 5.0, nkeys=clients) if lstm else None
        return run_fleet(sc, clients, interval_s, messages, brokers, agents, partitions, threads, lstm_scorer=lsc,
                         name=name, sources_per_agent=sources_per_agent, qos=qos, window_s=window_s)
    import torch

    from streamml.models.autoencoder import Autoencoder
    from streamml.models.lstm import LSTMPredictor
    from streamml.ops.serve import LSTMScoringServer, ScoringServer
    dev = torch.device(device)
    ae = Autoencoder(device=dev, input_normalizer="cardata", seed=0)
    ae.compile()
    with ScoringServer(ae, threshold=5.0) as srv:
        if not lstm:
            r = run_fleet(srv, clients, interval_s, messages, brokers, agents, partitions, threads, name=name,
                          sources_per_agent=sources_per_agent, qos=qos, window_s=window_s)
        else:
            lm = LSTMPredictor.reference(look_back=1, device=dev)
            with LSTMScoringServer(lm, nkeys=clients, threshold=5.0) as lsrv:
                r = run_fleet(srv, clients, interval_s, messages, brokers, agents, partitions, threads,
                              lstm_scorer=lsrv, name=name, sources_per_agent=sources_per_agent, qos=qos,
                              window_s=window_s)
    r["scorers"] = ["autoencoder (ae_serve.hip)"] + (["LSTM reference stack, look_back 1 (lstm_serve.hip)"] if lstm
                                                     else [])
    return r


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--device", default="cuda:0")
    ap.add_argument("--clients", type=int, default=100_000)
    ap.add_argument("--interval", type=float, default=10.0)
    ap.add_argument("--messages", type=int, default=3)
    ap.add_argument("--brokers", type=int, default=None, help="default: as many as the descriptor limit needs")
    ap.add_argument("--agents", type=int, default=None)
    ap.add_argument("--partitions", type=int, default=10)
    ap.add_argument("--threads", type=int, default=4)
    ap.add_argument("--sources-per-agent", type=int, default=1)
    ap.add_argument("--no-lstm", action="store_true")
    ap.add_argument("--qos", type=int, default=0)
    ap.add_argument("--scenario", choices=sorted(SCENARIOS), default=None,
                    help="the reference scenario's clients / interval / messages / QoS (--messages still caps the "
                         "rounds if given)")
    ap.add_argument("--window", type=float, default=None, help="timeline window (s); default the send interval")
    ap.add_argument("--out", default=None, help="also write the JSON here")
    a = ap.parse_args()
    clients, interval, messages, qos = a.clients, a.interval, a.messages, a.qos
    if a.scenario:
        sc = SCENARIOS[a.scenario]
        clients, interval, qos = sc["clients"], sc["interval_s"], sc["qos"]
        messages = min(a.messages, sc["messages"]) if "--messages" in sys.argv else sc["messages"]
    r = measure(a.device, clients, interval, messages, a.brokers, a.agents, a.partitions, a.threads, not a.no_lstm,
                sources_per_agent=a.sources_per_agent, qos=qos, window_s=a.window)
    r["scenario"] = a.scenario
    r["qos"] = qos
    ae = r.get("timeline", {}).get("ae", [])
    r["soak_summary"] = {
        "windows": len(ae), "scored": r["ae"]["scored"], "published": r["published"], "dropped": r["dropped"],
        "p99_us_per_window": [w["p99_us"] for w in ae], "max_us": r["ae"]["publish_to_result_max_us"],
        "broker_rss_mb": r["broker_rss_mb"], "short_windows": sum(1 for w in ae[:-1] if w["scored"] < w["offered"]),
        "kafka_log": r.get("kafka_log"), "scorer_rss_mb": r.get("scorer_rss_mb")}
    line = json.dumps(r)
    if a.out:
        with open(a.out, "w") as f:
            f.write(line + "\n")
    print(line, flush=True)


if __name__ == "__main__":
    main()
