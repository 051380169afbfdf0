"""Device fleet end to end (streamml.mqtt.fleet) at CPU-test scale: simulator agent
processes -> broker-node processes -> Kafka bridge -> in-process Kafka -> the C++ scoring
loop on JSON events (EchoScorer standing in for the GPU scorer) -> result topic.  Every
published event must come out scored exactly once, with an exact publish -> result latency
(reference scale axis: infrastructure/test-generator/scenario.xml:13, 48-49)."""
import json

import numpy as np

from streamml.kafka import KafkaClient
from streamml.mqtt.fleet import run_fleet
from streamml.ops._ext import load_io


def test_fleet_small_scale_no_drops():
    echo = load_io().EchoScorer(18, 1e9)
    lecho = load_io().EchoScorer(18, 1e9, nkeys=400)    # keyed (the LSTM forecaster's API)
    r = run_fleet(echo, clients=300, interval_s=0.5, messages=4, brokers=2, agents=3, partitions=4,
                  threads=2, lstm_scorer=lecho, name="fleet-cpu-test", start_delay_s=4.0)
    assert r["connections"] == 300 and r["connect_failed"] == 0, r
    assert r["published"] == 1200 and r["publish_failed"] == 0
    assert r["broker_incoming"] == 1200 and r["bridged_to_kafka"] == 1200 and r["bridge_failed"] == 0
    assert r["dropped"] == 0 and r["ae"]["scored"] == 1200 and r["ae"]["skipped"] == 0
    assert r["lstm"]["scored"] == 1200 and r["lstm"]["keys"] == 300    # one slot per car
    assert 0 < r["ae"]["publish_to_result_p50_us"] < 2e6
    c = KafkaClient(r["kafka"])
    n = 0
    cars = set()
    for p in range(4):
        b = c.fetch("model-predictions", p, 0, 1 << 24, 10)
        vals, vo = b["values"], b["value_offsets"]
        for i in range(len(vo) - 1):
            d = json.loads(vals[vo[i]:vo[i + 1]])
            cars.add(d["car"])
            assert np.isfinite(d["score"])
        n += len(vo) - 1
    assert n == 1200 and len(cars) == 300
    assert all(k.startswith("vehicles/sensor/data/electric-vehicle-") for k in cars)
