"""KSQL-equivalent per-car 5-minute tumbling counts."""
import json

import numpy as np

from streamml.data import ksql
from streamml.data import produce as prod
from streamml.data import stream as st


def test_tumbling_counter_matches_bruteforce():
    rng = np.random.default_rng(0)
    keys = [f"car{int(k)}" for k in rng.integers(0, 7, 5000)]
    ts = np.sort(rng.integers(0, 3_600_000, 5000))
    tc = ksql.TumblingCounter(300_000)
    for s in range(0, 5000, 777):
        tc.update(keys[s:s + 777], ts[s:s + 777])
    ref = {}
    for k, t in zip(keys, ts):
        w = (t // 300_000) * 300_000
        ref[(k, int(w))] = ref.get((k, int(w)), 0) + 1
    closed = tc.closed()
    assert all(w + 300_000 <= tc.watermark for _, w, _ in closed)
    got = {(k, w): c for k, w, c in closed}
    got.update(tc.table())
    assert got == ref


def test_kafka_job_events_per_5min():
    srv = "fake://ksql-test"
    src = st.synthetic(3000, chunk=1000, scenario="evaluation")   # 25 cars, 1 msg / 5 s
    n = prod.produce(src, srv, "SENSOR_DATA_S_AVRO_REKEY", partitions=3)
    assert n == 3000
    out = ksql.run_events_per_window(srv, "SENSOR_DATA_S_AVRO_REKEY", "SENSOR_DATA_EVENTS_PER_5MIN_T", 300)
    from streamml.kafka import fake_broker
    b = fake_broker("ksql-test")
    recs = b.read("SENSOR_DATA_EVENTS_PER_5MIN_T", 0, 0, 1 << 20)
    assert len(recs) == out > 0
    vals = [json.loads(v) for _, _, v in recs]
    assert sum(v["EVENT_COUNT"] for v in vals) == 3000
    # 25 cars x 1 event / 5 s -> 60 events per car per full 5-minute window
    full = [v["EVENT_COUNT"] for v in vals]
    assert max(full) == 60
    assert {v["CAR"] for v in vals} == {f"electric-vehicle-{i:05d}" for i in range(25)}
    # offline form agrees
    table = ksql.events_per_window(st.synthetic(3000, chunk=1000, scenario="evaluation").map(
        lambda c: st.Chunk(c.x, c.label, [f"electric-vehicle-{int(d):05d}" for d in c.meta["device"]],
                           meta={"timestamp": np.asarray(c.meta["timestamp"]) * 1000})), 300)
    assert sorted(table.values()) == sorted(full)
