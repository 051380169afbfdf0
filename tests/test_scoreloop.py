"""Low-latency streaming scorer loop (csrc/io/scoreloop.cpp) + C++ result formatting
(csrc/io/format.cpp), on CPU: the GPU scorer is replaced by _io.EchoScorer (score =
mean(x^2), recon = x / 2) through the same SmlScorerApi table."""
import json
import os
import threading

import numpy as np
import pytest

from streamml.data import stream as S
from streamml.data.avro import AvroCodec
from streamml.data.produce import encode_chunk
from streamml.kafka import KafkaClient, fake_broker
from streamml.kafka.scoreloop import LowLatencyScorer, paced_produce
from streamml.ops._ext import load_io


def _records(n, seed=0):
    c = next(iter(S.synthetic(n, chunk=n, seed=seed, failure_rate=0.1)))
    buf, offs = encode_chunk(AvroCodec("cardata-v1"), c.x, c.label)
    offs = np.asarray(offs)
    return c.x.astype(np.float32), [bytes(buf[offs[i]:offs[i + 1]]) for i in range(n)], buf, offs


def _expected_score(x):
    s = np.float32(0)
    for v in x:
        s = np.float32(s + np.float32(v) * np.float32(v))
    return np.float32(s / np.float32(len(x)))


def test_array2string_and_json_match_python_exactly():
    io = load_io()
    rng = np.random.default_rng(0)
    for t in range(3000):
        a = (rng.standard_normal(rng.integers(1, 25)) * 10.0 ** rng.integers(-7, 10)).astype(np.float32)
        if t % 7 == 0:
            a[0] = 0
        if t % 11 == 0:
            a = np.round(a, 2).astype(np.float32)
        assert io.array2string_f32(a) == np.array2string(a)
    for a in (np.array([np.nan, -np.inf, 1.0], np.float32), np.zeros(18, np.float32), np.array([], np.float32)):
        assert io.array2string_f32(a) == np.array2string(a)
    for v in [0.0, -0.0, 1e16, 1e15, 1e-4, 1e-5, float("nan"), float("inf"), 0.1, 2.5e-7] + \
            list(rng.standard_normal(500) * 10.0 ** rng.integers(-30, 30, 500)):
        assert io.json_float(float(v)) == json.dumps(float(v))


def test_score_records_match_json_dumps():
    io = load_io()
    rng = np.random.default_rng(1)
    k = 50
    keys = [f"car-{i}" for i in range(k)]
    keys[3], keys[4], keys[5] = None, 'quo"te\\\n\x01', "ünï-\U0001F697"
    offs = np.arange(100, 100 + k, dtype=np.int64)
    scores = (rng.standard_normal(k) ** 2 * 3).astype(np.float32)
    flags = (scores > 5).astype(np.uint8)
    recon = rng.standard_normal((k, 18)).astype(np.float32)
    got = io.score_records(keys, 7, offs, scores, flags, recon)
    for i in range(k):
        ref = json.dumps({"car": keys[i], "partition": 7, "offset": int(offs[i]), "score": float(scores[i]),
                          "anomaly": bool(flags[i]), "reconstruction": np.array2string(recon[i])})
        assert got[i] == ref.encode()


def test_loop_scores_every_event_and_commits(tmp_path):
    name = "scoreloop-basic"
    b = fake_broker(name)
    b.create_topic("SENSOR", 2)
    b.create_topic("RESULTS", 2)
    x, vals, _, _ = _records(300)
    cli = KafkaClient(f"fake://{name}")
    keys = [f"car{i % 13}" for i in range(300)]
    cli.produce("SENSOR", 0, vals[:200], keys=[k.encode() for k in keys[:200]])
    cli.produce("SENSOR", 1, vals[200:] + [b"\x00garbage"], keys=[k.encode() for k in keys[200:]] + [None])
    echo = load_io().EchoScorer(18, 2.0)
    loop = LowLatencyScorer(f"fake://{name}", "SENSOR", "RESULTS", [0, 1], echo, group="g1", emit_recon=True,
                            max_batch=64, max_wait_ms=5)
    st = loop.run(idle_timeout_s=0.2)
    assert st["events"] == 300 and st["skipped"] == 1
    assert loop.positions() == [200, 101]
    assert cli.committed("g1", "SENSOR", 0) == 200 and cli.committed("g1", "SENSOR", 1) == 101
    res = b.read("RESULTS", 0, 0) + b.read("RESULTS", 1, 0)
    assert len(res) == 300
    seen = {}
    for r in res:
        d = json.loads(r[2])
        seen[(d["partition"], d["offset"])] = d
    for i in range(300):
        p, o = (0, i) if i < 200 else (1, i - 200)
        d = seen[(p, o)]
        assert d["car"] == keys[i]
        assert np.float32(d["score"]) == _expected_score(x[i])
        assert d["anomaly"] == bool(_expected_score(x[i]) > 2.0)
        assert d["reconstruction"] == np.array2string(x[i] * np.float32(0.5))
    assert st["anomalies"] == sum(1 for d in seen.values() if d["anomaly"])


def test_long_poll_delivers_paced_events_promptly():
    """Events appended at 2 000/s while the loop long-polls: each result is visible a
    few ms at most after its append (CPU box, loopback sockets)."""
    name = "scoreloop-latency"
    b = fake_broker(name)
    b.create_topic("SENSOR", 1)
    b.create_topic("RESULTS", 1)
    _, _, buf, offs = _records(400, seed=2)
    echo = load_io().EchoScorer(18, 5.0)
    loop = LowLatencyScorer(f"fake://{name}", "SENSOR", "RESULTS", [0], echo, starts=[0], max_wait_ms=50,
                            record_latency=True)
    out = {}
    th = threading.Thread(target=lambda: out.update(loop.run(max_events=400, idle_timeout_s=5.0)))
    th.start()
    sent = paced_produce(f"fake://{name}", "SENSOR", 0, bytes(buf), offs, qps=2000.0)
    th.join(30)
    assert not th.is_alive() and out["events"] == 400
    lat = loop.latency_records()
    assert lat.shape == (400, 7)
    d = (lat[np.argsort(lat[:, 1]), 2] - sent) / 1e3
    assert (d > 0).all()
    assert np.percentile(d, 50) < 5000, np.percentile(d, 50)   # us; ~100 us typical
    assert out["empty_fetches"] < 400   # long-poll, not a busy poll


def test_spin_mode_and_broker_append_times():
    """Low-latency socket policy (busy-poll before blocking, broker and client) keeps every
    result, in order; the broker's recorded append times give the append -> result latency."""
    n = 400
    x, vals, buf, offs = _records(n, seed=3)
    b = fake_broker("spin-unit")
    b.create_topic("S", 1)
    b.create_topic("R", 1)
    b.record_append_times(True)
    b.set_spin_us(100)
    pin = min(os.sched_getaffinity(0))
    b.set_thread_cpus([pin])   # connection threads start on this CPU only
    echo = load_io().EchoScorer(18, 5.0)
    loop = LowLatencyScorer("fake://spin-unit", "S", "R", [0], echo, starts=[0], max_wait_ms=50,
                            record_latency=True, spin_us=100)
    out = {}
    th = threading.Thread(target=lambda: out.update(loop.run(max_events=n, idle_timeout_s=5.0)))
    th.start()
    paced_produce("fake://spin-unit", "S", 0, bytes(buf), offs, qps=20000, spin_us=100)
    th.join(60)
    b.set_spin_us(0)
    if len(os.sched_getaffinity(0)) > 1:
        c = KafkaClient("fake://spin-unit")   # a live connection: its broker thread is pinned
        assert c.latest("R", 0) == n
        masks = []
        for t in os.listdir("/proc/self/task"):
            try:
                masks.append(os.sched_getaffinity(int(t)))
            except OSError:   # the thread ended
                pass
        assert {pin} in masks, masks
        del c
    assert out["events"] == n and b.end_offset("R", 0) == n
    t_in = b.append_times("S", 0, 0, n)
    t_res = b.append_times("R", 0, 0, n)
    assert (t_in > 0).all() and (t_res > 0).all()
    assert (np.diff(t_in) >= 0).all() and (t_res > t_in).all()
    assert (b.append_times("S", 0, n, 3) == -1).all()     # not appended yet
    recs = b.read("R", 0, 0, n)
    assert [json.loads(v)["offset"] for _, _, v in recs] == list(range(n))


# ---- JSON source records (jsonrow.h) and keyed scorers --------------------------------------
def _json_events(n, seed=0, stamp=False):
    """Device-simulator payloads (the bridge's sensor-data records) + the float32 rows."""
    from streamml.data.cardata import FEATURES
    from streamml.mqtt import car_payload
    vals, rows = [], []
    for i in range(n):
        v = car_payload(i % 17, i, 1000 + i, seed=seed)
        d = json.loads(v)
        if stamp:
            d["sent_ns"] = 123456789012 + i
            v = json.dumps(d).encode()
        vals.append(v)
        canon = {k.replace("_", "").lower(): x for k, x in d.items()}
        rows.append([np.float32(canon[f.replace("_", "")]) for f in FEATURES])
    return vals, np.asarray(rows, np.float32)


def test_json_rows_matches_json_loads():
    from streamml.kafka.scoreloop import json_columns
    io = load_io()
    vals, rows = _json_events(200, stamp=True)
    # other spellings of the same columns, nulls, strings, nesting, junk
    extra = [b'{"COOLANT_TEMP": "12.5", "tirePressure11": 31, "failure_occurred": "TRUE", "x": {"a": [1, {"b": 2}]}}',
             b'{"speed": null, "FAILURE_OCCURRED": false, "s": "esc\\"aped", "sent_ns": 7}',
             b'{}', b'not json', b'{"speed": 1,}', b'[1, 2]']
    allv = vals + extra
    offs = np.cumsum([0] + [len(v) for v in allv])
    x, lab, st, ok = io.json_rows(b"".join(allv), offs.tolist(), json_columns(), "failure_occurred", "sent_ns")
    assert ok.tolist() == [1] * 200 + [1, 1, 1, 0, 0, 0]
    np.testing.assert_array_equal(x[:200], rows)
    assert st[:200].tolist() == [123456789012 + i for i in range(200)]
    want_lab = [{"false": 0, "true": 1}[json.loads(v)["failure_occurred"]] for v in vals]
    assert lab[:200].tolist() == want_lab
    a = x[200]
    assert a[0] == np.float32(12.5) and a[9] == 31 and np.isnan(a[1]) and lab[200] == 1
    assert np.isnan(x[201, 6]) and lab[201] == 0 and st[201] == 7
    assert np.isnan(x[202]).all() and lab[202] == 2
    assert io.json_canonical("Tire_Pressure_1_1") == "tirepressure11"


def test_loop_follows_json_records_with_stamps():
    name = "scoreloop-json"
    b = fake_broker(name)
    b.create_topic("sensor-data", 2)
    b.create_topic("R", 2)
    vals, rows = _json_events(120, stamp=True)
    cli = KafkaClient(f"fake://{name}")
    cli.produce("sensor-data", 0, vals[:70], keys=[f"vehicles/sensor/data/car{i % 5}".encode() for i in range(70)])
    cli.produce("sensor-data", 1, vals[70:] + [b"{broken"], keys=None)
    echo = load_io().EchoScorer(18, 1e9)
    loop = LowLatencyScorer(f"fake://{name}", "sensor-data", "R", [0, 1], echo, starts=[0, 0], max_wait_ms=5,
                            record_latency=True, source_format="json", json_stamp="sent_ns")
    st = loop.run(idle_timeout_s=0.2)
    assert st["events"] == 120 and st["skipped"] == 1
    lat = loop.latency_records()
    got = {(int(p), int(o)): int(s) for p, o, s in zip(lat[:, 0], lat[:, 1], lat[:, 6])}
    assert got[(0, 5)] == 123456789012 + 5 and got[(1, 0)] == 123456789012 + 70
    res = [json.loads(r[2]) for r in b.read("R", 0, 0) + b.read("R", 1, 0)]
    by = {(d["partition"], d["offset"]): d for d in res}
    for i in range(120):
        p, o = (0, i) if i < 70 else (1, i - 70)
        assert np.float32(by[(p, o)]["score"]) == _expected_score(rows[i])


def test_keyed_scorer_maps_record_keys_to_stable_slots():
    """A keyed scorer (the LSTM forecaster's API): each distinct record key gets one slot,
    first come first served, stable across fetches and partitions; flag 2 (no previous
    forecast) is not an anomaly; more keys than slots is an error."""
    name = "scoreloop-keyed"
    b = fake_broker(name)
    b.create_topic("S", 2)
    b.create_topic("R", 1)
    _, vals, _, _ = _records(90, seed=4)
    cli = KafkaClient(f"fake://{name}")
    keys = [f"car{(i * 7) % 9}".encode() for i in range(90)]
    cli.produce("S", 0, vals[:50], keys=keys[:50])
    cli.produce("S", 1, vals[50:], keys=keys[50:])
    echo = load_io().EchoScorer(18, 5.0, nkeys=9)   # score = the key's slot
    loop = LowLatencyScorer(f"fake://{name}", "S", "R", [0, 1], echo, starts=[0, 0], result_partitions=[0, 0],
                            max_wait_ms=5, max_batch=16)
    st = loop.run(idle_timeout_s=0.2)
    assert st["events"] == 90 and st["keys"] == 9 and st["anomalies"] == 0
    res = [json.loads(r[2]) for r in b.read("R", 0, 0)]
    slot = {}
    for d in res:
        slot.setdefault(d["car"], set()).add(d["score"])
    assert all(len(v) == 1 for v in slot.values()) and len(slot) == 9
    assert sorted(s.pop() for s in slot.values()) == list(range(9))
    first = [d for d in res if d["partition"] == 0][:9]   # first sight of each key in partition 0
    assert [d["score"] for d in first] == list(range(9))
    # a tenth key does not fit, and a null key has no car: both skipped and counted, the
    # loop keeps running and commits past them (no abort, no shared "" slot)
    b.create_topic("S2", 1)
    cli.produce("S2", 0, vals[:12], keys=[f"k{i}".encode() for i in range(10)] + [None, b"k3"])
    loop2 = LowLatencyScorer(f"fake://{name}", "S2", "R", [0], load_io().EchoScorer(18, 5.0, nkeys=9), starts=[0],
                             max_wait_ms=5, group="g-keyed")
    st2 = loop2.run(idle_timeout_s=0.2)
    assert st2["events"] == 10 and st2["keys"] == 9 and st2["keys_dropped"] == 2, st2
    assert loop2.positions() == [12] and cli.committed("g-keyed", "S2", 0) == 12


def test_loop_key_shares_split_a_partition():
    """Two replicas sharing one partition through key-hash shares (kafka/assign.py "keys"):
    each car scored by exactly one replica, the other counts it as foreign."""
    from streamml.kafka.assign import HASH_SPACE, key_hash
    name = "scoreloop-shares"
    b = fake_broker(name)
    b.create_topic("S", 1)
    b.create_topic("R", 1)
    _, vals, _, _ = _records(400, seed=5)
    cli = KafkaClient(f"fake://{name}")
    keys = [f"electric-vehicle-{(i * 37) % 150:05d}".encode() for i in range(400)]
    cli.produce("S", 0, vals, keys=keys)
    cut = HASH_SPACE // 2
    got = []
    for lo, hi in ((0, cut), (cut, HASH_SPACE)):
        loop = LowLatencyScorer(f"fake://{name}", "S", "R", [0], load_io().EchoScorer(18, 5.0), starts=[0],
                                result_partitions=[0], max_wait_ms=5, hash_ranges=[(lo, hi)])
        st = loop.run(idle_timeout_s=0.2)
        mine = sum(1 for k in keys if lo <= key_hash(k) < hi)
        assert st["events"] == mine and st["foreign"] == 400 - mine, st
        got.append(st["events"])
    assert sum(got) == 400 and min(got) > 100
    cars = {}
    for r in b.read("R", 0, 0):
        d = json.loads(r[2])
        cars.setdefault(d["car"], []).append(d["offset"])
    assert sum(len(v) for v in cars.values()) == 400
    for offs in cars.values():
        assert offs == sorted(offs)


def test_key_shares_balance_eight_replicas_over_ten_partitions():
    """BASELINE config 5 topology (8 replicas, the reference's 10-partition topic,
    01_installConfluentPlatform.sh:180): with the producer's murmur2 partitioner and 100 000
    car keys, every key lands on exactly one replica and the max / min replica load is <= 1.1
    (round-robin whole partitions: 2.0)."""
    from streamml.cli.serve import serve_shares, shard_partitions
    from streamml.kafka.assign import key_hash
    from streamml.mqtt import kafka_partition
    P, W = 10, 8
    shares = [serve_shares(P, r, W) for r in range(W)]
    load = np.zeros(W, np.int64)
    rr = np.zeros(W, np.int64)
    for i in range(100_000):
        k = f"electric-vehicle-{i:05d}".encode()
        p, h = kafka_partition(k, P), key_hash(k)
        owners = [r for r in range(W) for q, lo, hi in shares[r] if q == p and lo <= h < hi]
        assert len(owners) == 1, (k, owners)
        load[owners[0]] += 1
        rr[p % W] += 1
    assert load.sum() == 100_000 and load.max() / load.min() <= 1.1, load
    assert rr.max() / rr.min() >= 1.8   # what round-robin partition ownership gives
    for r in range(W):   # each replica reads at most 3 partitions (~1.25 partitions of keys)
        assert 1 <= len(shares[r]) <= 3
    assert sorted(p for r in range(W) for p in shard_partitions(P, r, W)) == list(range(P))


def test_l3_cpus_picks_distinct_cores_of_one_l3():
    """utils.affinity: the placement of the e2e bench's spinning threads and ``serve --cpus auto``."""
    from streamml.utils.affinity import l3_cpus, parse_cpus, resolve_cpus
    allowed = os.sched_getaffinity(0)
    assert l3_cpus(len(allowed) + 1) is None
    assert resolve_cpus(None) is None and resolve_cpus("") is None
    assert resolve_cpus("0-2,5") == parse_cpus("0-2,5") == {0, 1, 2, 5}
    c = l3_cpus(1)
    if c is None:   # no cache topology in sysfs
        assert resolve_cpus("auto") is None
        return
    # two calls sample the load on their own, so under load the least-busy core may differ
    # between them: "auto" is one core of the SAME (slot-0) L3 domain
    auto = resolve_cpus("auto")
    l3_of = lambda x: open(f"/sys/devices/system/cpu/cpu{x}/cache/index3/shared_cpu_list").read()
    assert len(c) == 1 and c[0] in allowed and len(auto) == 1 and auto <= allowed
    assert l3_of(next(iter(auto))) == l3_of(c[0])
    for k in (2, 3):
        cs = l3_cpus(k)
        if cs is None:
            continue
        assert len(set(cs)) == k and set(cs) <= allowed
        l3 = {open(f"/sys/devices/system/cpu/cpu{x}/cache/index3/shared_cpu_list").read() for x in cs}
        cores = {open(f"/sys/devices/system/cpu/cpu{x}/topology/thread_siblings_list").read() for x in cs}
        assert len(l3) == 1 and len(cores) == k


def test_l3_cpus_slots_take_distinct_domains_whatever_the_load(monkeypatch):
    """Replicas started one after another each sample the CPU load on their own: the domain a
    slot gets must not depend on that sample, only the cores inside it."""
    import random
    from streamml.utils import affinity
    allowed = sorted(os.sched_getaffinity(0))
    doms = set()
    for c in allowed:
        try:
            doms.add(open(f"/sys/devices/system/cpu/cpu{c}/cache/index3/shared_cpu_list").read())
        except OSError:
            return   # no cache topology in sysfs
    rng = random.Random(0)
    monkeypatch.setattr(affinity, "cpu_busy", lambda sample_s=0.05: {c: rng.random() for c in allowed})
    got = []
    for slot in range(len(doms)):
        cs = affinity.l3_cpus(1, slot)
        got.append(open(f"/sys/devices/system/cpu/cpu{cs[0]}/cache/index3/shared_cpu_list").read())
    assert len(set(got)) == len(doms)
