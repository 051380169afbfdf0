"""Kafka append -> result append, leg by leg, on this machine: the serve --low-latency loop
with (a) a host echo scorer (Kafka + C++ loop cost alone) and (b) the persistent GPU scorer
(bench/bench_infer.kafka_e2e).  20 000 events at 10 000 events/s each."""
import json
import os
import sys
import threading

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "bench"))

import itertools

import numpy as np

_RUNS = itertools.count()


def echo_run(events=20000, warm=200, qps=10000.0, spin=200, pin=True):
    from streamml.data.avro import AvroCodec
    from streamml.data.produce import encode_chunk
    from streamml.kafka import fake_broker
    from streamml.kafka.scoreloop import LowLatencyScorer, paced_produce
    from streamml.ops._ext import load_io
    name = f"legs-echo-{os.getpid()}-{spin}-{int(pin)}-{next(_RUNS)}"
    b = fake_broker(name)
    b.create_topic("S", 1)
    b.create_topic("R", 1)
    b.record_append_times(True)
    b.set_spin_us(spin)
    n = events + warm
    ev = np.random.default_rng(0).uniform(0, 40, (n, 18)).astype(np.float32)
    buf, offs = encode_chunk(AvroCodec("cardata-v1"), ev, np.zeros(n, np.uint8))
    echo = load_io().EchoScorer(18, 5.0)
    loop = LowLatencyScorer(f"fake://{name}", "S", "R", [0], echo, starts=[0], max_wait_ms=100, record_latency=True,
                            spin_us=spin)
    out = {}
    from bench_infer import _serving_cpus
    cpus = _serving_cpus(2) if pin else None

    def serve():
        if cpus:
            os.sched_setaffinity(0, {cpus[0]})
        out.update(loop.run(max_events=n, idle_timeout_s=10.0))

    th = threading.Thread(target=serve)
    th.start()
    mask = os.sched_getaffinity(0)
    if cpus:
        os.sched_setaffinity(0, {cpus[1]})
    try:
        paced_produce(f"fake://{name}", "S", 0, bytes(buf), offs, keys=[f"car{i % 1000}" for i in range(n)], qps=qps,
                      spin_us=spin)
    finally:
        os.sched_setaffinity(0, mask)
    th.join(120)
    b.set_spin_us(0)
    t_in, t_res = b.append_times("S", 0, 0, n)[warm:], b.append_times("R", 0, 0, n)[warm:]
    lat = loop.latency_records()
    lat = lat[np.argsort(lat[:, 1])][warm:]
    d = (t_res - t_in) / 1e3
    med = lambda a: float(np.median(a)) / 1e3   # noqa: E731
    return {"scorer": "echo (host)", "pinned_cpus": cpus, "p50_us": float(np.percentile(d, 50)), "p99_us": float(np.percentile(d, 99)),
            "legs_p50_us": {"append_to_fetched": med(lat[:, 3] - t_in), "fetched_to_scored": med(lat[:, 4] - lat[:, 3]),
                            "scored_to_formatted": med(lat[:, 5] - lat[:, 4]),
                            "formatted_to_result_append": med(t_res - lat[:, 5]),
                            "result_append_to_ack": med(lat[:, 2] - t_res)}}


def main():
    import torch
    from bench_infer import kafka_e2e
    from streamml.data.cardata import synthetic_device_tensor
    from streamml.models.autoencoder import Autoencoder
    print(json.dumps(echo_run(pin=False)), flush=True)
    print(json.dumps(echo_run()), flush=True)
    dev = torch.device("cuda", 0)
    m = Autoencoder(device=dev, input_normalizer="cardata")
    m.compile()
    ev = synthetic_device_tensor(21000, dev, seed=3).cpu().numpy()
    for pin in (False, True, False, True):
        r = kafka_e2e(m, ev, 10000.0, 5.0, 20000, pin=pin)
        r = {k: r[k] for k in ("p50_us", "p99_us", "legs_p50_us", "per_event_us", "pinned_cpus")}
        r["scorer"] = "persistent GPU (ae_serve.hip)"
        print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
