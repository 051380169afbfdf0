"""The bench's Kafka broker as a separate process: the reference's brokers are
remote pods, so the consumer's fetch + decode cost is measured with the broker's socket threads
outside the consumer's process, on CPUs of their own.

    python bench/broker_proc.py --rows N --partitions P [--topic T]

Fills the topic with the same Confluent-Avro events as ``bench_fit._fill_topic`` (no GPU is ever
touched here), prints ONE JSON line ``{"addr", "log_bytes", "produce_s", "cpus"}`` and serves until
its stdin closes (the parent ends it by closing the pipe)."""
import argparse
import json
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, HERE)


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, required=True)
    ap.add_argument("--partitions", type=int, default=32)
    ap.add_argument("--topic", default="SENSOR_DATA_S_AVRO")
    a = ap.parse_args()
    from bench_fit import _fill_topic   # noqa: E402 - after the path fix
    from streamml.kafka.client import FakeBroker
    b = FakeBroker()
    t0 = time.perf_counter()
    nbytes = _fill_topic(b, a.topic, a.rows, a.partitions)
    print(json.dumps({"addr": b.address, "log_bytes": int(nbytes), "produce_s": time.perf_counter() - t0,
                      "cpus": sorted(os.sched_getaffinity(0)), "pid": os.getpid()}), flush=True)
    try:
        sys.stdin.read()          # until the parent closes the pipe
    finally:
        b.stop()
    return 0


if __name__ == "__main__":
    sys.exit(main())
