"""bench/broker_proc.py: the bench's Kafka broker in a child process."""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "bench"))


def test_broker_process_serves_the_topic_and_exits_on_close():
    import bench_fit
    from streamml.kafka.client import KafkaClient
    mine, theirs = bench_fit._split_cpus()
    assert mine and (theirs is None or not (mine & theirs))
    proc, info = bench_fit._broker_process(20_000, 4, theirs)
    try:
        assert info["pid"] == proc.pid and info["log_bytes"] > 20_000 * 100
        c = KafkaClient(info["addr"])
        assert sum(c.latest("SENSOR_DATA_S_AVRO", p) for p in range(4)) == 20_000
        if theirs:
            assert set(info["cpus"]) <= theirs
    finally:
        proc.stdin.close()
        assert proc.wait(timeout=30) == 0
