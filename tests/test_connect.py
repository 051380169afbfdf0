"""Kafka Connect sink equivalents (streamml.connect): the MongoDB digital-twin sink and the
GCS Avro data-lake sink of infrastructure/kafka-connect/, driven by the same connector JSON."""
import io
import json
import os

import numpy as np
import pytest

from streamml.connect import (AvroLake, iter_lake_records, load_connector_config, read_avro_file, run_sink,
                              write_avro_file)
from streamml.kafka import fake_broker

MONGO_CM = "/root/reference/infrastructure/kafka-connect/mongodb/mongodb-connector-configmap.yaml"

GCS_CONFIG = json.dumps({
    "name": "sink-gcs",
    "config": {"connector.class": "io.confluent.connect.gcs.GcsSinkConnector", "tasks.max": "1",
               "topics": "SENSOR_DATA_S_AVRO", "gcs.bucket.name": "car-demo-sensor-data-avro", "flush.size": "3",
               "format.class": "io.confluent.connect.gcs.format.avro.AvroFormat"}})


def test_avro_container_roundtrip():
    bio = io.BytesIO()
    recs = [b"\x02abc", b"\x00", b"\x04\x01\x02"]
    write_avro_file(bio, '{"type":"record","name":"r","fields":[]}', recs)
    schema, blocks, n = read_avro_file(bio.getvalue())
    assert n == 3 and b"".join(blocks) == b"".join(recs) and json.loads(schema)["name"] == "r"
    bad = bytearray(bio.getvalue())
    bad[-1] ^= 0xFF
    with pytest.raises(ValueError):
        read_avro_file(bytes(bad))


def test_mongodb_sink_digital_twin(tmp_path):
    if not os.path.exists(MONGO_CM):
        pytest.skip("reference tree not mounted")
    cfg = load_connector_config(MONGO_CM)
    assert cfg["connector.class"].endswith("MongoSinkConnector") and cfg["topics"] == "sensor-data"
    kb = fake_broker("connect-mongo")
    kb.create_topic("sensor-data", 2)
    for i in range(20):   # two readings per car: the twin keeps the latest per key
        car = f"vehicles/sensor/data/electric-vehicle-{i % 10:05d}"
        kb.append("sensor-data", i % 2, [json.dumps({"speed": float(i), "seq": i}).encode()], [car.encode()])
    st = run_sink(cfg, "fake://connect-mongo", str(tmp_path))
    assert st["records"] == 20 and st["documents"] == 10
    path = tmp_path / "confluent-kafka-digital-twin" / "sensor-data.jsonl"
    docs = {d["_id"]: d for d in map(json.loads, path.read_text().splitlines())}
    assert docs["vehicles/sensor/data/electric-vehicle-00003"]["seq"] == 13
    # restart resumes from the committed offsets: nothing is re-applied
    assert run_sink(cfg, "fake://connect-mongo", str(tmp_path))["records"] == 0


def test_gcs_avro_lake_sink(tmp_path):
    from streamml.data import produce as prod
    from streamml.data import stream as st
    kb = fake_broker("connect-gcs")
    kb.create_topic("SENSOR_DATA_S_AVRO", 1)
    n = prod.produce(st.synthetic(10, chunk=10), "fake://connect-gcs", "SENSOR_DATA_S_AVRO", create=False)
    cfg = load_connector_config(GCS_CONFIG)
    out = run_sink(cfg, "fake://connect-gcs", str(tmp_path))
    assert out["records"] == n == 10 and out["files"] == 4                    # flush.size 3 -> 3+3+3+1
    root = tmp_path / "car-demo-sensor-data-avro" / "topics" / "SENSOR_DATA_S_AVRO" / "partition=0"
    assert sorted(os.listdir(root)) == [f"SENSOR_DATA_S_AVRO+0+{o:010d}.avro" for o in (0, 3, 6, 9)]
    rows = np.concatenate([b["numeric"] for _, b in iter_lake_records(str(tmp_path))])
    assert rows.shape[0] == 10 and np.isfinite(rows).all()
