"""``python -m streamml.cli <command> ...`` dispatcher.

Commands (reference script in parentheses):

  cardata-v3   <servers> <topic> <offset> <result_topic> <mode> <model-file> <project>
               (AUTOENCODER-TensorFlow-IO-Kafka/cardata-v3.py)
  cardata-v1   <servers> <topic> <offset> [result_topic]   (AUTOENCODER-.../cardata-v1.py)
  lstm-v2      <servers> <topic> <offset> <result_topic> <mode> <model-file>
               (LSTM-TensorFlow-IO-Kafka/cardata-v2.py)
  lstm-v1      <servers> <topic> <offset> [result_topic]   (LSTM-.../cardata-v1.py)
  creditcard   [servers] [--evaluate]     (autoencoder-anomaly-detection/*.py, notebooks)
  mnist        [servers] [--simplified]   (tensorflow-kafka-mnist*.py, confluent-tensorflow-io-kafka*.py)
  produce      <servers> <topic> [--source ...]   (test-data feeders)
  broker       [--port 9092] [--sasl user:pw] [--preload TOPIC=ROWS]
  train        [--config job.yaml] [--key=value ...] [--ckpt-dir D]   restartable (torchrun) training job
  ksql         <servers> <source_topic> <target_topic> [--window 300]   per-car tumbling event counts
  ksql-avro    <servers> [--source sensor-data] [--target SENSOR_DATA_S_AVRO]   KSQL JSON -> Avro (+ REKEY)
  mqtt-broker  [--port 1883] [--kafka SERVERS] [--kafka-extension kafka-config.yaml]   HiveMQ + Kafka extension
  devsim       run -s scenario.xml [--broker host:port] [--clients N]   HiveMQ device simulator
  connect      <servers> --config connector.json [--sink-store DIR]   Kafka Connect sinks (MongoDB, GCS Avro)
  serve        <servers> <topic> <result_topic> <model-file> [--replicas W --replica-index R]
               long-running shard-by-key anomaly scorer (one replica per GPU; model-predictions Deployment)
  fleet        <csv|synthetic> [--models N] [--epochs E]   one AE per car, all trained at once on one GPU
"""
from __future__ import annotations

import sys

from . import common


def _commands():
    from . import cardata_autoencoder as ae
    from . import cardata_lstm as ls
    from . import creditcard, fleet, mnist, mqtt, serve, tools, train
    return {
        "cardata-v3": ae.main_v3,
        "cardata-v1": ae.main_v1,
        "lstm-v2": ls.main_v2,
        "lstm-v1": ls.main_v1,
        "creditcard": creditcard.main,
        "mnist": mnist.main,
        "produce": tools.main_produce,
        "broker": tools.main_broker,
        "train": train.main,
        "ksql": tools.main_ksql,
        "ksql-avro": mqtt.main_ksql_avro,
        "mqtt-broker": mqtt.main_broker,
        "devsim": mqtt.main_devsim,
        "connect": mqtt.main_connect,
        "serve": serve.main,
        "fleet": fleet.main,
    }


def main(argv=None) -> int:
    argv = list(sys.argv[1:] if argv is None else argv)
    cmds = _commands()
    if not argv or argv[0] not in cmds:
        print(__doc__)
        return 1
    return common.run(cmds[argv[0]], argv[1:])


if __name__ == "__main__":
    sys.exit(main())
