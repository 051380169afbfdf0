"""Kafka ingestion / result sink over the native wire-protocol client (``streamml._io``).

Replaces the reference's tensorflow-io Kafka ops:

* ``KafkaDataset(["topic:partition:offset"], servers, group, eof, config_global)``
  (AUTOENCODER-TensorFlow-IO-Kafka/cardata-v3.py:44-47) -> :class:`KafkaDataset`
* ``KafkaOutputSequence(topic, servers, configuration).setitem(i, msg); flush()``
  (cardata-v3.py:238-252) -> :class:`KafkaOutputSequence`

``servers`` may be a real ``host:port[,host:port]`` list or ``fake://[name]``,
which resolves to an in-process broker (:class:`FakeBroker`) that speaks the
same protocol over 127.0.0.1 -- the test / synthetic-streaming backend.
"""
from .client import (FakeBroker, KafkaClient, KafkaError, fake_broker, parse_config,  # noqa: F401
                     parse_topic_spec, resolve_servers)
from .dataset import KafkaDataset  # noqa: F401
from .output import KafkaOutputSequence  # noqa: F401
