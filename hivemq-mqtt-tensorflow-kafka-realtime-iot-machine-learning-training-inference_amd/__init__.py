"""streamml — an MI355X-native streaming-ML engine for IoT sensor anomaly detection.

Capabilities mirror the HiveMQ -> Kafka -> TensorFlow-IO connected-car demo
(reference: uurl/hivemq-mqtt-tensorflow-kafka-realtime-iot-machine-learning-training-inference):
stream Confluent-framed Avro car-sensor events, normalise them, train / serve a
dense autoencoder and an LSTM predictor, write predictions and anomaly scores
back to a result topic, and persist Keras-compatible ``.h5`` checkpoints.

Compute path: PyTorch-ROCm tensors + hand-written HIP kernels for gfx950
(``streamml._C``); host I/O codecs (Avro, Kafka wire protocol, HDF5) are C++
(``streamml._io``); multi-GPU data parallelism uses RCCL via torch.distributed.
"""

__version__ = "0.1.0"

from . import config  # noqa: F401  (light, pure-python)
