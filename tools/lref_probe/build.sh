#!/bin/bash
# Build the reference-LSTM probe binary (CPU container; runs on the GPU box).
# Extra device flags (e.g. -DSML_LREF_VARIANT=1) pass through as arguments.
set -e
cd "$(dirname "$0")/../.."
P=hivemq-mqtt-tensorflow-kafka-realtime-iot-machine-learning-training-inference_amd
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -DSML_LREF_PROBE "$@" -I$P/csrc/include \
  -munsafe-fp-atomics -mllvm -amdgpu-mfma-vgpr-form \
  $P/csrc/kernels/lstm_ref_train.hip tools/lref_probe/probe.cpp -o tools/lref_probe/lref_probe
