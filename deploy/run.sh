#!/usr/bin/env bash
# Build the MI355X image and start the pipeline (counterpart of the reference's
# python-scripts/AUTOENCODER-TensorFlow-IO-Kafka/run.sh and infrastructure/*/setup.sh).
set -euo pipefail
IMAGE=${IMAGE:-streamml/mi355x:latest}
HERE=$(cd "$(dirname "$0")" && pwd)
docker build -t "$IMAGE" -f "$HERE/Dockerfile" "$HERE/.."
docker push "$IMAGE" || true
kubectl create configmap devsim-scenario --from-file=scenario.xml="${SCENARIO:-$HERE/scenarios/car-fleet-evaluation.xml}" \
  --dry-run=client -o yaml | kubectl apply -f -
kubectl apply -f "$HERE/k8s/mqtt-broker.yaml"
kubectl apply -f "$HERE/k8s/stream-jobs.yaml"
kubectl apply -f "$HERE/k8s/devsim-job.yaml"
kubectl apply -f "$HERE/k8s/model-training.yaml"
kubectl wait --for=condition=complete --timeout=30m job/sensor-model-training
kubectl apply -f "$HERE/k8s/model-predictions.yaml"
