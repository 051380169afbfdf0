#!/usr/bin/env bash
# same-box A/B of batched AE scoring (bench_infer.py batched_events_per_s): tree _C.so vs tools/ab/_C_old.so
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"
P="$R/hivemq-mqtt-tensorflow-kafka-realtime-iot-machine-learning-training-inference_amd"
mkdir -p "$R/gpurun_out"
cp "$P/_C.so" /tmp/_C_new.so
cp "$R/tools/ab/_C_old.so" /tmp/_C_old.so
for v in new old new old; do
  cp "/tmp/_C_$v.so" "$P/_C.so"
  timeout -k 10 120 python "$R/bench/bench_infer.py" --events 300 > "$R/gpurun_out/absc_$v.json" 2>/dev/null || exit 1
  echo "$v $(python -c "import json;d=json.loads(open('$R/gpurun_out/absc_$v.json').read().strip().splitlines()[-1]);print(round(d['batched_events_per_s']/1e9,3))")"
done
cp /tmp/_C_new.so "$P/_C.so"
