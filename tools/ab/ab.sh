#!/usr/bin/env bash
# same-box A/B: the tree's _C.so ("new") vs tools/ab/_C_old.so ("old") on bench_lstm
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"
P="$R/hivemq-mqtt-tensorflow-kafka-realtime-iot-machine-learning-training-inference_amd"
cp "$P/_C.so" /tmp/_C_new.so
for v in new old new old; do
  cp "/tmp/_C_$v.so" "$P/_C.so" 2>/dev/null || cp "$R/tools/ab/_C_old.so" "$P/_C.so"
  timeout -k 10 120 python "$R/bench/bench_lstm.py" > "$R/gpurun_out/ab_$v.json" 2>/dev/null || exit 1
  echo "$v $(python -c "import json;d=json.loads(open('$R/gpurun_out/ab_$v.json').read().strip().splitlines()[-1]);print(round(d['value']/1e6,2), round(d['ms_per_step'],4))")"
done
cp /tmp/_C_new.so "$P/_C.so"
