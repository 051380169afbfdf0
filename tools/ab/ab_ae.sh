#!/usr/bin/env bash
# same-box A/B of the headline AE step: the tree's _C.so ("new") vs tools/ab/_C_old.so ("old"),
# headline-only bench.py runs alternated three times each
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"
P="$R/hivemq-mqtt-tensorflow-kafka-realtime-iot-machine-learning-training-inference_amd"
mkdir -p "$R/gpurun_out"
cp "$P/_C.so" /tmp/_C_new.so
cp "$R/tools/ab/_C_old.so" /tmp/_C_old.so
for v in new old new old new old; do
  cp "/tmp/_C_$v.so" "$P/_C.so"
  timeout -k 10 120 python "$R/bench.py" --infer-events 0 --fleet-models 0 --batch32-steps 0 --fit-rows 0 \
      --stream-rows 0 > "$R/gpurun_out/abae_$v.json" 2>/dev/null || exit 1
  echo "$v $(python -c "import json;d=json.loads(open('$R/gpurun_out/abae_$v.json').read().strip().splitlines()[-1]);print(round(d['value']/1e9,3), round(d['ms_per_step'],4), d['final_epoch_loss'])")"
done
cp /tmp/_C_new.so "$P/_C.so"
