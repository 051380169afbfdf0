set -u
mkdir -p gpurun_out/fleet
( while sleep 30; do echo "tick $(date +%T)"; done ) &
HB=$!
timeout -k 10 420 python bench/bench_mqtt.py --messages 12 --interval 10 --out gpurun_out/fleet/gpu_100k_12msg.json > gpurun_out/fleet/gpu_100k.log 2>&1
rc=$?
echo "fleet rc=$rc"
if [ $rc -eq 0 ]; then
  timeout -k 10 300 python bench/bench_mqtt.py --scenario evaluation --out gpurun_out/fleet/gpu_evaluation_qos1.json > gpurun_out/fleet/gpu_eval.log 2>&1
  echo "eval rc=$?"
fi
kill $HB
