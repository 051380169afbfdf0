#!/bin/bash
# round 4 GPU check A: ADVICE fixes (serve D=32, LSTM reset, pack key, stream first-batch
# decision), LSTM Kafka low-latency path, the N-rank bench rehearsal (4 and 8 ranks on GPU 0),
# the default bench with per-phase timings, and the 100k-car MQTT fleet end to end
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r04a
mkdir -p $O
step() {
  local name=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$name.out 2> $O/$name.err
  local rc=$?
  echo "== $name rc=$rc"
  case $rc in 0) ;; *) tail -20 $O/$name.err; tail -30 $O/$name.out; exit $rc;; esac
}
echo "hws_max_conc_proc=$(cat /sys/module/amdgpu/parameters/hws_max_conc_proc 2>/dev/null) nofile=$(ulimit -n)/$(ulimit -Hn) nproc=$(nproc)"
step tests_fix 500 python -u -m pytest -x -v --timeout 150 --timeout-method thread -m gpu \
  tests/test_serve_gpu.py tests/test_lstm_serve_gpu.py tests/test_fit_throughput_gpu.py tests/test_stream_doorbell_gpu.py
grep -E "passed|failed" $O/tests_fix.out | tail -2
step mqtt 300 python bench/bench_mqtt.py --clients 100000 --messages 2
cat $O/mqtt.out
step bench 600 python bench.py --steps 20 --warmup 5
python - <<'PY'
import json
for l in open("gpurun_out/r04a/bench.out"):
    if l.startswith("{"):
        d = json.loads(l)
        print({k: d.get(k) for k in ("value", "ms_per_step", "p50_infer_us", "kafka_e2e_p50_us", "lstm_seq50_windows_per_s",
                                     "lstm_infer_p50_us", "lstm_kafka_e2e_p50_us", "mqtt_connections", "mqtt_dropped",
                                     "mqtt_publish_to_result_p50_us")})
        print(d["phase_s"], d["budget"])
PY
step tests_dp 700 python -u -m pytest -x -v --timeout 320 --timeout-method thread -m gpu tests/test_bench_dp_gpu.py
grep -E "passed|failed" $O/tests_dp.out | tail -2
echo ALLDONE
