#!/bin/bash
# round 4 final check: smoke, the whole GPU suite, the driver-contract bench (N=1, defaults)
# and a kernel trace of the headline step
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=${O:-gpurun_out/r04z4}
mkdir -p $O
step() {
  local name=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$name.out 2> $O/$name.err
  local rc=$?
  echo "== $name rc=$rc"
  case $rc in 0) ;; *) tail -30 $O/$name.err; tail -40 $O/$name.out; exit $rc;; esac
}
step smoke 180 python -c "import __graft_entry__ as g; g.smoke()"
cat $O/smoke.out
step tests_gpu 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider
grep -E "passed|failed" $O/tests_gpu.out | tail -1
step bench 400 python bench.py
O=$O python - <<'PY'
import json, os
d = json.load(open(os.environ["O"] + "/bench.out"))
keys = ["value", "ms_per_step", "vs_baseline", "keras_batch32", "fit_batch100_rows_per_s", "stream_e2e_rows_per_s",
        "stream_large_batch_rows_per_s", "lstm_seq50_windows_per_s", "lstm_ref_us_per_step", "p50_infer_us",
        "kafka_e2e_p50_us", "lstm_kafka_e2e_p50_us", "lstm_infer_p50_us", "mqtt_connections", "mqtt_dropped",
        "mqtt_publish_to_result_p50_us"]
print({k: (d.get(k)["rows_per_s"] if isinstance(d.get(k), dict) else d.get(k)) for k in keys})
print("phase_s", d.get("phase_s"), "budget", d.get("budget"))
PY
cd /tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/$O/trace" -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --headline-only --steps 20 --warmup 5 > "$GRAFT_REPO_ROOT/$O/trace.log" 2>&1
echo "== trace rc=$?"
cd "$GRAFT_REPO_ROOT"
step head_probe 120 python tools/lstm_probe/head_probe.py
cat $O/head_probe.out
echo ALLDONE
