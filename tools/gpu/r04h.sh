#!/bin/bash
# round 4 GPU check H: LSTM variants on one build, same box -- bias mode (d db-column, 1 bias
# columns, 0 plain) x forward x prefetch (2 / 4) x layer-1 backward loop (pair, C placement /
# SML_LSTM_PAIR=0 one-step), against the round-start kernels with SML_LSTM_DBX=1
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r04h
mkdir -p $O
PKG=hivemq-mqtt-tensorflow-kafka-realtime-iot-machine-learning-training-inference_amd
step() {
  local name=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$name.out 2> $O/$name.err
  local rc=$?
  echo "== $name rc=$rc"
  case $rc in 0) ;; *) tail -20 $O/$name.err; tail -30 $O/$name.out; exit $rc;; esac
}
cp $PKG/_C.so ab/_C_tree.so
step tests_lstm 300 env SML_LSTM_BIASCOL=d SML_LSTM_FWD_PF=2 python -u -m pytest -x -v --timeout 150 --timeout-method thread -m gpu tests/test_lstm_gpu.py tests/test_lstm_serve_gpu.py
grep -E "passed|failed" $O/tests_lstm.out | tail -1
B="python bench/bench_lstm.py --steps 20 --warmup 3"
for k in 1 2 3; do
  cp ab/_C_tree.so $PKG/_C.so
  step d2_$k 200 env SML_LSTM_BIASCOL=d SML_LSTM_FWD_PF=2 $B
  step d2np_$k 200 env SML_LSTM_BIASCOL=d SML_LSTM_FWD_PF=2 SML_LSTM_PAIR=0 $B
  step bx2_$k 200 env SML_LSTM_BIASCOL=1 SML_LSTM_FWD_PF=2 $B
  step p2_$k 200 env SML_LSTM_BIASCOL=0 SML_LSTM_FWD_PF=2 $B
  step d4_$k 200 env SML_LSTM_BIASCOL=d SML_LSTM_FWD_PF=4 $B
  cp ab/_C_head.so $PKG/_C.so
  step headdbx_$k 200 env SML_LSTM_DBX=1 $B
done
cp ab/_C_tree.so $PKG/_C.so
for f in $O/*_[123].out; do echo "$f $(python -c "import json,sys; d=json.load(open('$f')); print(round(d['value']/1e6,2), round(d['ms_per_step'],3))")"; done
cd /tmp
R=$GRAFT_REPO_ROOT
for v in "d2:SML_LSTM_BIASCOL=d SML_LSTM_FWD_PF=2" "d2np:SML_LSTM_BIASCOL=d SML_LSTM_FWD_PF=2 SML_LSTM_PAIR=0"; do
  n=${v%%:*}; e=${v#*:}
  env $e timeout -k 10 150 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$O/trace_$n" -o run -- python3 "$R/bench/bench_lstm.py" --steps 10 --warmup 2 > "$R/$O/trace_$n.log" 2>&1
  echo "== trace_$n rc=$?"
done
cp $R/ab/_C_head.so $R/$PKG/_C.so
SML_LSTM_DBX=1 timeout -k 10 150 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$O/trace_headdbx" -o run -- python3 "$R/bench/bench_lstm.py" --steps 10 --warmup 2 > "$R/$O/trace_headdbx.log" 2>&1
echo "== trace_headdbx rc=$?"
cp $R/ab/_C_tree.so $R/$PKG/_C.so
echo ALLDONE
