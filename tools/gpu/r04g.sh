#!/bin/bash
# round 4 GPU check G: LSTM bias modes on one build (SML_LSTM_BIASCOL = 1 bias columns,
# d db-column only, 0 plain) with the layer-1 pair loop, against the round-start kernels
# with their db-column switch (ab/_C_head.so, SML_LSTM_DBX=1); forward x prefetch 4 (default) vs
# SML_LSTM_FWD_PF=2, layer-2 register fragments vs SML_LSTM_DXRF=0; bf16 oracle tests in modes 1, d
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r04g
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
step tests_lstm 300 python -u -m pytest -x -v --timeout 150 --timeout-method thread -m gpu tests/test_lstm_gpu.py tests/test_lstm_serve_gpu.py
grep -E "passed|failed" $O/tests_lstm.out | tail -1
step tests_lstm_d 300 env SML_LSTM_BIASCOL=d SML_LSTM_FWD_PF=2 SML_LSTM_DXRF=0 python -u -m pytest -x -v --timeout 150 --timeout-method thread -m gpu tests/test_lstm_gpu.py
grep -E "passed|failed" $O/tests_lstm_d.out | tail -1
for k in 1 2 3; do
  cp ab/_C_tree.so $PKG/_C.so
  step lstm_bx_$k 200 python bench/bench_lstm.py --steps 20 --warmup 3
  step lstm_d_$k 200 env SML_LSTM_BIASCOL=d python bench/bench_lstm.py --steps 20 --warmup 3
  step lstm_dxrf0_$k 200 env SML_LSTM_DXRF=0 python bench/bench_lstm.py --steps 20 --warmup 3
  step lstm_bxpf2_$k 200 env SML_LSTM_FWD_PF=2 python bench/bench_lstm.py --steps 20 --warmup 3
  cp ab/_C_head.so $PKG/_C.so
  step lstm_headdbx_$k 200 env SML_LSTM_DBX=1 python bench/bench_lstm.py --steps 20 --warmup 3
done
cp ab/_C_tree.so $PKG/_C.so
for f in $O/lstm_*.out; do echo "$f $(python -c "import json,sys; d=json.load(open('$f')); print(round(d['value']/1e6,2), round(d['ms_per_step'],3))")"; done
cd /tmp
for m in 1 d; do
  SML_LSTM_BIASCOL=$m timeout -k 10 150 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/$O/trace_$m" -o run -- python3 "$GRAFT_REPO_ROOT/bench/bench_lstm.py" --steps 10 --warmup 2 > "$GRAFT_REPO_ROOT/$O/trace_$m.log" 2>&1
  echo "== trace_$m rc=$?"
done
cd "$GRAFT_REPO_ROOT"
step tests_mb 300 python -u -m pytest -x -v --timeout 150 --timeout-method thread -m gpu tests/test_ae_minibatch_gpu.py
grep -E "passed|failed" $O/tests_mb.out | tail -1
for k in 1 2; do
  step fit_tree_$k 200 python bench/bench_fit.py --rows 2000000 --skip-stream
  cp ab/_C_head.so $PKG/_C.so
  step fit_head_$k 200 python bench/bench_fit.py --rows 2000000 --skip-stream
  cp ab/_C_tree.so $PKG/_C.so
done
for f in $O/fit_*.out; do echo "$f $(python -c "import json; d=json.load(open('$f')); print({k: round(v['rows_per_s']/1e6, 2) for k, v in d.items()})")"; done
echo ALLDONE
