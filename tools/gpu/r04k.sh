#!/bin/bash
# round 4 GPU check K: sigmoid gates pre-scaled by -log2(e) in the LSTM MFMA operands (tree)
# vs the build before (ab/_C_prev.so), same box; bf16-oracle tests; head probe
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r04k
mkdir -p $O
PKG=hivemq-mqtt-tensorflow-kafka-realtime-iot-machine-learning-training-inference_amd
step() {
  local name=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$name.out 2> $O/$name.err
  local rc=$?
  echo "== $name rc=$rc"
  case $rc in 0) ;; *) tail -30 $O/$name.err; tail -40 $O/$name.out; exit $rc;; esac
}
cp $PKG/_C.so ab/_C_tree.so
step tests 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_lstm_gpu.py tests/test_lstm_persistent_gpu.py tests/test_lstm_serve_gpu.py tests/test_loss_gpu.py tests/test_debug_modes_gpu.py
grep -E "passed|failed" $O/tests.out | tail -1
step head_probe 120 python tools/lstm_probe/head_probe.py
cat $O/head_probe.out
for k in 1 2 3; do
  cp ab/_C_tree.so $PKG/_C.so
  step tree_$k 200 python bench/bench_lstm.py --steps 20 --warmup 3
  cp ab/_C_prev.so $PKG/_C.so
  step prev_$k 200 python bench/bench_lstm.py --steps 20 --warmup 3
done
cp ab/_C_tree.so $PKG/_C.so
for f in $O/*_[123].out; do echo "$f $(python -c "import json,sys; d=json.load(open('$f')); print(round(d['value']/1e6,2), round(d['ms_per_step'],3))")"; done
cd /tmp
timeout -k 10 150 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/$O/trace" -o run -- python3 "$GRAFT_REPO_ROOT/bench/bench_lstm.py" --steps 10 --warmup 2 > "$GRAFT_REPO_ROOT/$O/trace.log" 2>&1
echo "== trace rc=$?"
echo ALLDONE
