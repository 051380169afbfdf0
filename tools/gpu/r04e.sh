#!/bin/bash
# round 4 GPU check E: fused LSTM kernels -- bf16 oracle tests, then a same-box A/B of
# {SLP-packed f32 VALU, -fno-slp-vectorize} x {bias columns (BX), SML_LSTM_BIASCOL=0}
# (the two builds are swapped in as _C.so from ab/), issue counters; then the Kafka
# scoring-leg probes and the large-batch decode curve
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r04e
mkdir -p $O
R=$GRAFT_REPO_ROOT
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
grep -E "passed|failed" $O/tests_lstm.out | tail -2
for k in 1 2; do
  for v in slp noslp; do
    cp ab/_C_$v.so $PKG/_C.so
    step lstm_${v}_bx_$k 200 python bench/bench_lstm.py --steps 20 --warmup 3
    step lstm_${v}_nobx_$k 200 env SML_LSTM_BIASCOL=0 python bench/bench_lstm.py --steps 20 --warmup 3
  done
done
cp ab/_C_tree.so $PKG/_C.so
for f in $O/lstm_*.out; do echo "$f $(python -c "import json,sys; d=json.load(open('$f')); print(round(d['value']/1e6,2), round(d['ms_per_step'],3))")"; done
cd /tmp
pass() {  # pass <name> <counters...>
  local name=$1; shift
  timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv --kernel-include-regex "lstm_fused" \
    -d "$R/$O/$name" -o run --pmc "$@" -- python3 "$R/bench/bench_lstm.py" --steps 3 --warmup 1 > "$R/$O/$name.log" 2>&1
  local rc=$?
  echo "== pmc $name rc=$rc"
  [ $rc -eq 0 ] || exit $rc
}
timeout -k 10 150 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$O/trace" -o run -- python3 "$R/bench/bench_lstm.py" --steps 10 --warmup 2 > "$R/$O/trace.log" 2>&1
echo "== trace rc=$?"
pass issue SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES
pass insts SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS
cd "$R"
step thread_probe 200 python tools/serve_probe/thread_probe.py
cat $O/thread_probe.out
step legs 300 python tools/serve_probe/kafka_legs.py
cat $O/legs.out
step large_batch 400 python bench/bench_fit.py --large-batch --rows 32000000
cat $O/large_batch.out
echo ALLDONE
