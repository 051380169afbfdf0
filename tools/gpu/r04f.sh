#!/bin/bash
# round 4 GPU check F: layer-1 LSTM backward with the pair loop + 16x16x32 pair weight
# gradients (tree _C.so) -- bf16 oracle tests, then a same-box A/B against the round-start
# kernels (ab/_C_head.so, HEAD before this round's LSTM work; SML_LSTM_DBX=1 its
# db-column variant), kernel trace, issue counters
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r04f
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
for k in 1 2 3; do
  for v in head tree; do
    cp ab/_C_$v.so $PKG/_C.so
    step lstm_${v}_$k 200 python bench/bench_lstm.py --steps 20 --warmup 3
  done
  cp ab/_C_head.so $PKG/_C.so
  step lstm_headdbx_$k 200 env SML_LSTM_DBX=1 python bench/bench_lstm.py --steps 20 --warmup 3
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
echo ALLDONE
