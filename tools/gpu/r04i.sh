#!/bin/bash
# round 4 GPU check I: LSTM backward on a persistent grid (one weight-gradient slab per CU
# workgroup) vs one tile group per workgroup (SML_LSTM_PERSIST=0), defaults = bias columns,
# x prefetch 2, pair loop; round-start kernels + SML_LSTM_DBX=1 as the fixed reference; the
# full LSTM GPU tests first
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r04i
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
step tests_lstm_np 300 env SML_LSTM_PERSIST=0 SML_LSTM_BIASCOL=d python -u -m pytest -x -q --timeout 150 --timeout-method thread -m gpu tests/test_lstm_gpu.py
grep -E "passed|failed" $O/tests_lstm_np.out | tail -1
B="python bench/bench_lstm.py --steps 20 --warmup 3"
for k in 1 2 3; do
  cp ab/_C_tree.so $PKG/_C.so
  step persist_$k 200 $B
  step nopersist_$k 200 env SML_LSTM_PERSIST=0 $B
  step dpersist_$k 200 env SML_LSTM_BIASCOL=d $B
  cp ab/_C_head.so $PKG/_C.so
  step headdbx_$k 200 env SML_LSTM_DBX=1 $B
done
cp ab/_C_tree.so $PKG/_C.so
for f in $O/*_[123].out; do echo "$f $(python -c "import json,sys; d=json.load(open('$f')); print(round(d['value']/1e6,2), round(d['ms_per_step'],3))")"; done
cd /tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 150 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$O/trace" -o run -- python3 "$R/bench/bench_lstm.py" --steps 10 --warmup 2 > "$R/$O/trace.log" 2>&1
echo "== trace rc=$?"
timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv --kernel-include-regex "lstm_fused" -d "$R/$O/issue" -o run --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES -- python3 "$R/bench/bench_lstm.py" --steps 3 --warmup 1 > "$R/$O/issue.log" 2>&1
echo "== pmc issue rc=$?"
timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv --kernel-include-regex "lstm_fused" -d "$R/$O/insts" -o run --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS -- python3 "$R/bench/bench_lstm.py" --steps 3 --warmup 1 > "$R/$O/insts.log" 2>&1
echo "== pmc insts rc=$?"
echo ALLDONE
