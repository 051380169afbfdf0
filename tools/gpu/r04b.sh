#!/bin/bash
# round 4 GPU check B: config 3 (seq-50 LSTM) -- kernel trace of the step and counter passes
# on every LSTM kernel of it (each pass its own rocprofv3 run, kernel trace only)
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r04b
mkdir -p $O
R=$GRAFT_REPO_ROOT
step() {
  local name=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$name.out 2> $O/$name.err
  local rc=$?
  echo "== $name rc=$rc"
  case $rc in 0) ;; *) tail -20 $O/$name.err; tail -30 $O/$name.out; exit $rc;; esac
}
step lstm 200 python bench/bench_lstm.py --steps 20 --warmup 3
cat $O/lstm.out
cd /tmp
pass() {  # pass <name> <counters...>
  local name=$1; shift
  timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv --kernel-include-regex "lstm_fused|mse_acc|reduce_adam|slab_sum|rowgemm|wgrad" \
    -d "$R/$O/$name" -o run --pmc "$@" -- python3 "$R/bench/bench_lstm.py" --steps 3 --warmup 1 > "$R/$O/$name.log" 2>&1
  local rc=$?
  echo "== pmc $name rc=$rc"
  [ $rc -eq 0 ] || exit $rc
}
timeout -k 10 150 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$O/trace" -o run -- python3 "$R/bench/bench_lstm.py" --steps 10 --warmup 2 > "$R/$O/trace.log" 2>&1
echo "== trace rc=$?"
pass issue SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES
pass insts SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS
pass fetch FETCH_SIZE
pass write WRITE_SIZE
echo ALLDONE
