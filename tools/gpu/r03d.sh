#!/bin/bash
# round 3 GPU check D: single-asm serve polls (AE + LSTM forecaster), streaming doorbell epoch,
# stream_e2e with the one-launch epoch
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r03d
mkdir -p $O
step() {   # step <name> <timeout> <cmd...>: stop the whole script after a crash / timeout / abort
  local name=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$name.out 2> $O/$name.err
  local rc=$?
  echo "== $name rc=$rc"
  case $rc in 124|137|134|139) tail -20 $O/$name.err; exit $rc;; esac
  return 0
}
step t_serve 300 python -u -m pytest -x -v --timeout 150 --timeout-method thread tests/test_lstm_serve_gpu.py \
  tests/test_serve_gpu.py
step t_stream 300 python -u -m pytest -v --timeout 150 --timeout-method thread tests/test_stream_doorbell_gpu.py \
  tests/test_fit_persistent_gpu.py
tail -4 $O/t_serve.out $O/t_stream.out
step bench_fit 400 python bench/bench_fit.py --rows 20000000 --partitions 16 --compare-chunks
tail -5 $O/bench_fit.out
echo ALLDONE
