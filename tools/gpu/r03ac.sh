#!/bin/bash
# round 3 GPU check AC: LSTM forecaster (parallel key-state loads, unrolled head): tests + legs
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r03ac
mkdir -p $O
step() {
  local name=$1 t=$2; shift 2
  timeout -k 5 $t "$@" > $O/$name.out 2> $O/$name.err
  local rc=$?
  echo "== $name rc=$rc"
  case $rc in 0) ;; *) tail -20 $O/$name.err; tail -20 $O/$name.out; exit $rc;; esac
}
step t_serve 200 python -u -m pytest -x -v --timeout 100 --timeout-method thread tests/test_lstm_serve_gpu.py
grep -E "PASS|FAIL|passed|failed" $O/t_serve.out | tail -12
step legs 200 python tools/serve_probe/lstm_serve_legs.py
cat $O/legs.out
echo ALLDONE
