#!/bin/bash
# round 3 GPU check E: doorbell stall diagnosis, LSTM forecaster T=50 mismatch, request ring placement
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r03e
mkdir -p $O
step() {   # step <name> <timeout> <cmd...>: stop the whole script after a crash / timeout / abort
  local name=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$name.out 2> $O/$name.err
  local rc=$?
  echo "== $name rc=$rc"
  case $rc in 124|137|134|139) tail -20 $O/$name.err; exit $rc;; esac
  return 0
}
step doorbell 200 python -u tools/debug/doorbell_debug.py
cat $O/doorbell.out
step lstm 200 python -u -m pytest -x -v --timeout 150 --timeout-method thread "tests/test_lstm_serve_gpu.py::test_lstm_serve_matches_oracle"
grep -E "PASS|FAIL|^E " $O/lstm.out | head -30
step probe 120 tools/serve_probe/vram_ring 5000
cat $O/probe.out
echo ALLDONE
