#!/bin/bash
# round 3 GPU check G: poll_ready standalone test, scorer tests, small-batch accuracy A/B, serve store A/B
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r03g
mkdir -p $O
step() {   # step <name> <timeout> <cmd...>: stop the whole script after a crash / timeout / abort
  local name=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$name.out 2> $O/$name.err
  local rc=$?
  echo "== $name rc=$rc"
  case $rc in 124|137|134|139) tail -20 $O/$name.err; exit $rc;; esac
  return 0
}
step poll 60 tools/debug/poll_ready_test
cat $O/poll.out
step mb32 120 python tools/pmc_small.py mb32
SML_PMC_NOACC=1 step mb32_noacc 120 python tools/pmc_small.py mb32
step mb100 120 python tools/pmc_small.py mb100
SML_PMC_NOACC=1 step mb100_noacc 120 python tools/pmc_small.py mb100
cat $O/mb32.out $O/mb32_noacc.out $O/mb100.out $O/mb100_noacc.out | grep us/step
grep -q PASS $O/poll.out || { echo "poll_ready failed: skipping scorer runs"; echo ALLDONE; exit 0; }
step t_serve 300 python -u -m pytest -v --timeout 150 --timeout-method thread tests/test_serve_gpu.py \
  tests/test_lstm_serve_gpu.py
grep -E "FAIL|passed|failed" $O/t_serve.out | tail -8
step ab_cached 200 python tools/serve_probe/serve_ab.py
SML_SERVE_STORES=nt step ab_nt 200 python tools/serve_probe/serve_ab.py
cat $O/ab_cached.out $O/ab_nt.out
echo ALLDONE
