#!/bin/bash
# round 3 GPU check I: one-event AE scorer diagnosis, small-batch accuracy placement A/B,
# persistent-fit oracle tests, K8 HBM counters
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r03i
mkdir -p $O
step() {   # step <name> <timeout> <cmd...>: stop the whole script after a crash / timeout / abort
  local name=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$name.out 2> $O/$name.err
  local rc=$?
  echo "== $name rc=$rc"
  case $rc in 124|137|134|139) tail -20 $O/$name.err; exit $rc;; esac
  return 0
}
step aedbg 120 python -u tools/debug/ae_serve_debug.py
cat $O/aedbg.out
step mb32 120 python tools/pmc_small.py mb32
SML_PMC_NOACC=1 step mb32_noacc 120 python tools/pmc_small.py mb32
step mb100 120 python tools/pmc_small.py mb100
SML_PMC_NOACC=1 step mb100_noacc 120 python tools/pmc_small.py mb100
cat $O/mb32.out $O/mb32_noacc.out $O/mb100.out $O/mb100_noacc.out | grep us/step
step t_fit 300 python -u -m pytest -v --timeout 150 --timeout-method thread tests/test_fit_persistent_gpu.py \
  tests/test_stream_doorbell_gpu.py tests/test_lstm_gpu.py
grep -E "FAIL|passed|failed" $O/t_fit.out | tail -8
step k8 400 bash tools/gpu/r03h.sh
tail -3 $O/k8.out
echo ALLDONE
