#!/bin/bash
# round 3 GPU check AH: reference-LSTM trainer with bank-spread backward images: tests, same-box
# A/B against the committed kernel, LDS counters
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r03ah
mkdir -p $O
step() {
  local name=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$name.out 2> $O/$name.err
  local rc=$?
  echo "== $name rc=$rc"
  case $rc in 0) ;; *) tail -20 $O/$name.err; tail -20 $O/$name.out; exit $rc;; esac
}
step t_lstmref 120 python -u -m pytest -x -v --timeout 60 --timeout-method thread tests/test_lstm_persistent_gpu.py
grep -E "passed|failed" $O/t_lstmref.out | tail -2
for r in 1 2; do
  step probe_new$r 30 tools/lref_probe/lref_probe 1000 5
  step probe_old$r 30 tools/lref_probe/lref_probe_old 1000 5
  cat $O/probe_new$r.out $O/probe_old$r.out
done
cd /tmp
timeout -s KILL 90 rocprofv3 --kernel-trace --output-format csv --kernel-include-regex lstm_ref -d "$GRAFT_REPO_ROOT/$O/pmc_insts" \
  -o run --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_BUSY_CYCLES SQ_WAVE_CYCLES \
  SQ_INSTS_VALU_TRANS_F32 SQ_ACTIVE_INST_LDS -- python3 "$GRAFT_REPO_ROOT/tools/pmc_small.py" lstmref > "$GRAFT_REPO_ROOT/$O/pmc.log" 2>&1
echo "== pmc rc=$?"
echo ALLDONE
