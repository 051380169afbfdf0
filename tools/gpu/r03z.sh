#!/bin/bash
# round 3 GPU check U: batch-1 reference-LSTM trainer with Adam pipelined under the next chain
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r03z
mkdir -p $O
step() {
  local name=$1 t=$2; shift 2
  timeout -k 5 $t "$@" > $O/$name.out 2> $O/$name.err
  local rc=$?
  echo "== $name rc=$rc"
  case $rc in 0) ;; *) tail -20 $O/$name.err; cat $O/$name.out | tail -20; exit $rc;; esac
}
step probe1 20 tools/lref_probe/lref_probe 40 1
cat $O/probe1.out
step probe 30 tools/lref_probe/lref_probe 1000 5
cat $O/probe.out
step t_lstmref 120 python -u -m pytest -x -v --timeout 60 --timeout-method thread tests/test_lstm_persistent_gpu.py
grep -E "PASS|FAIL|passed|failed|Error" $O/t_lstmref.out | tail -12
step lstmref 120 python -c "
import sys, json; sys.path.insert(0, 'bench')
import bench_lstm as b
print(json.dumps(b.measure_reference(batch=1, epochs=5, steps_per_epoch=1000, autograd_steps=100)))"
cat $O/lstmref.out
echo ALLDONE
