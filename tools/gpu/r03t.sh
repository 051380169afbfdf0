#!/bin/bash
# round 3 GPU check T: image-based batch-1 reference-LSTM trainer: tests, phase probe, bench field
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r03t
mkdir -p $O
step() {
  local name=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$name.out 2> $O/$name.err
  local rc=$?
  echo "== $name rc=$rc"
  case $rc in 124|137|134|139) tail -20 $O/$name.err; exit $rc;; esac
  return 0
}
step probe 60 tools/lref_probe/lref_probe 1000 5
cat $O/probe.out $O/probe.err
step t_lstmref 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_lstm_persistent_gpu.py
grep -E "PASS|FAIL|passed|failed|Error" $O/t_lstmref.out | tail -12
step lstmref 200 python -c "
import sys, json; sys.path.insert(0, 'bench')
import bench_lstm as b
print(json.dumps(b.measure_reference(batch=1, epochs=5, steps_per_epoch=1000, autograd_steps=100)))"
cat $O/lstmref.out
echo ALLDONE
