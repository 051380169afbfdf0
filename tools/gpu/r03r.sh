#!/bin/bash
# round 3 GPU check R: batch-1 reference-LSTM trainer (one-wave chain) tests + timing,
# then the full GPU suite, smoke and the default-contract bench at HEAD
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r03r
mkdir -p $O
step() {   # step <name> <timeout> <cmd...>: stop the whole script after a crash / timeout / abort
  local name=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$name.out 2> $O/$name.err
  local rc=$?
  echo "== $name rc=$rc"
  case $rc in 124|137|134|139) tail -20 $O/$name.err; exit $rc;; esac
  return 0
}
step t_lstmref 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_lstm_persistent_gpu.py
grep -E "PASS|FAIL|passed|failed|Error" $O/t_lstmref.out | tail -12
step lstmref 200 python -c "
import sys, json; sys.path.insert(0, 'bench')
import bench_lstm as b
print(json.dumps(b.measure_reference(batch=1, epochs=5, steps_per_epoch=1000, autograd_steps=100)))"
cat $O/lstmref.out
step tests 900 python -u -m pytest -x -v --timeout 150 --timeout-method thread -m gpu tests
grep -E "FAIL|passed|failed|skipped" $O/tests.out | tail -8
step smoke 120 python __graft_entry__.py
cat $O/smoke.out
step bench 600 python bench.py --steps 20 --warmup 5
python - <<'PY'
import json
for l in open("gpurun_out/r03r/bench.out"):
    if l.startswith("{"):
        d = json.loads(l)
        print({k: d.get(k) for k in ("value", "ms_per_step", "clock_settle", "p50_infer_us", "kafka_e2e_p50_us",
                                     "kafka_e2e_p99_us", "fit_large_batch_rows_per_s", "fresh_rows_per_s",
                                     "fit_batch100_rows_per_s", "stream_e2e_rows_per_s", "lstm_seq50_windows_per_s",
                                     "lstm_ref_us_per_step")})
PY
echo ALLDONE
