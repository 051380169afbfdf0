#!/bin/bash
# round 3 GPU check AU (end of session 3: full suite, smoke, bench): full GPU suite, smoke, default-contract bench, and a
# kernel-trace --stats profile of the default bench
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r03au
mkdir -p $O
step() {
  local name=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$name.out 2> $O/$name.err
  local rc=$?
  echo "== $name rc=$rc"
  case $rc in 0) ;; *) tail -20 $O/$name.err; tail -20 $O/$name.out; exit $rc;; esac
}
step tests 900 python -u -m pytest -x -v --timeout 150 --timeout-method thread -m gpu tests
grep -E "FAIL|passed|failed|skipped" $O/tests.out | tail -3
step smoke 120 python __graft_entry__.py
cat $O/smoke.out
step bench 600 python bench.py --steps 20 --warmup 5
python - <<'PY'
import json
for l in open("gpurun_out/r03au/bench.out"):
    if l.startswith("{"):
        d = json.loads(l)
        print({k: d.get(k) for k in ("value", "ms_per_step", "p50_infer_us", "p99_infer_us", "kafka_e2e_p50_us",
                                     "fit_large_batch_rows_per_s", "fresh_rows_per_s", "fit_batch100_rows_per_s",
                                     "stream_e2e_rows_per_s", "lstm_seq50_windows_per_s", "lstm_ref_us_per_step",
                                     "lstm_infer_p50_us", "lstm_infer_p99_us")})
PY
echo ALLDONE
