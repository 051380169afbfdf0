#!/bin/bash
# round 3 GPU check K: scorer tests after restoring the pipelined poll, serve store A/B, full bench
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r03k
mkdir -p $O
step() {   # step <name> <timeout> <cmd...>: stop the whole script after a crash / timeout / abort
  local name=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$name.out 2> $O/$name.err
  local rc=$?
  echo "== $name rc=$rc"
  case $rc in 124|137|134|139) tail -20 $O/$name.err; exit $rc;; esac
  return 0
}
step t_serve 300 python -u -m pytest -v --timeout 150 --timeout-method thread tests/test_serve_gpu.py \
  tests/test_lstm_serve_gpu.py
grep -E "FAIL|passed|failed" $O/t_serve.out | tail -8
step ab_cached 200 python tools/serve_probe/serve_ab.py
SML_SERVE_STORES=nt step ab_nt 200 python tools/serve_probe/serve_ab.py
cat $O/ab_cached.out $O/ab_nt.out
step bench 600 python bench.py --steps 20 --warmup 5
python - <<'PY'
import json
for l in open("gpurun_out/r03k/bench.out"):
    if l.startswith("{"):
        d = json.loads(l)
        print({k: d.get(k) for k in ("value", "ms_per_step", "clock_settle", "p50_infer_us", "kafka_e2e_p50_us",
                                     "kafka_e2e_p99_us", "fit_large_batch_rows_per_s", "fresh_rows_per_s",
                                     "fit_batch100_rows_per_s", "stream_e2e_rows_per_s", "lstm_seq50_windows_per_s",
                                     "lstm_ref_us_per_step")})
        print(json.dumps(d["kafka_e2e"])[:800])
PY
echo ALLDONE
