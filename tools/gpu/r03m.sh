#!/bin/bash
# round 3 GPU check M: the whole GPU test suite, then the full default bench
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r03m
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 150 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc"
grep -E "FAILED|ERROR|passed|failed" $O/pytest_gpu.log | tail -15
case $rc in 124|137|134|139) exit $rc;; esac
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > $O/bench.out 2> $O/bench.err
echo "bench rc=$?"
python - <<'PY'
import json
for l in open("gpurun_out/r03m/bench.out"):
    if l.startswith("{"):
        d = json.loads(l)
        print({k: d.get(k) for k in ("value", "ms_per_step", "clock_settle", "p50_infer_us", "kafka_e2e_p50_us",
                                     "fit_large_batch_rows_per_s", "fresh_rows_per_s", "fit_batch100_rows_per_s",
                                     "stream_e2e_rows_per_s", "lstm_seq50_windows_per_s", "lstm_ref_us_per_step")})
        print(json.dumps((d.get("kafka_e2e") or {}).get("legs_p50_us")))
PY
echo ALLDONE
