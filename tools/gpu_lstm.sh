#!/usr/bin/env bash
# LSTM-only GPU check: fused-LSTM numerics tests, bench_lstm, rocprofv3 kernel stats.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
step() { local n=$1 t=$2; shift 2; echo "== $n"; timeout -k 10 "$t" "$@" > "gpurun_out/$n.log" 2>&1; local rc=$?;
         tail -n 3 "gpurun_out/$n.log"; [ $rc -eq 0 ] || { echo "FAILED $n rc=$rc"; exit $rc; }; }
step pytest_lstm 300 python -u -m pytest tests/test_lstm_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider
step bench_lstm 300 python bench/bench_lstm.py
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/prof_lstm" -o run \
   -- python3 "$GRAFT_REPO_ROOT/bench/bench_lstm.py" --steps 10 --warmup 2 > "$GRAFT_REPO_ROOT/gpurun_out/rocprof_lstm.log" 2>&1 \
   || { echo "rocprof lstm failed"; exit 1; }
echo "== done"
