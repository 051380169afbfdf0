#!/usr/bin/env bash
# unit-block split LSTM backward: tests, config-3 A/B, kernel stats
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"
O="$R/gpurun_out/r06c/split${TAG:-}"
mkdir -p "$O"
export TMPDIR=/tmp
step() { local n=$1 t=$2; shift 2; echo "== $n ($(date +%T))"; timeout -k 10 "$t" "$@" > "$O/$n.log" 2>&1; local rc=$?;
         tail -n 2 "$O/$n.log" | cut -c1-300; [ $rc -eq 0 ] || { echo "FAILED $n rc=$rc"; exit $rc; }; }
step pytest_split 300 python -u -m pytest "$R/tests/test_lstm_split_gpu.py" -x -q --timeout 120 --timeout-method thread
step pytest_lstm 400 python -u -m pytest "$R/tests/test_lstm_gpu.py" "$R/tests/test_lstm_serve_gpu.py" -x -q --timeout 120 --timeout-method thread
step lstm_split 200 python "$R/bench/bench_lstm.py" --steps 20 --warmup 5
step lstm_onewave 200 env SML_LSTM_SPLIT=0 python "$R/bench/bench_lstm.py" --steps 20 --warmup 5
step lstm_nopersist 200 env SML_LSTM_PERSIST=0 python "$R/bench/bench_lstm.py" --steps 20 --warmup 5
step lstm_half 200 python "$R/bench/bench_lstm.py" --steps 20 --warmup 5 --batch 32768
cd /tmp
step prof_lstm 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof_lstm" -o run \
    -- python3 "$R/bench/bench_lstm.py" --steps 10 --warmup 2
echo "== done"
