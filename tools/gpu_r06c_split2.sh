#!/usr/bin/env bash
# split LSTM backward: tests at both workgroup shapes, config-3 A/B, kernel stats
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"
O="$R/gpurun_out/r06c/split2${TAG:-}"
mkdir -p "$O"
export TMPDIR=/tmp
step() { local n=$1 t=$2; shift 2; echo "== $n ($(date +%T))"; timeout -k 10 "$t" "$@" > "$O/$n.log" 2>&1; local rc=$?;
         tail -n 2 "$O/$n.log" | cut -c1-240; [ $rc -eq 0 ] || { echo "FAILED $n rc=$rc"; exit $rc; }; }
step pytest_split2 300 python -u -m pytest "$R/tests/test_lstm_split_gpu.py" -x -q --timeout 120 --timeout-method thread
step pytest_split1 300 env SML_LSTM_SPLIT_NTW=1 python -u -m pytest "$R/tests/test_lstm_split_gpu.py" -x -q --timeout 120 --timeout-method thread
step lstm_ntw2 200 python "$R/bench/bench_lstm.py" --steps 20 --warmup 5
step lstm_ntw1 200 env SML_LSTM_SPLIT_NTW=1 python "$R/bench/bench_lstm.py" --steps 20 --warmup 5
step lstm_onewave 200 env SML_LSTM_SPLIT=0 python "$R/bench/bench_lstm.py" --steps 20 --warmup 5
cd /tmp
step prof2 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof2" -o run \
    -- python3 "$R/bench/bench_lstm.py" --steps 10 --warmup 2
echo "== done"
