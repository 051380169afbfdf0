#!/usr/bin/env bash
# uniform-base addressing in the LSTM kernels: tests, config-3 bench, kernel stats, DP rehearsal
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"
O="$R/gpurun_out/r06c/addr${TAG:-}"
mkdir -p "$O"
export TMPDIR=/tmp
step() { local n=$1 t=$2; shift 2; echo "== $n ($(date +%T))"; timeout -k 10 "$t" "$@" > "$O/$n.log" 2>&1; local rc=$?;
         tail -n 2 "$O/$n.log" | cut -c1-240; [ $rc -eq 0 ] || { echo "FAILED $n rc=$rc"; exit $rc; }; }
step pytest_lstm 400 python -u -m pytest "$R/tests/test_lstm_gpu.py" "$R/tests/test_lstm_split_gpu.py" "$R/tests/test_lstm_serve_gpu.py" -x -q --timeout 120 --timeout-method thread
step lstm 200 python "$R/bench/bench_lstm.py" --steps 20 --warmup 5
step lstm_b 200 python "$R/bench/bench_lstm.py" --steps 20 --warmup 5
cd /tmp
step prof 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof" -o run \
    -- python3 "$R/bench/bench_lstm.py" --steps 10 --warmup 2
cd "$R"
step rehearsal4 330 python -u -m pytest "$R/tests/test_bench_dp_gpu.py" -x -q --timeout 320 --timeout-method thread -k "rehearsal and 4"
echo "== done"
