#!/usr/bin/env bash
# fused LSTM head: LSTM tests, config-3 bench A/B, kernel timeline
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"
O="$R/gpurun_out/r06c/head${TAG:-}"
mkdir -p "$O"
export TMPDIR=/tmp
step() { local n=$1 t=$2; shift 2; echo "== $n ($(date +%T))"; timeout -k 10 "$t" "$@" > "$O/$n.log" 2>&1; local rc=$?;
         tail -n 2 "$O/$n.log" | cut -c1-240; [ $rc -eq 0 ] || { echo "FAILED $n rc=$rc"; exit $rc; }; }
step pytest_lstm 400 python -u -m pytest "$R/tests/test_lstm_gpu.py" "$R/tests/test_lstm_split_gpu.py" -q --timeout 120 --timeout-method thread
step lstm_fused_head 200 python "$R/bench/bench_lstm.py" --steps 20 --warmup 5
step lstm_kernel_head 200 env SML_LSTM_SLAB2=0 python "$R/bench/bench_lstm.py" --steps 20 --warmup 5
step lstm_fused_head_b 200 python "$R/bench/bench_lstm.py" --steps 20 --warmup 5
cd /tmp
step prof 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof" -o run \
    -- python3 "$R/bench/bench_lstm.py" --steps 10 --warmup 2
echo "== done"
