#!/usr/bin/env bash
# full bench.py line, then config 3 standalone on the same box (full-bench vs standalone LSTM A/B)
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"
O="$R/gpurun_out/r06c/bench2${TAG:-}"
mkdir -p "$O"
export TMPDIR=/tmp
step() { local n=$1 t=$2; shift 2; echo "== $n ($(date +%T))"; timeout -k 10 "$t" "$@" > "$O/$n.log" 2>&1; local rc=$?;
         tail -n 1 "$O/$n.log" | cut -c1-200; [ $rc -eq 0 ] || { echo "FAILED $n rc=$rc"; exit $rc; }; }
step lstm_before 200 python "$R/bench/bench_lstm.py" --steps 20 --warmup 5
step bench 600 python "$R/bench.py"
step lstm_after 200 python "$R/bench/bench_lstm.py" --steps 20 --warmup 5
echo "== done"
