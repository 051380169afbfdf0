#!/usr/bin/env bash
# restored-container sanity: GPU suite, LSTM config-3 bench + kernel stats, headline-only bench
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"
O="$R/gpurun_out/r06c/sanity"
mkdir -p "$O"
export TMPDIR=/tmp
step() { local n=$1 t=$2; shift 2; echo "== $n ($(date +%T))"; timeout -k 10 "$t" "$@" > "$O/$n.log" 2>&1; local rc=$?;
         tail -n 2 "$O/$n.log" | cut -c1-400; [ $rc -eq 0 ] || { echo "FAILED $n rc=$rc"; exit $rc; }; }
step pytest 600 python -u -m pytest "$R/tests" -m gpu -x -q --timeout 120 --timeout-method thread
step lstm 200 python "$R/bench/bench_lstm.py" --steps 20 --warmup 5
cd /tmp
step prof_lstm 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof_lstm" -o run \
    -- python3 "$R/bench/bench_lstm.py" --steps 10 --warmup 2
step head 300 python "$R/bench.py" --headline-only --steps 20 --warmup 5
echo "== done"
