#!/usr/bin/env bash
# round 6 (session c) final evidence: GPU suite, full bench.py line, kernel stats of the headline and config 3
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"
O="$R/gpurun_out/r06c/final${TAG:-}"
mkdir -p "$O"
export TMPDIR=/tmp
step() { local n=$1 t=$2; shift 2; echo "== $n ($(date +%T))"; timeout -k 10 "$t" "$@" > "$O/$n.log" 2>&1; local rc=$?;
         tail -n 2 "$O/$n.log" | cut -c1-300; [ $rc -eq 0 ] || { echo "FAILED $n rc=$rc"; exit $rc; }; }
[ -n "${SKIPTESTS:-}" ] || step pytest 900 python -u -m pytest "$R/tests" -m gpu -q --timeout 320 --timeout-method thread
[ -n "${SKIPBENCH:-}" ] || step bench 600 python "$R/bench.py"
cd /tmp
step prof_head 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof_head" -o run \
    -- python3 "$R/bench.py" --headline-only --steps 20 --warmup 5
step prof_lstm 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof_lstm" -o run \
    -- python3 "$R/bench/bench_lstm.py" --steps 10 --warmup 2
echo "== done"
