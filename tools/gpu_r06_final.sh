#!/usr/bin/env bash
# round 6 final evidence: full bench.py line, kernel stats of the headline step and of config 3
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"
O="$R/gpurun_out/r06/final"
mkdir -p "$O"
export TMPDIR=/tmp
step() { local n=$1 t=$2; shift 2; echo "== $n ($(date +%T))"; timeout -k 10 "$t" "$@" > "$O/$n.log" 2>&1; local rc=$?;
         tail -n 2 "$O/$n.log" | cut -c1-400; [ $rc -eq 0 ] || { echo "FAILED $n rc=$rc"; exit $rc; }; }
[ -n "${SKIPBENCH:-}" ] || step bench 500 python "$R/bench.py"
cd /tmp
step prof_head 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof_head" -o run \
    -- python3 "$R/bench.py" --headline-only --steps 20 --warmup 5
step prof_lstm 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof_lstm" -o run \
    -- python3 "$R/bench/bench_lstm.py" --steps 10 --warmup 2
echo "== done"
