#!/usr/bin/env bash
# round 6: forecaster tests + seq-50 A/B, fresh-rows direct-step occupancy A/B, headline rounds A/B
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"
O="$R/gpurun_out/r06/serve"
mkdir -p "$O"
step() { local n=$1 t=$2; shift 2; echo "== $n"; timeout -k 10 "$t" "$@" > "$O/$n.log" 2>&1; local rc=$?;
         tail -n 4 "$O/$n.log"; [ $rc -eq 0 ] || { echo "FAILED $n rc=$rc"; exit $rc; }; }
step pytest_serve 400 python -u -m pytest "$R/tests/test_lstm_serve_gpu.py" -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider
step seq50_ab 240 python "$R/tools/serve_seq50_ab.py" 20000
step fresh_occ3 150 env SML_AE_DIRECT_OCC=3 python "$R/tools/probe_fresh.py"
step fresh_occ4 150 env SML_AE_DIRECT_OCC=4 python "$R/tools/probe_fresh.py"
[ -n "${ROUNDS:-}" ] || exit 0
SKIPTEST=1 VARIANTS="$ROUNDS" bash "$R/tools/gpu_r06_ab.sh"
