#!/usr/bin/env bash
# Adam fused into the paired slab sum: LSTM + AE numerics, config-3 A/B, kernel stats
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"
O="$R/gpurun_out/r06d/slabadam${TAG:-}"
mkdir -p "$O"
export TMPDIR=/tmp
step() { local n=$1 t=$2; shift 2; echo "== $n ($(date +%T))"; timeout -k 10 "$t" "$@" > "$O/$n.log" 2>&1; local rc=$?;
         tail -n 1 "$O/$n.log" | cut -c1-200; [ $rc -eq 0 ] || { echo "FAILED $n rc=$rc"; tail -n 30 "$O/$n.log"; exit $rc; }; }
step pytest 500 python -u -m pytest "$R/tests/test_lstm_gpu.py" "$R/tests/test_lstm_split_gpu.py" "$R/tests/test_ae_fused_reduce_gpu.py" "$R/tests/test_ae_kernel_gpu.py" -x -q --timeout 200 --timeout-method thread
for i in 1 2; do
  step lstm_sep_$i 200 env SML_LSTM_SLAB2ADAM=0 python "$R/bench/bench_lstm.py" --steps 20 --warmup 5
  step lstm_fused_$i 200 python "$R/bench/bench_lstm.py" --steps 20 --warmup 5
done
step head 200 python "$R/bench.py" --headline-only --steps 100 --warmup 10
cd /tmp
step prof 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof" -o run \
    -- python3 "$R/bench/bench_lstm.py" --steps 10 --warmup 2
echo "== done"
