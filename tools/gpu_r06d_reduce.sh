#!/usr/bin/env bash
# one-launch wide reduction (slab_adam_kernel): bit-identity test, AE tests, headline A/B, kernel stats
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"
O="$R/gpurun_out/r06d/reduce${TAG:-}"
mkdir -p "$O"
export TMPDIR=/tmp
step() { local n=$1 t=$2; shift 2; echo "== $n ($(date +%T))"; timeout -k 10 "$t" "$@" > "$O/$n.log" 2>&1; local rc=$?;
         tail -n 1 "$O/$n.log" | cut -c1-220; [ $rc -eq 0 ] || { echo "FAILED $n rc=$rc"; tail -n 30 "$O/$n.log"; exit $rc; }; }
step pytest_reduce 300 python -u -m pytest "$R/tests/test_ae_fused_reduce_gpu.py" -x -v --timeout 120 --timeout-method thread
step pytest_ae 500 python -u -m pytest "$R/tests/test_ae_kernel_gpu.py" "$R/tests/test_ae_fleet_gpu.py" "$R/tests/test_ae_minibatch_gpu.py" "$R/tests/test_lstm_gpu.py" "$R/tests/test_rccl_gpu.py" -x -q --timeout 200 --timeout-method thread
for i in 1; do
  step head_two_$i 200 env SML_AE_FUSED_REDUCE=0 python "$R/bench.py" --headline-only --steps 100 --warmup 10
  step head_one_$i 200 python "$R/bench.py" --headline-only --steps 100 --warmup 10
done
cd /tmp
step prof 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof" -o run \
    -- python3 "$R/bench.py" --headline-only --steps 20 --warmup 5
echo "== done"
