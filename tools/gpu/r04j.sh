#!/bin/bash
# round 4 GPU check J: the MSE accumulator fold (no same-address atomics) -- the GPU tests that
# run it, the head probe again, and the seq-50 LSTM bench
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r04j
mkdir -p $O
step() {
  local name=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$name.out 2> $O/$name.err
  local rc=$?
  echo "== $name rc=$rc"
  case $rc in 0) ;; *) tail -30 $O/$name.err; tail -40 $O/$name.out; exit $rc;; esac
}
step tests 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_loss_gpu.py tests/test_lstm_gpu.py tests/test_lstm_persistent_gpu.py tests/test_lstm_serve_gpu.py tests/test_no_vendor_fallback_gpu.py tests/test_rccl_gpu.py tests/test_debug_modes_gpu.py
grep -E "passed|failed" $O/tests.out | tail -1
step head_probe 120 python tools/lstm_probe/head_probe.py
cat $O/head_probe.out
for k in 1 2 3; do
  step lstm_$k 200 python bench/bench_lstm.py --steps 20 --warmup 3
done
for f in $O/lstm_[123].out; do echo "$f $(python -c "import json,sys; d=json.load(open('$f')); print(round(d['value']/1e6,2), round(d['ms_per_step'],3))")"; done
echo ALLDONE
