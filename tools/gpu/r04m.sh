#!/bin/bash
# round 4 GPU check M: one-pass slab reduction (default) vs the multi-level one (SML_SLAB_1P=0)
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r04m
mkdir -p $O
step() {
  local name=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$name.out 2> $O/$name.err
  local rc=$?
  echo "== $name rc=$rc"
  case $rc in 0) ;; *) tail -30 $O/$name.err; tail -40 $O/$name.out; exit $rc;; esac
}
step tests 500 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_dense_gpu.py tests/test_lstm_gpu.py tests/test_lstm_persistent_gpu.py tests/test_ae_kernel_gpu.py tests/test_fit_throughput_gpu.py tests/test_mnist_gpu.py tests/test_debug_modes_gpu.py tests/test_no_vendor_fallback_gpu.py
grep -E "passed|failed" $O/tests.out | tail -1
for k in 1 2 3; do
  step one_$k 200 python bench/bench_lstm.py --steps 20 --warmup 3
  step multi_$k 200 env SML_SLAB_1P=0 python bench/bench_lstm.py --steps 20 --warmup 3
done
for f in $O/*_[123].out; do echo "$f $(python -c "import json,sys; d=json.load(open('$f')); print(round(d['value']/1e6,2), round(d['ms_per_step'],3))")"; done
step headline_one 300 python bench.py --headline-only
step headline_multi 300 env SML_SLAB_1P=0 python bench.py --headline-only
for f in $O/headline_*.out; do echo "$f $(python -c "import json,sys; d=json.load(open('$f')); print(round(d['value']/1e9,3), round(d['ms_per_step'],4))")"; done
echo ALLDONE
