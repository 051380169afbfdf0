#!/bin/bash
# round 3 GPU check AJ: throughput fit with deferred epoch metrics and the clock settle:
# fit tests, then headline + fit_large_batch twice on one box
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r03aj
mkdir -p $O
step() {
  local name=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$name.out 2> $O/$name.err
  local rc=$?
  echo "== $name rc=$rc"
  case $rc in 0) ;; *) tail -20 $O/$name.err; tail -20 $O/$name.out; exit $rc;; esac
}
step t_fit 300 python -u -m pytest -x -v --timeout 150 --timeout-method thread tests/test_fit_throughput_gpu.py \
  tests/test_autoencoder_api_gpu.py tests/test_fit_persistent_gpu.py
grep -E "passed|failed" $O/t_fit.out | tail -2
for r in 1 2; do
  step bench$r 300 python bench.py --steps 20 --warmup 5 --infer-events 0 --e2e-events 0 --batch32-steps 0 \
    --lstm-steps 0 --stream-rows 0 --fit-rows 0 --fresh-steps 0
  python -c "
import json
for l in open('$O/bench$r.out'):
    if l.startswith('{'):
        d=json.loads(l); f=d['fit_large_batch']
        print(round(d['value']/1e9,2), round(d['fit_large_batch_rows_per_s']/1e9,2), round(f['shuffled']['rows_per_s']/1e9,2), round(d['fit_large_batch_rows_per_s']/d['value'],3))"
done
echo ALLDONE
