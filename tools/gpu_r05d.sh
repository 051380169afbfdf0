#!/usr/bin/env bash
# stacked LSTM forward: bit-identity tests, the fused-step tests, then a same-box A/B of the seq-50 step
set -o pipefail
O=gpurun_out/r05d; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_lstm_gpu.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $O/tests.log 2>&1; rc=$?
tail -3 $O/tests.log
[ $rc -eq 0 ] || exit $rc
for v in 1 0 1 0 1 0; do
  SML_LSTM_FWD2=$v timeout -k 10 120 python bench/bench_lstm.py --steps 30 --warmup 5 > $O/ab_$v.json 2>/dev/null || exit 1
  echo "fwd2=$v $(python -c "import json;d=json.loads(open('$O/ab_$v.json').read().strip().splitlines()[-1]);print(round(d['value']/1e6,2), round(d['ms_per_step'],4))")"
done
