#!/bin/bash
# round 3 GPU check C: LSTM forecaster fix, remaining GPU tests, request-ring probe, bench, pmc passes
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r03c
mkdir -p $O
step() {   # step <name> <timeout> <cmd...>: stop the whole script after a crash / timeout / abort
  local name=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$name.out 2> $O/$name.err
  local rc=$?
  echo "== $name rc=$rc"
  case $rc in 124|137|134|139) tail -20 $O/$name.err; exit $rc;; esac
  return 0
}
step t_lstm 300 python -u -m pytest -x -v --timeout 150 --timeout-method thread tests/test_lstm_serve_gpu.py
grep -q "failed" $O/t_lstm.out && step lstm_debug 120 python tools/serve_probe/lstm_serve_debug.py
step t_rest 400 python -u -m pytest -v --timeout 150 --timeout-method thread tests/test_serve_gpu.py \
  tests/test_no_vendor_fallback_gpu.py tests/test_autoencoder_api_gpu.py tests/test_fit_throughput_gpu.py
step probe 120 tools/serve_probe/vram_ring 5000
step bench 500 python bench.py --steps 20 --warmup 5
tail -3 $O/t_lstm.out $O/t_rest.out; cat $O/probe.out
step pmc 900 bash tools/gpu/r03c_pmc.sh
echo ALLDONE
