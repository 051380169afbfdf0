#!/bin/bash
# round 3 GPU check B: short-run gap trace, throughput fit, LSTM forecaster, housekeeping tests, bench
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r03b
mkdir -p $O
Q="--infer-events 0 --e2e-events 0 --lstm-steps 0 --batch32-steps 0 --fit-rows 0 --stream-rows 0 --fit-epochs 0 --fresh-steps 0"
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof_short -o run -- python3 bench.py --steps 20 --warmup 5 $Q > $O/short.json 2> $O/short.err || { tail -20 $O/short.err; exit 1; }
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof_long -o run -- python3 bench.py --steps 200 --warmup 20 $Q > $O/long.json 2> $O/long.err || { tail -20 $O/long.err; exit 1; }
timeout -k 10 400 python -u -m pytest -x -v --timeout 150 --timeout-method thread \
  tests/test_fit_throughput_gpu.py tests/test_lstm_serve_gpu.py tests/test_serve_gpu.py tests/test_no_vendor_fallback_gpu.py \
  tests/test_autoencoder_api_gpu.py > $O/t.log 2>&1 || { tail -60 $O/t.log; exit 1; }
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
echo ALLDONE
