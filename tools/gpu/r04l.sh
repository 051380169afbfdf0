#!/bin/bash
# round 4 GPU check L: persistent LSTM forward grid (occupancy-sized) vs one tile group per
# workgroup (SML_LSTM_FWD_PERSIST=0), same build, same box
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r04l
mkdir -p $O
step() {
  local name=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$name.out 2> $O/$name.err
  local rc=$?
  echo "== $name rc=$rc"
  case $rc in 0) ;; *) tail -30 $O/$name.err; tail -40 $O/$name.out; exit $rc;; esac
}
step tests 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_lstm_gpu.py tests/test_lstm_persistent_gpu.py tests/test_lstm_serve_gpu.py
grep -E "passed|failed" $O/tests.out | tail -1
for k in 1 2 3; do
  step pf_$k 200 python bench/bench_lstm.py --steps 20 --warmup 3
  step nopf_$k 200 env SML_LSTM_FWD_PERSIST=0 python bench/bench_lstm.py --steps 20 --warmup 3
done
for f in $O/*_[123].out; do echo "$f $(python -c "import json,sys; d=json.load(open('$f')); print(round(d['value']/1e6,2), round(d['ms_per_step'],3))")"; done
cd /tmp
timeout -k 10 150 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/$O/trace" -o run -- python3 "$GRAFT_REPO_ROOT/bench/bench_lstm.py" --steps 10 --warmup 2 > "$GRAFT_REPO_ROOT/$O/trace.log" 2>&1
echo "== trace rc=$?"
echo ALLDONE
