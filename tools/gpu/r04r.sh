#!/bin/bash
# round 4 GPU check R: config-3 step with the loss / accuracy / step-count work folded into the
# loss kernel's fold launch (default) vs SML_LSTM_FOLD=0, and replayed as captured HIP graphs
# (--graph 1); LSTM GPU tests first
cd "$GRAFT_REPO_ROOT" || exit 1
O=${O:-gpurun_out/r04r}
mkdir -p $O
step() {
  local name=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$name.out 2> $O/$name.err
  local rc=$?
  echo "== $name rc=$rc"
  case $rc in 0) ;; *) tail -20 $O/$name.err; tail -30 $O/$name.out; exit $rc;; esac
}
step tests_lstm 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_lstm_gpu.py tests/test_lstm_persistent_gpu.py tests/test_loss_gpu.py tests/test_resume.py
grep -E "passed|failed" $O/tests_lstm.out | tail -1
for k in 1 2 3; do
  step fold_$k 200 python bench/bench_lstm.py --steps 20 --warmup 3
  step nofold_$k 200 env SML_LSTM_FOLD=0 python bench/bench_lstm.py --steps 20 --warmup 3
  step graph_$k 200 python bench/bench_lstm.py --steps 20 --warmup 3 --graph 1
done
for f in $O/*_[123].out; do echo "$f $(python -c "import json,sys; d=json.load(open('$f')); print(round(d['value']/1e6,2), round(d['ms_per_step'],3), d['hip_graph'], d['final_loss'])")"; done
echo ALLDONE
