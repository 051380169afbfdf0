#!/usr/bin/env bash
# LSTM seq-50 A/B on one box: alternates env settings, 3 runs each (bench/bench_lstm.py).
#   AB="SML_LSTM_FWD2_NT=1 SML_LSTM_FWD2_NT=2" bash tools/gpu_lstm_ab.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out/lstm_ab
OUT=gpurun_out/lstm_ab/ab.txt
: > "$OUT"
for r in 1 2 3; do
  for v in ${AB}; do
    line=$(env $v timeout -k 10 200 python bench/bench_lstm.py --steps 30 --warmup 5 2>/dev/null | grep '^{' | tail -1)
    rc=$?
    if [ $rc -ne 0 ]; then echo "$v failed rc=$rc"; exit 1; fi
    echo "$v $(echo "$line" | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("%.2f %.4f" % (d["value"] / 1e6, d["ms_per_step"]))')" | tee -a "$OUT"
  done
done
