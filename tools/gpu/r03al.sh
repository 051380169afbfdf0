#!/bin/bash
# round 3 GPU check AL: one-wave LSTM forecaster vs the general kernel (relu and tanh stacks)
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r03al
mkdir -p $O
timeout -k 10 200 python -u -m pytest -x -v --timeout 100 --timeout-method thread tests/test_lstm_serve_gpu.py > $O/t.out 2>&1
echo "== rc=$?"; grep -E "PASS|FAIL|Error|passed|failed" $O/t.out | tail -14
