#!/usr/bin/env bash
# round 6: swizzled LDS transposes -- AE + LSTM GPU tests, config-3 LSTM bench, counters, headline
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"
O="$R/gpurun_out/r06/swz"
mkdir -p "$O"
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread "$R/tests/test_ae_kernel_gpu.py" \
    "$R/tests/test_lstm_gpu.py" > "$O/pytest.txt" 2>&1 || { tail -30 "$O/pytest.txt"; exit 1; }
tail -1 "$O/pytest.txt"
for i in 1 2; do
  timeout -k 10 200 python "$R/bench/bench_lstm.py" --steps 30 --warmup 5 > "$O/lstm_$i.json" 2> "$O/lstm_$i.err" || exit 1
  tail -1 "$O/lstm_$i.json" | cut -c1-300
done
timeout -k 10 150 python "$R/bench.py" --headline-only --steps 20 --warmup 5 > "$O/head.json" 2> "$O/head.err" || exit 1
python -c "import json;d=json.loads(open('$O/head.json').read().strip().splitlines()[-1]);print('headline', round(d['value']/1e9,3), round(d['ms_per_step'],4))"
bash "$R/tools/gpu_r06_lstm_pmc.sh" > /dev/null
python3 "$R/tools/pmc_table.py" "$R/gpurun_out/r06/lstm_pmc/A" "$R/gpurun_out/r06/lstm_pmc/B" --min-grid 10000 > "$O/lstm_table.txt"
