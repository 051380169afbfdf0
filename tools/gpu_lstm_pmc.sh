#!/usr/bin/env bash
# LSTM counter passes (each its own rocprofv3 run, kernel trace only): SQ issue/wait mix,
# then HBM fetch and write bytes.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
R="$GRAFT_REPO_ROOT"
cd /tmp
timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv -d "$R/gpurun_out/pmc_lstm_sq" -o run \
  --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS \
  -- python3 "$R/bench/bench_lstm.py" --steps 3 --warmup 1 > "$R/gpurun_out/pmc_lstm_sq.log" 2>&1 || { echo "sq pass failed"; exit 1; }
timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv -d "$R/gpurun_out/pmc_lstm_fetch" -o run \
  --pmc FETCH_SIZE \
  -- python3 "$R/bench/bench_lstm.py" --steps 3 --warmup 1 > "$R/gpurun_out/pmc_lstm_fetch.log" 2>&1 || { echo "fetch pass failed"; exit 1; }
timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv -d "$R/gpurun_out/pmc_lstm_write" -o run \
  --pmc WRITE_SIZE SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD \
  -- python3 "$R/bench/bench_lstm.py" --steps 3 --warmup 1 > "$R/gpurun_out/pmc_lstm_write.log" 2>&1 || { echo "write pass failed"; exit 1; }
echo "== done"
