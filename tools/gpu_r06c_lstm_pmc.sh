#!/usr/bin/env bash
# round 6: counters of the config-3 LSTM step kernels (two passes, --kernel-trace + --pmc only)
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R="${GRAFT_REPO_ROOT:-/root/repo}"
O="$R/gpurun_out/r06c/lstm_pmc${TAG:-}"
mkdir -p "$O"
A="SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS"
B="SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE"
for p in A B; do
  eval "C=\$$p"
  timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv -d "$O/$p" -o run --pmc $C \
      -- python3 "$R/bench/bench_lstm.py" --steps 6 --warmup 2 > "$O/$p.log" 2>&1 \
      || { echo "lstm pmc pass $p failed"; tail -20 "$O/$p.log"; exit 1; }
done
python3 "$R/tools/pmc_table.py" "$O/A" "$O/B" --min-grid 100000 > "$O/table.txt" || exit 1
grep -A2 "lstm_" "$O/table.txt"
