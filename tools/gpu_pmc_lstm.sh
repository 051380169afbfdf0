#!/usr/bin/env bash
# Counter passes on the fused LSTM kernels of bench/bench_lstm.py (each pass its own
# rocprofv3 run, kernel trace only, <= 8 SQ counters per pass).
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"
O="$R/gpurun_out/pmc_lstm"
mkdir -p "$O"
export TMPDIR=/tmp
cd /tmp
run() {  # run <name> <counters...>
  local name=$1; shift
  echo "== $name: $*"
  timeout -s KILL 150 rocprofv3 --kernel-trace --output-format csv --kernel-include-regex lstm_fused -d "$O/$name" -o run \
    --pmc "$@" -- python3 "$R/bench/bench_lstm.py" --steps 3 --warmup 1 > "$O/$name.log" 2>&1
  local rc=$?
  echo "   rc=$rc"
  return $rc
}
run issue SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS \
  SQ_ACTIVE_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES || exit 1
run insts SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT \
  SQ_ACTIVE_INST_VMEM SQ_WAVES || exit 1
echo "== done"
