#!/bin/bash
# Counter passes (each its own rocprofv3 run, kernel trace only, <= 8 SQ counters) on the
# the batch-1 reference-LSTM trainer after the one-wave chain / pipelined Adam rewrite
R="${GRAFT_REPO_ROOT:-$(pwd)}"
O="$R/gpurun_out/r03af"
mkdir -p "$O"
export TMPDIR=/tmp
cd /tmp
run() {  # run <mode> <regex> <name> <counters...>
  local mode=$1 rx=$2 name=$3; shift 3
  echo "== $mode $name: $*"
  timeout -s KILL 90 rocprofv3 --kernel-trace --output-format csv --kernel-include-regex "$rx" -d "$O/${mode}_$name" \
    -o run --pmc "$@" -- python3 "$R/tools/pmc_small.py" "$mode" > "$O/${mode}_$name.log" 2>&1
  local rc=$?
  echo "   rc=$rc"
  return $rc
}
for mode in lstmref; do
  rx=ae_minibatch; [ $mode = lstmref ] && rx=lstm_ref
  run $mode $rx issue SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU \
    SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA || exit 1
  run $mode $rx insts SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM SQ_INSTS_SMEM \
    SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT || exit 1
  run $mode $rx more SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_MISC SQ_INSTS_BRANCH SQ_VALU_MFMA_BUSY_CYCLES \
    SQ_INSTS_VALU_TRANS_F32 SQ_INST_LEVEL_LDS SQ_LDS_UNALIGNED_STALL SQ_WAVES || exit 1
done
echo "== done"
