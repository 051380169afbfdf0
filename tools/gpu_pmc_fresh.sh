#!/usr/bin/env bash
# Fresh-rows (direct step) counters, one rocprofv3 pass each, kernel trace only:
# both direct variants (SML_AE_DIRECT_PAIRS 0 / 1: one-tile vs packed-pair loop on raw rows)
# and the headline's packed-ring kernel run inside tools/ab/ab_fresh.py, told apart by kernel name.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"
O="$R/gpurun_out/pmc_fresh"
mkdir -p "$O"
export TMPDIR=/tmp AB_STEPS=3
cd /tmp
run() {  # run <name> <counters...>
  local name=$1; shift
  echo "== $name: $*"
  timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv --kernel-include-regex ae_train_kernel \
    -d "$O/$name" -o run --pmc "$@" -- python3 "$R/tools/ab/ab_fresh.py" > "$O/$name.log" 2>&1
  local rc=$?
  echo "   rc=$rc"
  return $rc
}
run sq SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES || exit 1
run fetch FETCH_SIZE GRBM_GUI_ACTIVE || exit 1
echo "== stats"
timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/stats" -o run -- \
  python3 "$R/tools/ab/ab_fresh.py" > "$O/stats.log" 2>&1 || exit 1
python3 "$R/tools/pmc_table.py" "$O/sq" "$O/fetch" --json > "$O/pmc_table.json" 2>&1
python3 "$R/tools/pmc_table.py" "$O/sq" "$O/fetch" > "$O/pmc_table.txt" 2>&1
cat "$O/pmc_table.txt"
echo "== done"
