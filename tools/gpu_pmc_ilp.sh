#!/usr/bin/env bash
# Counter passes for the headline AE train kernel, one-tile loop (SML_AE_ILP=1) vs the
# packed-pair loop (default, ILP 3): SQ issue mix and HBM read bytes, each pass its own
# rocprofv3 run with the kernel trace only.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"
O="$R/gpurun_out/pmc_ilp"
mkdir -p "$O"
export TMPDIR=/tmp
cd /tmp
BENCH="python3 $R/bench.py --steps 5 --warmup 2 --fleet-models 0 --batch32-steps 0 --dp-steps 0 --fit-rows 0 --stream-rows 0 --infer-events 0"
SQ="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CU_CYCLES"
for v in 1 3; do
  echo "== ilp$v sq"
  SML_AE_ILP=$v timeout -s KILL 150 rocprofv3 --kernel-trace --output-format csv --kernel-include-regex ae_train_kernel \
      -d "$O/ilp${v}_sq" -o run --pmc $SQ -- $BENCH > "$O/ilp${v}_sq.log" 2>&1 || exit 1
  echo "== ilp$v valu/lds"
  SML_AE_ILP=$v timeout -s KILL 150 rocprofv3 --kernel-trace --output-format csv --kernel-include-regex ae_train_kernel \
      -d "$O/ilp${v}_valu" -o run --pmc SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_WAIT_ANY GRBM_GUI_ACTIVE -- $BENCH \
      > "$O/ilp${v}_valu.log" 2>&1 || exit 1
  echo "== ilp$v fetch"
  SML_AE_ILP=$v timeout -s KILL 150 rocprofv3 --kernel-trace --output-format csv --kernel-include-regex ae_train_kernel \
      -d "$O/ilp${v}_fetch" -o run --pmc FETCH_SIZE GRBM_GUI_ACTIVE -- $BENCH > "$O/ilp${v}_fetch.log" 2>&1 || exit 1
done
echo "== done"
