#!/usr/bin/env bash
# round 6: headline-kernel counters for the packed-pair occupancy variants (one pass per counter
# set, headline-only bench, --kernel-trace + --pmc only; never combined with the trace domains)
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R="${GRAFT_REPO_ROOT:-/root/repo}"
O="$R/gpurun_out/r06/pmc"
mkdir -p "$O"
A="SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS"
B="SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_MFMA GRBM_GUI_ACTIVE"
for v in ${VARIANTS:-3:0 4:1}; do
  o=${v%%:*}; x=${v##*:}
  for p in A B; do
    eval "C=\$$p"
    SML_AE_PAIR_OCC=$o SML_AE_PAIR_XP=$x timeout -s KILL 90 rocprofv3 --kernel-trace --output-format csv -d "$O/v${o}x${x}_$p" -o run --pmc $C \
        -- python3 "$R/bench.py" --headline-only --steps 5 --warmup 2 > "$O/v${o}x${x}_$p.log" 2>&1 \
        || { echo "pmc $v pass $p failed"; tail -20 "$O/v${o}x${x}_$p.log"; exit 1; }
  done
  python3 "$R/tools/pmc_table.py" "$O/v${o}x${x}_A" "$O/v${o}x${x}_B" --min-grid 100000 > "$O/v${o}x${x}_table.txt" || exit 1
done
grep -h -A2 ae_train_kernel "$O"/v*_table.txt
