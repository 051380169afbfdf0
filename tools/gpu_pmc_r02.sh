#!/usr/bin/env bash
# Round-2 counter evidence (each pass its own rocprofv3 run, kernel trace only):
#   1. counter list of this box (rocprofv3 -L)
#   2. headline ae_train_kernel: SQ issue mix (VALU busy, wave cycles, waits) + GRBM
#   3. headline: FETCH_SIZE (+ GRBM), then TCC_EA0_RDREQ (+ 32B) -- bytes per step
#   4. LSTM bench: FETCH_SIZE of the fused kernels, in-place windows vs materialised
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"
O="$R/gpurun_out/pmc_r02"
mkdir -p "$O"
export TMPDIR=/tmp
cd /tmp
timeout -s KILL 60 rocprofv3 -L > "$O/counters_list.txt" 2>&1 || echo "counter list failed (continuing)"
have() { grep -qw "$1" "$O/counters_list.txt"; }
SQ=""
for c in SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_BUSY_CU_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES; do
  if have "$c" && [ "$(echo $SQ | wc -w)" -lt 8 ]; then SQ="$SQ $c"; fi
done
echo "SQ pass counters:$SQ"
BENCH="python3 $R/bench.py --steps 5 --warmup 2 --fleet-models 0 --batch32-steps 0 --dp-steps 0 --fit-rows 0 --stream-rows 0 --infer-events 100"
run() {  # run <name> <regex> <counters...> -- <cmd>
  local name=$1 rx=$2; shift 2
  local pmc=()
  while [ "$1" != "--" ]; do pmc+=("$1"); shift; done
  shift
  echo "== $name: ${pmc[*]}"
  timeout -s KILL 150 rocprofv3 --kernel-trace --output-format csv --kernel-include-regex "$rx" -d "$O/$name" -o run \
    --pmc "${pmc[@]}" -- "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "   rc=$rc"
  return $rc
}
run hl_sq ae_train_kernel $SQ GRBM_GUI_ACTIVE -- $BENCH || exit 1
run hl_fetch ae_train_kernel FETCH_SIZE GRBM_GUI_ACTIVE -- $BENCH || exit 1
if have TCC_EA0_RDREQ_32B; then
  run hl_rdreq ae_train_kernel TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum GRBM_GUI_ACTIVE -- $BENCH || exit 1
fi
run lstm_fetch_inplace lstm_fused FETCH_SIZE -- python3 "$R/bench/bench_lstm.py" --steps 3 --warmup 1 || exit 1
run lstm_fetch_mat lstm_fused FETCH_SIZE -- python3 "$R/bench/bench_lstm.py" --steps 3 --warmup 1 --materialize || exit 1
echo "== done"
