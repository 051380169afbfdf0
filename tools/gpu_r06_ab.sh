#!/usr/bin/env bash
# round 6: pair-variant tests + headline A/B over env configurations (VARIANTS="occ:xp[:rounds] ...")
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"
O="$R/gpurun_out/r06"
mkdir -p "$O"
[ -n "${SKIPTEST:-}" ] || timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread "$R/tests/test_ae_kernel_gpu.py" \
    -k "${TESTK:-pair_occupancy or tile_pair_loop or direct_pair}" > "$O/pytest_pairs.txt" 2>&1 || { tail -30 "$O/pytest_pairs.txt"; exit 1; }
[ -n "${SKIPTEST:-}" ] || tail -1 "$O/pytest_pairs.txt"
for v in ${VARIANTS:-3:0 4:1 3:2}; do
  IFS=: read -r o x r <<< "$v"; r=${r:-3}; x=${x:-3}
  SML_AE_ROUNDS=$r SML_AE_PAIR_OCC=$o SML_AE_PAIR_XP=$x timeout -k 10 150 python "$R/bench.py" --headline-only --steps 20 --warmup 5 \
      > "$O/ab_${o}_${x}_${r}.json" 2> "$O/ab_${o}_${x}_${r}.err" || exit 1
  echo "occ $o xp $x rounds $r $(python -c "import json;d=json.loads(open('$O/ab_${o}_${x}_${r}.json').read().strip().splitlines()[-1]);print(round(d['value']/1e9,3), round(d['ms_per_step'],4), d.get('final_epoch_loss'))")"
done
