#!/usr/bin/env bash
# round 6: packed-pair variant tests + occupancy A/B of the headline step
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"
O="$R/gpurun_out/r06"
mkdir -p "$O"
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread "$R/tests/test_ae_kernel_gpu.py" \
    -k "pair_occupancy or tile_pair_loop or direct_pair" > "$O/pytest_pairs.txt" 2>&1 || { tail -30 "$O/pytest_pairs.txt"; exit 1; }
tail -3 "$O/pytest_pairs.txt"
for o in ${OCCS:-3 2 3 2}; do
  SML_AE_PAIR_OCC=$o timeout -k 10 150 python "$R/bench.py" --headline-only --steps 20 --warmup 5 \
      > "$O/ab_occ${o}.json" 2> "$O/ab_occ${o}.err" || exit 1
  echo "occ $o $(python -c "import json;d=json.loads(open('$O/ab_occ${o}.json').read().strip().splitlines()[-1]);print(round(d['value']/1e9,3), round(d['ms_per_step'],4))")"
done
