#!/usr/bin/env bash
# headline kernel: step time vs rows per step (fixed per-step overhead = 2 T(B/2) - T(B))
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"
O="$R/gpurun_out/r06c/scale_b"
mkdir -p "$O"
for rep in 1 2; do
  for b in 8388608 16777216 33554432 67108864; do
    timeout -k 10 150 python "$R/bench.py" --headline-only --steps 30 --warmup 5 --batch-per-gpu $b > "$O/b${b}_$rep.log" 2>&1 || { echo "FAILED b=$b"; exit 1; }
    python - "$O/b${b}_$rep.log" $b <<'PY'
import json, sys
l = [x for x in open(sys.argv[1]) if x.startswith('{')][-1]
d = json.loads(l)
print("rows", sys.argv[2], round(d["value"] / 1e9, 3), "G rows/s", round(d["ms_per_step"], 4), "ms")
PY
  done
done
