#!/usr/bin/env bash
# headline A/B: residency rounds of the packed-pair grid (same box, alternating)
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"
O="$R/gpurun_out/r06c/rounds"
mkdir -p "$O"
for rep in 1 2; do
  for r in 1 2 3 6; do
    timeout -k 10 120 env SML_AE_ROUNDS=$r python "$R/bench.py" --headline-only --steps 50 --warmup 10 > "$O/r${r}_$rep.log" 2>&1 || { echo "FAILED r=$r"; exit 1; }
    python - "$O/r${r}_$rep.log" $r <<'PY'
import json, sys
l = [x for x in open(sys.argv[1]) if x.startswith('{')][-1]
d = json.loads(l)
print("rounds", sys.argv[2], round(d["value"] / 1e9, 3), "G rows/s", round(d["ms_per_step"], 4), "ms")
PY
  done
done
