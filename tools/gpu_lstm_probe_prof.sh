#!/usr/bin/env bash
# Per-kernel time of the LSTM seq-50 step under env variants (rocprofv3 kernel stats, bench_lstm):
#   VARS="SML_LSTM_FWD2_PROBE=0 SML_LSTM_FWD2_PROBE=8" bash tools/gpu_lstm_probe_prof.sh
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd /tmp && export TMPDIR=/tmp
O="$R/gpurun_out/lstm_prof"
mkdir -p "$O"
for v in ${VARS}; do
  tag=$(echo "$v" | tr '=' '_')
  export $v
  timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/$tag" -o run -- \
      python3 "$R/bench/bench_lstm.py" --steps 10 --warmup 2 > "$O/$tag.log" 2>&1
  rc=$?
  unset "${v%%=*}"
  if [ $rc -ne 0 ]; then echo "$v rc=$rc"; exit $rc; fi
  f=$(find "$O/$tag" -name "*kernel_stats.csv" | head -1)
  python3 - "$f" "$v" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
out = []
for r in rows:
    n = r.get("Name", "")
    if "lstm" in n or "slab" in n or "adam" in n.lower():
        out.append("%s:%.1f" % (n.replace("void ", "").replace("(anonymous namespace)::", "").split("(")[0][:60], float(r["AverageNs"]) / 1e3))
print(sys.argv[2], " ".join(out))
PY
done
