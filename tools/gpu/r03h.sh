#!/bin/bash
# round 3 GPU check H: HBM traffic counters of the K8 ingest kernels (FETCH_SIZE, WRITE_SIZE in
# separate passes: they share the 4 TCC counter slots), one bench_k8 run per pass
R="${GRAFT_REPO_ROOT:-$(pwd)}"
O="$R/gpurun_out/r03i/k8c"
mkdir -p "$O"
export TMPDIR=/tmp
cd /tmp
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv --kernel-include-regex "rows_group|filter_" \
    -d "$O/k8_$c" -o run --pmc $c -- python3 "$R/bench/bench_k8.py" --iters 3 > "$O/k8_$c.log" 2>&1 || { echo "pmc $c rc=$?"; exit 1; }
  echo "== pmc $c ok"
done
timeout -k 10 120 python3 "$R/bench/bench_k8.py" > "$O/k8_timing.json" 2> "$O/k8_timing.err" || exit 1
cat "$O/k8_timing.json"
echo ALLDONE
