#!/bin/bash
# round 3 GPU check AT: one 16-byte poll of all four update counters per step -- numerics, A/B
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r03at
mkdir -p $O
step() {
  local name=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$name.out 2> $O/$name.err
  local rc=$?
  echo "== $name rc=$rc"
  case $rc in 0) ;; *) tail -30 $O/$name.err; tail -30 $O/$name.out; exit $rc;; esac
}
step tests 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_ae_minibatch_gpu.py tests/test_ae_fleet_gpu.py tests/test_stream_doorbell_gpu.py
grep -E "passed|failed" $O/tests.out | tail -1
for i in 1 2; do
  SML_MB_PIPE=1 step pipe_b32_$i 120 python bench/bench_minibatch.py --batch 32 --launches 5 --fleet 1024
  SML_MB_PIPE=0 step barrier_b32_$i 120 python bench/bench_minibatch.py --batch 32 --launches 5 --fleet 1024
done
python - <<'PY'
import json, glob, os
for n in sorted(glob.glob("gpurun_out/r03at/*_b32_*.out")):
    for l in open(n):
        if l.startswith("{"):
            d = json.loads(l)
            print(os.path.basename(n)[:-4], round(d["value"] / 1e6, 3), "M rows/s", {f["models"]: round(f["rows_per_s"] / 1e9, 3) for f in d.get("fleet", [])})
PY
echo ALLDONE
