#!/bin/bash
# round 3 GPU check AM: pipelined batch-32 persistent trainer -- numerics (oracle, fleet,
# bit-identity vs the two-barrier kernel), then a same-box A/B of SML_MB_PIPE=1 / 0
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r03am
mkdir -p $O
step() {
  local name=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$name.out 2> $O/$name.err
  local rc=$?
  echo "== $name rc=$rc"
  case $rc in 0) ;; *) tail -30 $O/$name.err; tail -30 $O/$name.out; exit $rc;; esac
}
step tests 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_ae_minibatch_gpu.py tests/test_ae_fleet_gpu.py tests/test_fit_persistent_gpu.py
grep -E "passed|failed" $O/tests.out | tail -2
for i in 1 2; do
  SML_MB_PIPE=1 step pipe$i 120 python bench/bench_minibatch.py --launches 5 --fleet 256,1024
  SML_MB_PIPE=0 step barrier$i 120 python bench/bench_minibatch.py --launches 5 --fleet 256,1024
done
python - <<'PY'
import json
for n in ("pipe1", "barrier1", "pipe2", "barrier2"):
    for l in open(f"gpurun_out/r03am/{n}.out"):
        if l.startswith("{"):
            d = json.loads(l)
            print(n, round(d["value"] / 1e6, 3), "M rows/s", {f["models"]: round(f["rows_per_s"] / 1e9, 3) for f in d.get("fleet", [])})
PY
echo ALLDONE
