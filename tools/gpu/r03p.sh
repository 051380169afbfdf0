#!/bin/bash
# round 3 GPU check P: throughput engine with the direct fused step for single-pass rows
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r03p
mkdir -p $O
timeout -k 10 300 python -u -m pytest -v --timeout 150 --timeout-method thread tests/test_fit_throughput_gpu.py \
  tests/test_autoencoder_api_gpu.py > $O/t.out 2>&1; echo "tests rc=$?"
grep -E "FAIL|passed|failed" $O/t.out | tail -6
timeout -k 10 600 python bench.py --steps 20 --warmup 5 --infer-events 0 --e2e-events 0 --batch32-steps 0 \
  --lstm-steps 0 --stream-rows 0 --fit-rows 0 > $O/bench.out 2> $O/bench.err; echo "bench rc=$?"
python - <<'PY'
import json
for l in open("gpurun_out/r03p/bench.out"):
    if l.startswith("{"):
        d = json.loads(l)
        print(round(d["value"] / 1e9, 2), json.dumps(d["fresh_rows"]), json.dumps(d["fit_large_batch"])[:300])
PY
echo ALLDONE
