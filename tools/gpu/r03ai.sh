#!/bin/bash
# round 3 GPU check AI: small-batch AE trainer phase split at batch 32 and 100
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r03ai
mkdir -p $O
for b in 32 100; do
  timeout -k 10 120 python bench/bench_minibatch.py --batch $b --fleet "" > $O/mb$b.out 2> $O/mb$b.err; rc=$?
  echo "== mb$b rc=$rc"; [ $rc -eq 0 ] || { tail -5 $O/mb$b.err; exit $rc; }
  python -c "
import json; d=json.loads(open('$O/mb$b.out').read().strip().splitlines()[-1])
print({k: d.get(k) for k in ('persistent_us_per_step','phase_cycles_per_step','cycles_per_step','launch_us_per_step')})"
done
echo ALLDONE
