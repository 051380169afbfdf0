#!/bin/bash
# round 3 GPU check Y: reference-LSTM batch-1 trainer phase probe only
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r03y
mkdir -p $O
for b in tools/lref_probe/lref_probe*; do
  [ -x "$b" ] || continue
  timeout -k 5 30 $b 1000 5 > $O/$(basename $b).out 2>&1; rc=$?
  echo "== $b rc=$rc"; cat $O/$(basename $b).out
  [ $rc -eq 0 ] || exit $rc
done
echo ALLDONE
