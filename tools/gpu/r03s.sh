#!/bin/bash
# round 3 GPU check S: phase split of the batch-1 reference-LSTM trainer (tools/lref_probe)
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r03s
mkdir -p $O
for b in tools/lref_probe/lref_probe*; do
  [ -x "$b" ] || continue
  timeout -k 10 60 $b 1000 5 > $O/$(basename $b).out 2>&1; rc=$?
  echo "== $b rc=$rc"; cat $O/$(basename $b).out
  case $rc in 0) ;; *) exit $rc;; esac
done
echo ALLDONE
