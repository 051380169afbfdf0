#!/bin/bash
# round 3 GPU check J: one-event AE scorer trace
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r03j
mkdir -p $O
timeout -k 10 120 python -u tools/debug/ae_serve_debug.py > $O/aedbg.out 2> $O/aedbg.err
echo "rc=$?"
cat $O/aedbg.out
