#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r03o
timeout -k 10 300 python -u tools/probe_fresh.py > gpurun_out/r03o/fresh.out 2> gpurun_out/r03o/fresh.err; echo "rc=$?"
cat gpurun_out/r03o/fresh.out
