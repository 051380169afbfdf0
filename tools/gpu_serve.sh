#!/usr/bin/env bash
# Serving-path GPU check: persistent scorer tests + bench_infer (config 5).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
step() { local n=$1 t=$2; shift 2; echo "== $n"; timeout -k 10 "$t" "$@" > "gpurun_out/$n.log" 2>&1; local rc=$?;
         tail -n 3 "gpurun_out/$n.log"; [ $rc -eq 0 ] || { echo "FAILED $n rc=$rc"; exit $rc; }; }
step pytest_serve 300 python -u -m pytest tests/test_serve_gpu.py tests/test_serve_cli.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider
step bench_infer 300 python bench/bench_infer.py
echo "== done"
