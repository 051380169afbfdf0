#!/usr/bin/env bash
# Full GPU check + profile snapshot: gpu tests, smoke, bench, rocprofv3 kernel stats,
# one SQ counter pass on the AE bench.  Each GPU step is time-limited; a failure stops.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
step() { local n=$1 t=$2; shift 2; echo "== $n"; timeout -k 10 "$t" "$@" > "gpurun_out/$n.log" 2>&1; local rc=$?;
         tail -n 3 "gpurun_out/$n.log"; [ $rc -eq 0 ] || { echo "FAILED $n rc=$rc"; exit $rc; }; }
step pytest_gpu 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step bench 600 python bench.py
cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/prof" -o run \
   -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 50 --warmup 5 --infer-events 100 > "$GRAFT_REPO_ROOT/gpurun_out/rocprof.log" 2>&1 \
   || { echo "rocprof failed"; tail -20 "$GRAFT_REPO_ROOT/gpurun_out/rocprof.log"; exit 1; }
timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/pmc" -o run \
   --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_ACTIVE_INST_VALU \
   -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 20 --warmup 2 --infer-events 0 > "$GRAFT_REPO_ROOT/gpurun_out/pmc.log" 2>&1 \
   || { echo "pmc failed"; tail -20 "$GRAFT_REPO_ROOT/gpurun_out/pmc.log"; exit 1; }
cd "$GRAFT_REPO_ROOT"
step bench_lstm 600 python bench/bench_lstm.py
step bench_infer 600 python bench/bench_infer.py
step bench_minibatch 300 python bench/bench_minibatch.py
cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/prof_lstm" -o run \
   -- python3 "$GRAFT_REPO_ROOT/bench/bench_lstm.py" --steps 10 --warmup 2 > "$GRAFT_REPO_ROOT/gpurun_out/rocprof_lstm.log" 2>&1 \
   || { echo "rocprof lstm failed"; exit 1; }
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/prof_mb" -o run \
   -- python3 "$GRAFT_REPO_ROOT/bench/bench_minibatch.py" --launches 2 > "$GRAFT_REPO_ROOT/gpurun_out/rocprof_mb.log" 2>&1 \
   || { echo "rocprof minibatch failed"; exit 1; }
echo "== done"
