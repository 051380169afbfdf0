#!/usr/bin/env bash
# Round check on one GPU box: full GPU test suite, smoke(), default bench, counter passes.
# Each GPU step has its own time limit; a crash / hang code stops the script.
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R"
O="$R/gpurun_out/round"
mkdir -p "$O"
export TMPDIR=/tmp
fatal() { case "$1" in 124|134|137|139) return 0 ;; *) return 1 ;; esac; }
step() {
  local name=$1 t=$2; shift 2
  echo "== $name ($(date +%T))"
  timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "   rc=$rc"; tail -n 3 "$O/$name.log"
  if fatal $rc; then echo "FATAL in $name"; exit $rc; fi
  return 0
}
STEPS=${STEPS:-"tests smoke bench pmc"}
for s in $STEPS; do
  case $s in
    tests) step pytest_gpu ${TESTS_TIMEOUT:-600} python -u -m pytest ${TESTS:-tests -m gpu} -x -q -p no:cacheprovider --timeout ${TEST_TIMEOUT:-120} --timeout-method thread ;;
    smoke) step smoke 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" ;;
    bench) step bench 400 python bench.py ${BENCH_ARGS:-} ;;
    pmc) step pmc 300 bash tools/gpu_pmc_r02.sh ;;
  esac
done
echo "== done"
