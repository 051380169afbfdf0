#!/bin/bash
# round 4 GPU check C: large-batch streaming from Kafka (decode curve vs workers + trained
# rows/s), the scoring-leg thread probe, the Kafka legs probe
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r04c
mkdir -p $O
step() {
  local name=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$name.out 2> $O/$name.err
  local rc=$?
  echo "== $name rc=$rc"
  case $rc in 0) ;; *) tail -20 $O/$name.err; tail -30 $O/$name.out; exit $rc;; esac
}
echo "cpus=$(nproc) affinity=$(python -c 'import os; print(len(os.sched_getaffinity(0)))') numa=$(ls /sys/devices/system/node | grep -c node)"
step thread_probe 200 python tools/serve_probe/thread_probe.py
cat $O/thread_probe.out
step large_batch 400 python bench/bench_fit.py --large-batch --rows 32000000
cat $O/large_batch.out
step legs 300 python tools/serve_probe/kafka_legs.py
cat $O/legs.out
echo ALLDONE
