#!/bin/bash
# round 3 GPU check F: doorbell epoch after the pinned-ring pool, serve store A/B, short-run vs long-run headline with / without a DPM clock settle,
# small-batch trainer timing + LDS bank-conflict counters after the swizzle
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r03f
mkdir -p $O
step() {   # step <name> <timeout> <cmd...>: stop the whole script after a crash / timeout / abort
  local name=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$name.out 2> $O/$name.err
  local rc=$?
  echo "== $name rc=$rc"
  case $rc in 124|137|134|139) tail -20 $O/$name.err; exit $rc;; esac
  return 0
}
step doorbell 200 python -u tools/debug/doorbell_debug.py
cat $O/doorbell.out
step t_stream 400 python -u -m pytest -v --timeout 150 --timeout-method thread tests/test_stream_doorbell_gpu.py \
  tests/test_lstm_serve_gpu.py tests/test_fit_persistent_gpu.py tests/test_autoencoder_api_gpu.py tests/test_debug_modes_gpu.py
grep -E "FAIL|passed|failed" $O/t_stream.out | tail -8
step bench_fit 400 python bench/bench_fit.py --rows 20000000 --partitions 16 --compare-chunks
tail -c 3000 $O/bench_fit.out
step ab_cached 200 python tools/serve_probe/serve_ab.py
SML_SERVE_STORES=nt step ab_nt 200 python tools/serve_probe/serve_ab.py
cat $O/ab_cached.out $O/ab_nt.out
step mb32 120 python tools/pmc_small.py mb32
step mb100 120 python tools/pmc_small.py mb100
cat $O/mb32.out $O/mb100.out
step s0a 200 python bench.py --headline-only --steps 20 --warmup 5
step s100 200 python bench.py --headline-only --steps 20 --warmup 5 --settle-ms 100
step s300 200 python bench.py --headline-only --steps 20 --warmup 5 --settle-ms 300
step long 200 python bench.py --headline-only --steps 200 --warmup 20
step s0b 200 python bench.py --headline-only --steps 20 --warmup 5
for f in s0a s100 s300 long s0b; do python -c "
import json,sys
for l in open('$O/$f.out'):
    if l.startswith('{'):
        d=json.loads(l); print('$f', d['steps'], d['warmup'], d['clock_settle'], round(d['value']/1e9,2), round(d['ms_per_step'],4))
"; done
cd /tmp
for mode in mb32 mb100; do
  timeout -s KILL 90 rocprofv3 --kernel-trace --output-format csv --kernel-include-regex ae_minibatch \
    -d "$GRAFT_REPO_ROOT/$O/${mode}_lds" -o run --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_INSTS_LDS \
    SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_VALU -- python3 "$GRAFT_REPO_ROOT/tools/pmc_small.py" $mode \
    > "$GRAFT_REPO_ROOT/$O/${mode}_lds.log" 2>&1 || exit 1
  echo "== pmc $mode ok"
done
echo ALLDONE
