#!/usr/bin/env bash
# One GPU-box session: gpu tests, smoke, bench, rocprofv3 kernel stats.
# Every GPU step has its own time limit; a fault / abort / timeout ends the script.
# Ordinary test failures (pytest exit 1) do not stop the later measurement steps.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
OUT=$ROOT/gpurun_out
mkdir -p "$OUT"
export TMPDIR=/tmp

fatal() {  # exit codes that mean the GPU step crashed / hung
  case "$1" in 124|134|137|139) return 0 ;; *) return 1 ;; esac
}

step() {  # step <name> <timeout> <cmd...>
  local name=$1 t=$2; shift 2
  echo "== $name ($(date +%T))"
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "   rc=$rc"; tail -n 5 "$OUT/$name.log"
  if fatal $rc; then echo "FATAL in $name (rc=$rc): stopping"; exit $rc; fi
  return $rc
}

STEPS=${STEPS:-"tests smoke bench prof"}
for s in $STEPS; do
  case $s in
    tests) step pytest_gpu 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread ;;
    testsel) step pytest_sel 600 python -u -m pytest ${TESTS:-tests} -m gpu -x -v -p no:cacheprovider --timeout 120 --timeout-method thread ;;
    fit) step bench_fit 600 python bench/bench_fit.py ${FIT_ARGS:-} ;;
    smoke) step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench) step bench 600 python bench.py ${BENCH_ARGS:-} ;;
    prof)
      (cd /tmp && step rocprof 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- \
          python3 "$ROOT/bench.py" --steps 50 --warmup 5 --infer-events 100 ${BENCH_ARGS:-}) ;;
    lstm) step bench_lstm 600 python bench/bench_lstm.py ${LSTM_ARGS:-} ;;
    infer) step bench_infer 600 python bench/bench_infer.py ${INFER_ARGS:-} ;;
    ingest) step bench_ingest 900 python bench/bench_ingest.py ${INGEST_ARGS:-} ;;
    proflstm)
      (cd /tmp && step rocprof_lstm 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_lstm" -o run -- \
          python3 "$ROOT/bench/bench_lstm.py" --steps 10 --warmup 2) ;;
    cli)
      step cli_ae_train 600 python -m streamml.cli cardata-v3 synthetic://50000 SENSOR_DATA_S_AVRO 0 model-predictions \
          train model1.h5 demo --workdir "$OUT/cli" --store "$OUT/cli/store" &&
      step cli_ae_predict 600 python -m streamml.cli cardata-v3 synthetic://50000 SENSOR_DATA_S_AVRO 0 \
          model-predictions predict model1.h5 demo --workdir "$OUT/cli" --store "$OUT/cli/store" &&
      step cli_lstm 600 python -m streamml.cli lstm-v1 synthetic://5000 SENSOR_DATA_S_AVRO 0 out --epochs 1 --take 300 &&
      step cli_mnist 600 python -m streamml.cli mnist --epochs 1 --steps-per-epoch 3000 --rows 20000 &&
      step cli_creditcard 600 python -m streamml.cli creditcard --evaluate --rows 100000 --epochs 3 ;;
    ilpab)   # headline-only A/B of the one-tile vs tile-pair train loop, alternated
      for r in 1 2; do
        for v in ${ILPS:-1 2}; do
          step "ilp${v}_run$r" 300 env SML_AE_ILP=$v python bench.py --infer-events 0 --fleet-models 0 --batch32-steps 0 \
              --fit-rows 0 --stream-rows 0 || true
        done
      done ;;
    rounds)   # pair-grid residency rounds A/B (headline only)
      for r in 1 2; do
        for v in ${ROUNDS:-1 2 3}; do
          step "rounds${v}_run$r" 300 env SML_AE_ROUNDS=$v python bench.py --max-blocks 8192 --infer-events 0 \
              --fleet-models 0 --batch32-steps 0 --fit-rows 0 --stream-rows 0 || true
        done
      done ;;
    sweep) step ae_sweep 600 python tools/ae_sweep.py ${SWEEP_ARGS:-} ;;
    counters) step counters 120 rocprofv3 -L ;;
    pmc)
      (cd /tmp && step pmc 600 rocprofv3 --kernel-trace --output-format csv -d "$OUT/pmc" -o run \
          --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU \
          SQ_INSTS_LDS SQ_INSTS_VMEM_RD -- python3 "$ROOT/bench.py" --steps 20 --warmup 2 --infer-events 0) ;;
    *) echo "unknown step $s" ;;
  esac
done
echo "== done"
