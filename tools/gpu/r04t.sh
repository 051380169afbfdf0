#!/bin/bash
# round 4 GPU check T: issue counters of the small-batch trainers, VALU tail (tree) vs MFMA tail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=gpurun_out/r04t
mkdir -p $O
PKG=hivemq-mqtt-tensorflow-kafka-realtime-iot-machine-learning-training-inference_amd
cp $PKG/_C.so ab/_C_keep.so
cd /tmp
for v in tree mfma; do
  cp $R/ab/_C_$v.so $R/$PKG/_C.so
  for b in 100 32; do
    timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv --kernel-include-regex "ae_minibatch" \
      -d "$R/$O/${v}_$b" -o run --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES \
      -- python3 "$R/bench/bench_minibatch.py" --batch $b --fleet '' --launches 1 --steps-per-launch 5000 > "$R/$O/${v}_$b.log" 2>&1
    rc=$?
    echo "== pmc ${v}_$b rc=$rc"
    [ $rc -eq 0 ] || { cp $R/ab/_C_keep.so $R/$PKG/_C.so; exit $rc; }
  done
done
cp $R/ab/_C_keep.so $R/$PKG/_C.so
echo ALLDONE
