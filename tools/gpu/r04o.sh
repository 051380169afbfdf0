#!/bin/bash
# round 4 GPU check O: layer 4's padded output tile on the VALU in the small-batch trainers
# (tree _C.so, SML_MB_L4V=1) vs the MFMA tile (ab/_C_l4mfma.so): minibatch / fleet / fit /
# stream tests on the tree build, then a same-box A/B at batch 100 and 32, alternated
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=${O:-gpurun_out/r04o}
mkdir -p $O
PKG=hivemq-mqtt-tensorflow-kafka-realtime-iot-machine-learning-training-inference_amd
step() {
  local name=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$name.out 2> $O/$name.err
  local rc=$?
  echo "== $name rc=$rc"
  case $rc in 0) ;; *) tail -20 $O/$name.err; tail -30 $O/$name.out; exit $rc;; esac
}
cp $PKG/_C.so ab/_C_tree.so
step tests_mb 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_ae_minibatch_gpu.py tests/test_ae_fleet_gpu.py tests/test_fit_persistent_gpu.py tests/test_stream_doorbell_gpu.py tests/test_autoencoder_api_gpu.py tests/test_p2p_gpu.py
grep -E "passed|failed" $O/tests_mb.out | tail -1
for k in 1 2 3; do  # refined: x broadcast off the chain
  for v in tree l4only l4mfma; do
    cp ab/_C_$v.so $PKG/_C.so
    step mb100_${v}_$k 200 python bench/bench_minibatch.py --batch 100 --fleet ''
    step mb32_${v}_$k 200 python bench/bench_minibatch.py --batch 32 --fleet ''
  done
done
cp ab/_C_tree.so $PKG/_C.so
for f in $O/mb*.out; do echo "$f $(python -c "
import json; d=json.load(open('$f')); print(round(d['value']/1e6,3), {k: round(v) for k, v in d.get('phase_cycles_per_step', {}).items()})")"; done
echo ALLDONE
