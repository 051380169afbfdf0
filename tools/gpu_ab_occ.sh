#!/usr/bin/env bash
# A/B of the AE train-kernel occupancy variants (SML_AE_OCC=3|4): numerics tests under
# both, kernel sweep, headline bench.  Every GPU step is time-limited; failures stop.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for occ in 4 3; do
  SML_AE_OCC=$occ timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
      tests/test_ae_kernel_gpu.py -p no:cacheprovider > gpurun_out/t_ae_occ$occ.log 2>&1 \
    || { echo "tests occ=$occ failed"; tail -30 gpurun_out/t_ae_occ$occ.log; exit 1; }
  tail -1 gpurun_out/t_ae_occ$occ.log
done
SML_AE_OCC=3 timeout -k 10 300 python tools/ae_sweep.py --batches 4194304,8388608 --blocks 768 --rounds 3 \
    > gpurun_out/sweep_occ3.log 2>&1 || exit 1
SML_AE_OCC=4 timeout -k 10 300 python tools/ae_sweep.py --batches 4194304,8388608 --blocks 1024,2048 --rounds 3 \
    > gpurun_out/sweep_occ4.log 2>&1 || exit 1
tail -2 gpurun_out/sweep_occ3.log; tail -4 gpurun_out/sweep_occ4.log
for occ in 3 4; do
  SML_AE_OCC=$occ timeout -k 10 300 python bench.py --infer-events 200 > gpurun_out/bench_occ$occ.log 2>&1 || exit 1
  tail -1 gpurun_out/bench_occ$occ.log | cut -c1-260
done
