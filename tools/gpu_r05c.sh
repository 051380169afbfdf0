set -o pipefail
mkdir -p gpurun_out/r05c
timeout -k 10 400 python -u -m pytest tests/test_ae_kernel_gpu.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/r05c/tests.log 2>&1; rc=$?
tail -3 gpurun_out/r05c/tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python tools/ab/ab_fresh.py > gpurun_out/r05c/ab_fresh.json 2> gpurun_out/r05c/ab_fresh.err
cat gpurun_out/r05c/ab_fresh.json
