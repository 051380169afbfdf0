#!/bin/bash
# round 3 GPU check A: ingest kernels, RCCL world-1 path, self-launch, bench short vs long
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r03a
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread \
  tests/test_ingest_kernels_gpu.py tests/test_preprocess_gpu.py tests/test_ae_kernel_gpu.py tests/test_ae_minibatch_gpu.py tests/test_p2p_gpu.py > $O/t_kernels.log 2>&1 || { tail -60 $O/t_kernels.log; exit 1; }
timeout -k 10 120 python bench/bench_k8.py > $O/k8.json 2> $O/k8.err || { tail $O/k8.err; exit 1; }
cat $O/k8.json
timeout -k 10 400 python -u -m pytest -x -v --timeout 240 --timeout-method thread \
  tests/test_rccl_gpu.py tests/test_bench_dp_gpu.py > $O/t_dp.log 2>&1 || { tail -60 $O/t_dp.log; exit 1; }
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/b_short.json 2> $O/b_short.err || { tail -30 $O/b_short.err; exit 1; }
Q="--infer-events 0 --e2e-events 0 --lstm-steps 0 --batch32-steps 0 --fit-rows 0 --stream-rows 0"
timeout -k 10 200 python bench.py --steps 200 --warmup 20 $Q > $O/b_long.json 2> $O/b_long.err || exit 1
timeout -k 10 200 python bench.py --steps 20 --warmup 5 $Q > $O/b_short2.json 2> $O/b_short2.err || exit 1
echo ALLDONE
