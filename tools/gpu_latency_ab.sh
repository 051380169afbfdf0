set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
timeout -k 10 200 python bench/bench_infer.py > gpurun_out/lat_infer1.log 2>&1 || exit 1
timeout -k 10 200 python bench.py --steps 20 --warmup 5 --infer-events 2000 --fleet-models 0 --batch32-steps 0 --fit-rows 0 --stream-rows 0 > gpurun_out/lat_bench1.log 2>&1 || exit 1
timeout -k 10 200 python bench.py --steps 1 --warmup 0 --dataset-rows 1048576 --batch-per-gpu 1048576 --infer-events 2000 --fleet-models 0 --batch32-steps 0 --fit-rows 0 --stream-rows 0 > gpurun_out/lat_bench2.log 2>&1 || exit 1
timeout -k 10 200 python bench/bench_infer.py > gpurun_out/lat_infer2.log 2>&1 || exit 1
for f in lat_infer1 lat_bench1 lat_bench2 lat_infer2; do echo $f $(grep -o '"value": [0-9.]*\|"p50_infer_us": [0-9.]*\|persistent_device_p50_us": [0-9.]*' gpurun_out/$f.log | tr '\n' ' '); done
