#!/bin/bash
# packed dedup slots: GPU parity tests, bench + kernel profile, then bench variants that isolate the
# step's floor (no durable store, no bus)
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
T=${1:-pk}
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_dedup_window.py \
    tests/test_store_dedup.py tests/test_gpu_bench_scale.py tests/test_checkpoint.py > gpurun_out/${T}_tests.log 2>&1 || exit $?
bash scripts/gpu_bench_prof.sh $T || exit $?
timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-durable > gpurun_out/${T}_nodur.json 2> gpurun_out/${T}_nodur.err || exit $?
timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-durable --no-bus > gpurun_out/${T}_nobus.json 2> gpurun_out/${T}_nobus.err || exit $?
