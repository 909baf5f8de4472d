#!/bin/bash
# Round 5 check: index / segment / bench-scale GPU tests, then the reads-while-ingesting runs.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
O=${1:-r5}
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread tests/test_gpu_index.py \
    tests/test_gpu_segments.py tests/test_gpu_bench_scale.py > gpurun_out/${O}_tests.log 2>&1 || exit $?
bash scripts/gpu_r5_reads.sh ${O}
