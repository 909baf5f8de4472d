#!/bin/bash
# Encoder correctness (GPU == CPU block tests) + microbench (k_seg_encode alone, 1M rows) with phase stamps.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu tests/test_gpu_segments.py > gpurun_out/seg_tests.log 2>&1 || { tail -30 gpurun_out/seg_tests.log; exit 1; }
timeout -k 10 240 python -u scripts/bench_seg_encode.py --n 1048576 --reps 20 --stamps > gpurun_out/seg_bench.json 2> gpurun_out/seg_bench.err || exit $?
timeout -k 10 240 python -u scripts/bench_seg_encode.py --n 1048576 --reps 20 --no-strings --stamps >> gpurun_out/seg_bench.json 2>> gpurun_out/seg_bench.err || exit $?
