#!/bin/bash
# Round-4 GPU check 2: encoder + dedup-filter parity (GPU vs host engines), bench-scale parity, then
# the bench and a kernel-stats profile.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 480 --timeout-method thread -m gpu \
    tests/test_gpu_segments.py tests/test_dedup_window.py tests/test_gpu_bench_scale.py tests/test_gpu_engine.py \
    > gpurun_out/r4c_gpu_tests.log 2>&1 || { tail -30 gpurun_out/r4c_gpu_tests.log; exit 1; }
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r4c_bench.json 2> gpurun_out/r4c_bench.err || exit $?
R=$PWD
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/r4c_prof" -o run -- \
    python -u "$R/bench.py" --steps 20 --warmup 5 > "$R/gpurun_out/r4c_prof_bench.json" 2> "$R/gpurun_out/r4c_prof.err"
